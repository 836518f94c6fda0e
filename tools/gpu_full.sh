#!/bin/bash
# Full GPU round: parity tests, bench line, kernel-trace profile, then PMC traffic passes.
# Usage (through gpurun): bash tools/gpu_full.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r}
bash tools/gpu_round.sh "$@" || exit $?
bash tools/pmc_round.sh "${TAG}_pmc" || exit $?
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc k_match gpurun_out/${TAG}_pmc/pmc_k_match.json 1
