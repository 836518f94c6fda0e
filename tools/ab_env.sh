#!/bin/bash
# A/B of environment settings on one build (diagnostic knobs: KME_LEDGER_HBITS, KME_LEDGER_GRID, ...).
# Usage (through gpurun): bash tools/ab_env.sh "<bench args>" "<env settings 1>" "<env settings 2>" ...
# ("-" = no settings)
set -o pipefail
ARGS=$1
shift
mkdir -p gpurun_out/abe
for rep in 1 2; do
  for E in "$@"; do
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 $ARGS > gpurun_out/abe/one.json 2>gpurun_out/abe/err.log || { tail -3 gpurun_out/abe/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abe/one.json'));print('[$E]', '$ARGS', round(d['value']/1e6,1), {k:v for k,v in d['phase_ms_last_epoch'].items() if v}, d.get('exact_ledger'))"
  done
done
