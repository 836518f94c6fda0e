#!/bin/bash
# pass cycles by record kind (stamps build, diagnostic)
set -o pipefail
bash tools/gpu_stamps_env.sh st6 '' 'HOT=1 --workload c4 --steps 2 --warmup 1' '--workload c2 --steps 3 --warmup 1' '--workload c3 --symbols 8192 --steps 3 --warmup 1' > /dev/null
rc=$?; cat gpurun_out/st6/stamps.jsonl 2>/dev/null; exit $rc
