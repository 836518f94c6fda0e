#!/bin/bash
# Bench lines over values of one environment variable (diagnostic).
# Usage (through gpurun): bash tools/sweep_env.sh VAR "v1 v2 ..." "<bench args>"
set -o pipefail
VAR=$1; VALS=$2; ARGS=$3
mkdir -p gpurun_out/sweep
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline $ARGS > gpurun_out/sweep/one.json 2>gpurun_out/sweep/err.log || { tail -3 gpurun_out/sweep/err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweep/one.json'));print('$VAR=$v', '$ARGS', round(d['value']/1e6,1), d['phase_ms_last_epoch']['match'])"
done
