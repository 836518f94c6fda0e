#!/bin/bash
# Host-path A/B of the row expansion's thread sizing (KME_EXPAND_MIN records per thread) at the drop-in's
# defaults.  Usage (through gpurun): bash tools/gpu_hostpath_ab.sh <tag> <min1> <min2> ...
set -o pipefail
OUT=gpurun_out/${1:-hpab}
shift
mkdir -p $OUT
for rep in 1 2; do
  for m in "$@"; do
    KME_EXPAND_MIN=$m timeout -k 10 300 python3 bench.py --java-defaults --no-cpu-baseline --steps 4 --warmup 2 > $OUT/one.json 2> $OUT/err.log || { tail -3 $OUT/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/one.json'));h=d['host_path'];print('min', $m, round(h['value']/1e6,1), h['host_s'])"
  done
done
