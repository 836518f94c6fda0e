#!/bin/bash
# A/B of several builds of libkme.so without the test pass (diagnostic; the variants' parity is
# checked separately).  Usage (through gpurun): bash tools/ab_quick.sh "<bench args>" lib1.so lib2.so ...
set -o pipefail
ARGS=$1
shift
mkdir -p gpurun_out/abq
for rep in 1 2; do
  for L in "$@"; do
    KME_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 8 --warmup 2 $ARGS > gpurun_out/abq/one.json 2>gpurun_out/abq/err.log || { tail -3 gpurun_out/abq/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abq/one.json'));print('$(basename $L)', '$ARGS', round(d['value']/1e6,1), {k:v for k,v in d['phase_ms_last_epoch'].items() if v})"
  done
done
