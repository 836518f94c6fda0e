#!/bin/bash
# round measurement of the current build, then a short A/B against earlier builds (diagnostic)
set -o pipefail
TAG=${1:-r03e}
bash tools/gpu_round3.sh $TAG || exit $?
K=kafka-matching-engine_amd/kme
mkdir -p gpurun_out/ab
run() {
  args=$1; shift
  for L in "$@"; do
    KME_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --host-path-epochs 0 $args > gpurun_out/ab/one.json 2>gpurun_out/ab/err.log || { tail -3 gpurun_out/ab/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/one.json'));print('$(basename $L)', '$args', round(d['value']/1e6,1), d['phase_ms_last_epoch']['match'])" | tee -a gpurun_out/$TAG/ab.txt
  done
}
run "--workload c5 --steps 5 --warmup 2" $K/libkme_8fef8c7.so $K/libkme_3844a19.so $K/libkme.so
run "--workload c2 --steps 5 --warmup 2" $K/libkme_3844a19.so $K/libkme.so
run "--workload c3 --symbols 8192 --steps 5 --warmup 2" $K/libkme_3844a19.so $K/libkme.so
