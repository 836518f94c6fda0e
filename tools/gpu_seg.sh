#!/bin/bash
# GPU tests of the current build, then earlier builds against it (diagnostic)
set -o pipefail
mkdir -p gpurun_out/ab
K=kafka-matching-engine_amd/kme
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/ab/tests.log
[ $rc -eq 0 ] || exit $rc
run() {
  args=$1; shift
  for L in "$@"; do
    KME_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --host-path-epochs 0 $args > gpurun_out/ab/one.json 2>gpurun_out/ab/err.log || { tail -3 gpurun_out/ab/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/one.json'));print('$(basename $L)', '$args', round(d['value']/1e6,1), d['phase_ms_last_epoch']['match'])"
  done
}
run "--workload c5 --steps 5 --warmup 2" $K/libkme_8fef8c7.so $K/libkme_3844a19.so $K/libkme.so $K/libkme_8fef8c7.so $K/libkme_3844a19.so $K/libkme.so
run "--workload c2 --steps 5 --warmup 2" $K/libkme_3844a19.so $K/libkme.so $K/libkme_3844a19.so $K/libkme.so
run "--workload c3 --symbols 8192 --steps 5 --warmup 2" $K/libkme_3844a19.so $K/libkme.so $K/libkme_3844a19.so $K/libkme.so
run "--workload c4 --steps 3 --warmup 1" $K/libkme_3844a19.so $K/libkme.so
