#!/bin/bash
# A/B of several builds of libkme.so (diagnostic): GPU tests with the default build, then the bench
# lines of every build, alternating, twice.  Usage (through gpurun):
#   bash tools/ab_multi.sh "<bench args>" lib1.so lib2.so ...
set -o pipefail
ARGS=$1
shift
mkdir -p gpurun_out/abm
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/abm/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/abm/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for L in "$@"; do
    KME_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline $ARGS > gpurun_out/abm/one.json 2>gpurun_out/abm/err.log || { tail -3 gpurun_out/abm/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abm/one.json'));print('$(basename $L)', '$ARGS', round(d['value']/1e6,1), d['p99_epoch_ms'], d['phase_ms_last_epoch'])"
  done
done
