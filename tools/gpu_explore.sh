#!/bin/bash
# Exploration run: parity tests, then bench lines for several workloads/epoch sizes, then stamps.
set -o pipefail
OUT=gpurun_out/${1:-explore}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for args in "--workload c2" "--workload c3" "--workload c3 --epoch 4194304" "--workload c3 --epoch 8388608 --steps 6 --warmup 2"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline $args >> $OUT/bench.jsonl 2>> $OUT/bench.err
  rc=$?; echo "bench [$args] rc=$rc"; tail -c 600 $OUT/bench.jsonl
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --stamps --workload c2 > $OUT/stamps_c2.json 2>&1; echo "stamps rc=$?"; cat $OUT/stamps_c2.json | tail -2
timeout -k 10 300 python3 -u bench.py --stamps --workload c3 > $OUT/stamps_c3.json 2>&1; echo "stamps rc=$?"; cat $OUT/stamps_c3.json | tail -2
