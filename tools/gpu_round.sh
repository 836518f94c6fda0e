#!/bin/bash
# One GPU round: parity tests, the bench line, and a rocprofv3 kernel-trace summary.
# Usage (through gpurun): bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench_rc=$rc"; cat $OUT/bench.json; tail -2 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -20 "$f"
exit $rc
