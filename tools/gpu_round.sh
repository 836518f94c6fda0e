#!/bin/bash
# One full GPU round (through gpurun): parity tests, PMC traffic passes for k_match, the bench line
# (with CPU baseline), a rocprofv3 kernel-trace/stats profile of the same command, extra bench
# lines.  Usage: bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-round}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_kmatch.sh $TAG/pmc k_match "$@" || exit $?
cp $OUT/pmc/pmc_summary.json profiles/pmc_k_match_c3.json
timeout -k 10 500 python3 -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench_rc=$rc"; cat $OUT/bench.json; tail -2 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"
[ $rc -eq 0 ] || exit $rc
for extra in "--workload c3 --symbols 32768" "--workload c3 --symbols 8192" "--workload c2" "--workload c4 --steps 2 --warmup 1" "--workload c5"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline $extra >> $OUT/bench_extra.jsonl 2>> $OUT/bench_extra.err
  rc=$?; echo "extra [$extra] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
# occupancy / LDS bank conflicts / traffic of the N = 8 shard shape too (every group busy: k_match)
bash tools/pmc_kmatch.sh $TAG/pmc8k k_match --symbols 8192 || exit $?
cp $OUT/pmc8k/pmc_summary.json profiles/pmc_k_match_c3_s8192.json
