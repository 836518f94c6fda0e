#!/bin/bash
# The end-of-round measurement set (through gpurun), every step under its own time limit:
#   1. the GPU parity suite and smoke;
#   2. the bench line (C3, CPU baseline, host path);
#   3. a rocprofv3 kernel trace of the same command (its averages are the frac's denominator);
#   4. the PMC traffic passes and the L2-request passes of k_match_lanes (the summary records the
#      profiled build's kme_build_id(); bench.py reports roofline.traffic only for that build);
#   5. the extra configuration lines (rank 0 of the N = 8 / 4 / 2 runs of C3, C2, C5, C4 and its N = 8
#      shard, the exact-ledger drop-in line),
#      plus the drop-in's own defaults (--java-defaults: 65,536-record epochs, exact ledger, host path)
#      and a commit point's checkpoint cost at C3;
#   6. a two-rank rehearsal of bench.py --gpus 2 on the one GPU (gloo: the N > 1 glue).
# Usage: bash tools/gpu_round5.sh <tag> [core|extra|all] [skip-tests]   (core = 1-4, extra = 5-6;
# each part fits one gpurun call)
set -o pipefail
TAG=${1:-round}
PART=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$PART" != "extra" ]; then
if [ "$3" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -2 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke_rc=$rc"; tail -1 $OUT/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench_rc=$rc"; cat $OUT/bench.json; tail -2 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-path-epochs 0 > $OUT/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f 5 $OUT/trace_summary.json "C3, 65,536 symbols, E = 2^22, 5 timed epochs" > /dev/null
bash tools/pmc_kmatch.sh $TAG/pmc k_match_lanes --host-path-epochs 0 || exit $?
bash tools/pmc_tcc.sh $TAG/tcc k_match_lanes kafka-matching-engine_amd/kme/libkme.so || exit $?
fi
[ "$PART" = "core" ] && exit 0
for extra in "--workload c3 --shard 0/8" "--workload c3 --shard 0/4" "--workload c3 --shard 0/2" "--workload c2" "--workload c5" "--workload c4 --steps 2 --warmup 1" "--workload c4 --shard 0/8 --steps 2 --warmup 1" "--workload c4 --epoch 262144 --steps 16 --warmup 2" "--flags exact_ledger,serial_fallback --steps 5 --warmup 2" "--java-defaults" "--steps 5 --warmup 2 --checkpoint /tmp/kmeck"; do
  hp="--host-path-epochs 0"; case "$extra" in *java-defaults*) hp="";; esac
  timeout -k 10 400 python3 -u bench.py --no-cpu-baseline $hp $extra >> $OUT/bench_extra.jsonl 2>> $OUT/bench_extra.err
  rc=$?; echo "extra [$extra] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_rehearse.sh $TAG/rehearse 2 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
