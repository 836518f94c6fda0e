#!/bin/bash
# A/B of library builds on one box: bench lines and kernel traces, alternating.
# Usage (through gpurun): bash tools/ab_trace.sh <tag> "<bench args>" lib1.so lib2.so ...
set -o pipefail
TAG=${1:-ab}
ARGS="$2"
shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    KME_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --host-path-epochs 0 --steps 5 $ARGS >> $OUT/$n.jsonl 2>> $OUT/$n.err
    rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; tail -3 $OUT/$n.err; exit $rc; }
  done
done
for L in "$@"; do
  n=$(basename $L .so)
  KME_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n.prof -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-path-epochs 0 $ARGS > $OUT/$n.prof.log 2>&1 || exit $?
  f=$(find $OUT/$n.prof -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py $f 5 $OUT/$n.trace.json "$n" > /dev/null
  python3 - $OUT/$n.jsonl $OUT/$n.trace.json $n <<'PY'
import json, sys
vals = [json.loads(l)["value"] / 1e6 for l in open(sys.argv[1])]
t = json.load(open(sys.argv[2]))
print(sys.argv[3], [round(v, 1) for v in vals], {k.split("::")[-1]: round(v["avg_ns_timed"] / 1e3, 1) for k, v in t.items()
      if k.startswith("kme::k_") and v["avg_ns_timed"] > 20000})
PY
done
