#!/bin/bash
# Iteration loop on the GPU box: parity tests (a -k selection), then bench lines.
# Usage (through gpurun): bash tools/gpu_iter.sh <tag> "<pytest -k expr or ALL>" "<bench args 1>" ...
set -o pipefail
OUT=gpurun_out/${1:-iter}
K=${2:-ALL}
shift 2 || true
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" = "ALL" ]; then SEL=(); else SEL=(-k "$K"); fi
if [ "$K" != "NONE" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread "${SEL[@]}" > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -3 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for args in "$@"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline $args >> $OUT/bench.jsonl 2>> $OUT/bench.err
  rc=$?; echo "bench [$args] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
done
[ -f $OUT/bench.jsonl ] || exit 0
python3 - $OUT/bench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "lane_stamps" in d:
        print({k: round(v) for k, v in d["lane_stamps"]["cycles_per_step"].items()}, round(d["lane_stamps"]["ms_per_epoch_match"], 3))
        continue
    print(d["config"]["symbols_per_gpu_rank0"], d["config"]["epoch_records"], round(d["value"] / 1e6, 1), "M/s p99",
          round(d["p99_epoch_ms"], 2), {k: v for k, v in d["phase_ms_last_epoch"].items() if v})
PY
