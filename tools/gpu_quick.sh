#!/bin/bash
# Quick GPU iteration: parity tests, then bench lines for the given workloads (no CPU baseline).
# Usage (through gpurun): bash tools/gpu_quick.sh <tag> "<bench args 1>" "<bench args 2>" ...
set -o pipefail
OUT=gpurun_out/${1:-quick}
shift || true
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -5 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for args in "$@"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline $args >> $OUT/bench.jsonl 2>> $OUT/bench.err
  rc=$?; echo "bench [$args] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/bench.err; exit $rc; }
done
python3 - $OUT/bench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"]["symbols_per_gpu_rank0"], d["config"]["epoch_records"], round(d["value"] / 1e6, 1), "M/s p99",
          round(d["p99_epoch_ms"], 2), d["phase_ms_last_epoch"])
PY
