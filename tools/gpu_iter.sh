#!/bin/bash
# An iteration on the GPU: the named test files, then bench / stamps lines.
# Usage (through gpurun): bash tools/gpu_iter.sh <tag> "<pytest files>" ["bench:<args>" | "stamps:<args>" ...]
set -o pipefail
OUT=gpurun_out/${1:-iter}
TESTS="$2"
shift 2 || true
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -15 $OUT/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for item in "$@"; do
  kind=${item%%:*}; args=${item#*:}
  if [ "$kind" = "stamps" ]; then
    hot=""
    case "$args" in HOT=1*) hot=1; args="${args#HOT=1 }";; esac
    KME_STAMPS_HOT=$hot timeout -k 10 300 python3 -u bench.py --stamps --no-cpu-baseline --host-path-epochs 0 $args >> $OUT/stamps.jsonl 2>> $OUT/stamps.err
  else
    timeout -k 10 400 python3 -u bench.py --no-cpu-baseline $args >> $OUT/bench.jsonl 2>> $OUT/bench.err
  fi
  rc=$?; echo "$kind [$args] rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/$kind.err 2>/dev/null; exit $rc; }
done
[ -f $OUT/stamps.jsonl ] && cat $OUT/stamps.jsonl
[ -f $OUT/bench.jsonl ] && python3 - $OUT/bench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"]["symbols_per_gpu_rank0"], d["config"]["epoch_records"], round(d["value"] / 1e6, 1), "M/s p99",
          round(d["p99_epoch_ms"], 2), "match", [round(x, 3) for x in d["match_ms_per_step"]][-3:], d["phase_ms_last_epoch"],
          "host_path", (d.get("host_path") or {}).get("value"), (d.get("host_path") or {}).get("host_s"))
PY
exit 0
