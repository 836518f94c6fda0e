#!/bin/bash
# GPU tests with the default settings, then bench lines under several environment settings
# (diagnostic A/B on one box).  Usage (through gpurun):
#   bash tools/ab_envs.sh <tag> "<pytest files or -: skip>" "<ENV=v ...>|<ENV=v ...>" "<bench args 1>" ...
# ("-" in the env list stands for the defaults; each setting runs twice, alternating.)
set -o pipefail
OUT=gpurun_out/${1:-abe}
TESTS="$2"
IFS='|' read -r -a ENVS <<< "$3"
shift 3 || true
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -3 $OUT/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for args in "$@"; do
  for rep in 1 2; do
    for E in "${ENVS[@]}"; do
      [ "$E" = "-" ] && E=""
      env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline --host-path-epochs 0 $args > $OUT/one.json 2> $OUT/err.log
      rc=$?; [ $rc -eq 0 ] || { echo "[$E] $args rc=$rc"; tail -3 $OUT/err.log; exit $rc; }
      cat $OUT/one.json >> $OUT/bench.jsonl
      python3 -c "import json;d=json.load(open('$OUT/one.json'));print('[$E]', '$args', round(d['value']/1e6,1), 'M/s p99', round(d['p99_epoch_ms'],2), 'match', d['phase_ms_last_epoch']['match'])"
    done
  done
done
