#!/bin/bash
# A/B of an environment setting (diagnostic): GPU tests with it, then alternating bench runs.
# Usage (through gpurun): bash tools/ab_env.sh "<VAR=value ...>" "<bench args 1>" ...
set -o pipefail
ENVSET=$1
shift || true
mkdir -p gpurun_out/ab
env $ENVSET timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo "tests [$ENVSET] rc=$rc"; tail -3 gpurun_out/ab/tests.log
[ $rc -eq 0 ] || exit $rc
for args in "$@"; do
  for E in ${AB_ORDER:-"" "$ENVSET" "" "$ENVSET"}; do
    env $E timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > gpurun_out/ab/one.json 2>gpurun_out/ab/err.log || { tail -3 gpurun_out/ab/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/one.json'));print('[$E]', '$args', round(d['value']/1e6,1), d['phase_ms_last_epoch']['match'])"
  done
done
