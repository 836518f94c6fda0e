#!/bin/bash
# A/B of two builds of libkme.so (diagnostic): GPU tests with the variant, then alternating bench
# runs.  Usage (through gpurun): bash tools/ab_lib.sh <variant .so> "<bench args 1>" ...
set -o pipefail
VAR=${1:-kafka-matching-engine_amd/kme/libkme_var.so}
shift || true
mkdir -p gpurun_out/ab
KME_LIB=$VAR timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1
rc=$?; echo tests_rc=$rc; tail -2 gpurun_out/ab/tests.log
[ $rc -eq 0 ] || exit $rc
for args in "$@"; do
  for L in kafka-matching-engine_amd/kme/libkme.so $VAR kafka-matching-engine_amd/kme/libkme.so $VAR; do
    KME_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > gpurun_out/ab/one.json 2>gpurun_out/ab/err.log || { tail -3 gpurun_out/ab/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/one.json'));print('$(basename $L)', '$args', round(d['value']/1e6,1), d['phase_ms_last_epoch']['match'])"
  done
done
