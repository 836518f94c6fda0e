set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1; echo tests_rc=$?; tail -2 gpurun_out/ab/tests.log
for L in libkme libkme_occ5 libkme libkme_occ5; do
  KME_LIB=kafka-matching-engine_amd/kme/$L.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab/$L.json 2>gpurun_out/ab/err.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$L.json'));print('$L', round(d['value']/1e6,1), d['phase_ms_last_epoch']['match'])"
done
