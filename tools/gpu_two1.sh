set -o pipefail
mkdir -p gpurun_out/two1
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fast.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/two1/fast.log 2>&1
rc=$?; echo "fast rc=$rc"; tail -5 gpurun_out/two1/fast.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_faults.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/two1/par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -5 gpurun_out/two1/par.log; [ $rc -eq 0 ] || exit $rc
