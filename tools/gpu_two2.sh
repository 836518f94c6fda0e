set -o pipefail
mkdir -p gpurun_out/two2
export TMPDIR=/tmp
KME_TWO_MAX=0 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fast.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/two2/one.log 2>&1
echo "one-wave rc=$?"; tail -3 gpurun_out/two2/one.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fast.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/two2/two.log 2>&1
echo "two-wave rc=$?"; grep -E "passed|failed|^FAILED" gpurun_out/two2/two.log | cut -c1-200
