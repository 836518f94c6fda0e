set -o pipefail
mkdir -p gpurun_out/two4
export TMPDIR=/tmp
KME_TWO_MAX=4096 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/two4/scale.log 2>&1
echo "rc=$?"; grep -E "passed|failed|^FAILED|^E  .*Fail" gpurun_out/two4/scale.log | cut -c1-300 | head -20
exit 0
