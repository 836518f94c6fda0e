set -o pipefail
mkdir -p gpurun_out/two3
export TMPDIR=/tmp
for v in 0 1; do
  KME_TWO_DRAIN=$v timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fast.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/two3/f$v.log 2>&1
  echo "KME_TWO_DRAIN=$v rc=$?"; grep -E "passed|failed|^FAILED" gpurun_out/two3/f$v.log | cut -c1-200
done
exit 0
