timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_ledger.py > gpurun_out/w5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/w5_tests.log; [ $rc -eq 0 ] || exit $rc
for args in "--workload c3 --shard 0/8 --host-path-epochs 0" "--workload c3 --shard 0/4 --host-path-epochs 0" "--workload c3 --shard 0/2 --host-path-epochs 0" "--workload c5 --host-path-epochs 0"; do
  bash tools/ab_quick.sh "$args" kafka-matching-engine_amd/kme/libkme_base.so kafka-matching-engine_amd/kme/libkme.so || exit 1
done
