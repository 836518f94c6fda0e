mkdir -p gpurun_out/r05t
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_fast.py tests/test_gpu_ledger.py tests/test_gpu_faults.py tests/test_gpu_pipeline.py > gpurun_out/r05t/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05t/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_quick.sh "--host-path-epochs 0" kafka-matching-engine_amd/kme/libkme_base.so kafka-matching-engine_amd/kme/libkme.so
