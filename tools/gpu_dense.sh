mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dense_tests.log 2>&1
rc=$?
tail -30 gpurun_out/dense_tests.log
exit $rc
