mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_matrix.py -v --timeout 120 --timeout-method thread > gpurun_out/matrix_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert|passed|failed" gpurun_out/matrix_tests.log | head -80
exit $rc
