mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmin.py -v --timeout 300 --timeout-method thread > gpurun_out/rmin_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert|passed|failed" gpurun_out/rmin_tests.log | head -80
exit $rc
