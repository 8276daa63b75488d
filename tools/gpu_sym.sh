set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py -v --timeout 300 --timeout-method thread > gpurun_out/sym_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert|passed|failed" gpurun_out/sym_tests.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/hessian_c3.py 2>&1 | tee gpurun_out/hessian_c3.log
