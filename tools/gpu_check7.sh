set -o pipefail
mkdir -p gpurun_out/c7
WFSA_KKT_TRACE=1 timeout -k 10 900 python -u tools/hessian_c3.py > gpurun_out/c7/hessian_c3.log 2>&1 || { tail -30 gpurun_out/c7/hessian_c3.log; exit 1; }
cat gpurun_out/c7/hessian_c3.log
timeout -k 10 120 tools/micro/dgemm_rocblas > gpurun_out/c7/dgemm.txt 2>&1 || { cat gpurun_out/c7/dgemm.txt; exit 1; }
cat gpurun_out/c7/dgemm.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 200 --timeout-method thread -k capacity > gpurun_out/c7/ranks.log 2>&1 || { tail -40 gpurun_out/c7/ranks.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/c7/ranks.log
