# c4 at full size, c5 per-element gradient, the per-Run cost fit, the stream-format micro
set -o pipefail
mkdir -p gpurun_out/c3
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_dense.py -x -v --timeout 500 --timeout-method thread > gpurun_out/c3/tests.log 2>&1 || { tail -40 gpurun_out/c3/tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/c3/tests.log | tail -12
WFSA_RUN_TRACE=1 timeout -k 10 300 python -u tools/run_cost.py > gpurun_out/c3/fit.txt 2> gpurun_out/c3/fit.err || { tail -20 gpurun_out/c3/fit.err; exit 1; }
cat gpurun_out/c3/fit.txt
timeout -k 10 120 tools/micro/chain_walk > gpurun_out/c3/chain_walk.txt 2>&1 || { cat gpurun_out/c3/chain_walk.txt; exit 1; }
cat gpurun_out/c3/chain_walk.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiprocess.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c3/mp.log 2>&1 || { tail -60 gpurun_out/c3/mp.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/c3/mp.log | tail -5
