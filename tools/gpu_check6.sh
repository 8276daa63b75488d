set -o pipefail
mkdir -p gpurun_out/c6
timeout -k 10 600 python -u -m pytest tests/test_gpu_sym.py tests/test_gpu_hessian.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c6/sym.log 2>&1 || { tail -60 gpurun_out/c6/sym.log; exit 1; }
grep -cE "PASSED" gpurun_out/c6/sym.log; tail -2 gpurun_out/c6/sym.log
timeout -k 10 400 python -u tools/ranks_bench.py > gpurun_out/c6/ranks.txt 2> gpurun_out/c6/ranks.err || { tail -30 gpurun_out/c6/ranks.err; cat gpurun_out/c6/ranks.txt; exit 1; }
cat gpurun_out/c6/ranks.txt
bash tools/exp_fbs_breakdown.sh > gpurun_out/c6/fbrk.txt 2>&1 || { tail -20 gpurun_out/c6/fbrk.txt; exit 1; }
cat gpurun_out/c6/fbrk.txt
