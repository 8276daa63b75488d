# dense-path rmin column: its GPU tests, then its cost at c5 size
set -o pipefail
mkdir -p gpurun_out/drmin
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -k rmin -x -v --timeout 300 --timeout-method thread > gpurun_out/drmin/tests.log 2>&1 || { tail -40 gpurun_out/drmin/tests.log; exit 1; }
tail -8 gpurun_out/drmin/tests.log
timeout -k 10 300 python -u tools/dense_rmin_time.py > gpurun_out/drmin/time.log 2>&1 || { tail -20 gpurun_out/drmin/time.log; exit 1; }
cat gpurun_out/drmin/time.log
