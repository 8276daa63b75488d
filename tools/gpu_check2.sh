# GPU tests (every -m gpu test, one process), then the per-Run cost fit and a
# 20-step bench (the driver's setting), then the c4 test
set -o pipefail
mkdir -p gpurun_out/c2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_c4.py > gpurun_out/c2/tests.log 2>&1 || { tail -40 gpurun_out/c2/tests.log; exit 1; }
tail -2 gpurun_out/c2/tests.log
WFSA_RUN_TRACE=1 timeout -k 10 300 python -u tools/run_cost.py > gpurun_out/c2/fit.txt 2> gpurun_out/c2/fit.err || { tail -20 gpurun_out/c2/fit.err; exit 1; }
cat gpurun_out/c2/fit.txt
timeout -k 10 300 python -u bench.py --no-sub --cpu-sample 0 --steps 20 --warmup 10 > gpurun_out/c2/b20.json 2> gpurun_out/c2/b20.err || { tail -20 gpurun_out/c2/b20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c2/b20.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['info_rmin']['ms_per_step'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py -x -v --timeout 500 --timeout-method thread > gpurun_out/c2/c4.log 2>&1 || { tail -40 gpurun_out/c2/c4.log; exit 1; }
tail -5 gpurun_out/c2/c4.log
