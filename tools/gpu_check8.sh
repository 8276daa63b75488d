set -o pipefail
mkdir -p gpurun_out/c8
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c8/dense.log 2>&1 || { tail -60 gpurun_out/c8/dense.log; exit 1; }
grep -cE "PASSED" gpurun_out/c8/dense.log; tail -2 gpurun_out/c8/dense.log
timeout -k 10 300 python -u bench.py --workload c5 --cpu-sample 0 > gpurun_out/c8/c5.json 2> gpurun_out/c8/c5.err || { tail -20 gpurun_out/c8/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c8/c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['evaluation_ms'])"
WFSA_DENSE_BLAS=0 timeout -k 10 300 python -u bench.py --workload c5 --cpu-sample 0 > gpurun_out/c8/c5_fused.json 2> gpurun_out/c8/c5_fused.err || { tail -20 gpurun_out/c8/c5_fused.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c8/c5_fused.json')); print('c5 fused', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['evaluation_ms'])"
