# round 4: dense path on both GEMM engines -- parity tests, then c5 timings
set -o pipefail
mkdir -p gpurun_out/r4d
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -v --timeout 180 --timeout-method thread --durations=10 > gpurun_out/r4d/tests.log 2>&1 || { tail -60 gpurun_out/r4d/tests.log; exit 1; }
tail -15 gpurun_out/r4d/tests.log
for e in 0 1; do
  WFSA_DENSE_BLAS=$e timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r4d/c5_blas$e.json 2> gpurun_out/r4d/c5_blas$e.err || { tail -20 gpurun_out/r4d/c5_blas$e.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4d/c5_blas$e.json'));print($e, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
WFSA_DENSE_BLAS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d/prof -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r4d/prof.log 2>&1 || { tail -20 gpurun_out/r4d/prof.log; exit 1; }
find gpurun_out/r4d/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
