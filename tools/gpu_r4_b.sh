# round 4: stream micro v4 with the delta formats; dense path after the scratch fix (both engines)
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 120 tools/micro/stream_v4 > gpurun_out/r4b/stream_v4.txt 2>&1 || { cat gpurun_out/r4b/stream_v4.txt; exit 1; }
cat gpurun_out/r4b/stream_v4.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r4b/dense_tests.log 2>&1 || { tail -40 gpurun_out/r4b/dense_tests.log; exit 1; }
tail -2 gpurun_out/r4b/dense_tests.log
for e in 0 1; do
  WFSA_DENSE_BLAS=$e timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/r4b/c5_blas$e.json 2> gpurun_out/r4b/c5_blas$e.err || { tail -20 gpurun_out/r4b/c5_blas$e.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4b/c5_blas$e.json'));print($e, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
WFSA_DENSE_BLAS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b/prof -o run -- python bench.py --workload c5 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/r4b/prof.log 2>&1 || { tail -20 gpurun_out/r4b/prof.log; exit 1; }
find gpurun_out/r4b/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
