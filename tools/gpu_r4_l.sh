# round 4: the first timed Run after preparation -- per-dispatch kernel times of every Run (bench_like under a kernel trace) and the bench at the driver's setting, twice
set -o pipefail
mkdir -p gpurun_out/r4l
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
WFSA_RUN_TRACE=1 BL_REPS=4 BL_STEPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4l/trace -o run -- python tools/bench_like.py > gpurun_out/r4l/trace.log 2>&1 || { tail -20 gpurun_out/r4l/trace.log; exit 1; }
grep -E "rep|qn_run" gpurun_out/r4l/trace.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4l/b$i.json 2> gpurun_out/r4l/b$i.err || { tail -20 gpurun_out/r4l/b$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4l/b$i.json'));print('driver setting', $i, round(d['ms_per_step']*1e3,2), 'us/step')"
done
