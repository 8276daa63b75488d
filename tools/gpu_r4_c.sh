# round 4: delta stream format -- every GPU test, the c3 bench A/B (delta on/off), rocprof of the headline
set -o pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/r4c/tests.log 2>&1
rc=$?
tail -15 gpurun_out/r4c/tests.log
[ $rc -eq 0 ] || exit $rc
for d in 1 0; do
  WFSA_DELTA=$d timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4c/c3_delta$d.json 2> gpurun_out/r4c/c3_delta$d.err || { tail -20 gpurun_out/r4c/c3_delta$d.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4c/c3_delta$d.json'));print('delta', $d, d['value']/1e9, d['ms_per_step']*1e3, d['roofline']['frac'], d['stream_bytes'] if 'stream_bytes' in d else '')"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c/prof -o run -- python bench.py --steps 200 --warmup 10 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4c/prof.log 2>&1 || { tail -20 gpurun_out/r4c/prof.log; exit 1; }
find gpurun_out/r4c/prof -name "*kernel_stats.csv" | head -1 | xargs head -8
WFSA_DENSE_BLAS=0 timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --boundary-steps 0 > gpurun_out/r4c/c5_blas0.json 2> gpurun_out/r4c/c5_blas0.err || { tail -20 gpurun_out/r4c/c5_blas0.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4c/c5_blas0.json'));print('c5 mfma', d['value'], d['ms_per_step'], d['roofline']['frac'])"
