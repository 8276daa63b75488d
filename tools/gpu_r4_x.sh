# round 4: the timed Run's host-side gaps on the final tree (bench clock, wrapper clock, library clock; CLOCK_MONOTONIC)
set -o pipefail
mkdir -p gpurun_out/r4x
for i in 1 2; do
  WFSA_BENCH_TRACE=1 WFSA_RUN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4x/b$i.json 2> gpurun_out/r4x/b$i.err || { tail -20 gpurun_out/r4x/b$i.err; exit 1; }
  grep -E "^\[bench\]|qn_run 20|wfsa.py|RunDevice" gpurun_out/r4x/b$i.err | head -8
  python -c "import json;d=json.load(open('gpurun_out/r4x/b$i.json'));print('driver setting', $i, round(d['ms_per_step']*1e3,2), 'us/step')"
done
