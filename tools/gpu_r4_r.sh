# round 4: where the driver-setting timed region's wall time goes (bench.py --steps 20 --warmup 5, library and bench traces)
set -o pipefail
mkdir -p gpurun_out/r4r
for i in 1 2 3; do
  WFSA_BENCH_TRACE=1 WFSA_RUN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4r/b$i.json 2> gpurun_out/r4r/b$i.err || { tail -20 gpurun_out/r4r/b$i.err; exit 1; }
  grep -E "^\[bench\]|qn_run|RunDevice" gpurun_out/r4r/b$i.err | tail -4
  python -c "import json;d=json.load(open('gpurun_out/r4r/b$i.json'));print('driver setting', $i, round(d['ms_per_step']*1e3,2), 'us/step')"
done
WFSA_BENCH_TRACE=1 WFSA_RUN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 100 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4r/w100.json 2> gpurun_out/r4r/w100.err || { tail -20 gpurun_out/r4r/w100.err; exit 1; }
grep -E "^\[bench\]|qn_run|RunDevice" gpurun_out/r4r/w100.err | tail -4
python -c "import json;d=json.load(open('gpurun_out/r4r/w100.json'));print('warmup 100', round(d['ms_per_step']*1e3,2), 'us/step')"
