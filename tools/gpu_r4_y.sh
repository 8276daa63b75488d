# round 4: Run returns once the last row is in (the stream's tail beside the return) -- every GPU test, the driver's setting twice, the default
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/r4y/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4y/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4y/d$i.json 2> gpurun_out/r4y/d$i.err || { tail -20 gpurun_out/r4y/d$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4y/d$i.json'));print('driver setting', $i, round(d['ms_per_step']*1e3,2), 'us/step')"
done
timeout -k 10 300 python -u bench.py --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4y/d200.json 2> gpurun_out/r4y/d200.err || { tail -20 gpurun_out/r4y/d200.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4y/d200.json'));print('200 steps', round(d['ms_per_step']*1e3,2), 'us/step')"
