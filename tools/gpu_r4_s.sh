# round 4: the timed Run's host-side gaps (bench clock vs the library's qn_run clock, both CLOCK_MONOTONIC)
set -o pipefail
mkdir -p gpurun_out/r4s
for i in 1 2; do
  WFSA_BENCH_TRACE=1 WFSA_RUN_TRACE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4s/b$i.json 2> gpurun_out/r4s/b$i.err || { tail -20 gpurun_out/r4s/b$i.err; exit 1; }
  grep -E "^\[bench\]|qn_run 20|RunDevice" gpurun_out/r4s/b$i.err | head -3
done
for i in 3 4; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4s/c$i.json 2> gpurun_out/r4s/c$i.err || { tail -20 gpurun_out/r4s/c$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4s/c$i.json'));print('driver setting', $i, round(d['ms_per_step']*1e3,2), 'us/step')"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4s/pipe.log 2>&1 || { tail -20 gpurun_out/r4s/pipe.log; exit 1; }
tail -1 gpurun_out/r4s/pipe.log
