set -o pipefail
mkdir -p gpurun_out/rc
timeout -k 10 300 python -u tools/run_cost.py > gpurun_out/rc/fit.txt 2> gpurun_out/rc/fit.err || { tail -20 gpurun_out/rc/fit.err; exit 1; }
cat gpurun_out/rc/fit.txt
WFSA_RUN_TRACE=1 timeout -k 10 300 python -u tools/run_cost.py > gpurun_out/rc/trace.txt 2> gpurun_out/rc/trace.err || exit 1
grep -A2 "K=20" gpurun_out/rc/trace.err | head -5 || true
timeout -k 10 300 python -u bench.py --no-sub --cpu-sample 0 --steps 20 --warmup 10 > gpurun_out/rc/b20.json 2> gpurun_out/rc/b20.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/rc/b20.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['info_rmin']['ms_per_step'])"
