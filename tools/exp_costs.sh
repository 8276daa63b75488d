# Load-balancer cost sweep (GPU box): the rows the wave dealer charges for a
# wave's small bubbles (WFSA_SMALL_COST), big bubbles (WFSA_BIG_COST) and the
# QN finish (WFSA_FIN_COST), wfsa_dev.hip; default 8 each.
set -o pipefail
mkdir -p gpurun_out/cost
run() {
  env "$@" timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/cost/b.json 2> gpurun_out/cost/b.err || { tail -5 gpurun_out/cost/b.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cost/b.json')); print('$*', round(d['value']/1e9, 2), 'G/s', round(d['ms_per_step']*1e3, 2), 'us/step fbs', round(d['roofline']['kernel_ms_per_launch']*1e3, 2), 'us')"
}
if [ -n "$COST_RUNS" ]; then eval "$COST_RUNS"; exit $?; fi
run A=default &&
run WFSA_SMALL_COST=4 && run WFSA_SMALL_COST=16 && run WFSA_SMALL_COST=24 &&
run WFSA_BIG_COST=4 && run WFSA_BIG_COST=16 && run WFSA_BIG_COST=32 &&
run WFSA_FIN_COST=0 && run WFSA_FIN_COST=16 &&
run WFSA_SMALL_COST=16 WFSA_BIG_COST=16 WFSA_FIN_COST=16
