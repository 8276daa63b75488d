# fbs time breakdown (GPU box): the default kernel against its timing variants
# (WFSA_FBS_DBG, fb_kernels.hip: 1 no table gathers, 3 no stream pass,
# 5 return at once, 8 no bubble code, 9 stream loads only).  Results of the
# variants are wrong by design; only the event-timed kernel durations matter.
set -o pipefail
mkdir -p gpurun_out/brk
run() {
  env "$@" timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/brk/b.json 2> gpurun_out/brk/b.err || { tail -5 gpurun_out/brk/b.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/brk/b.json')); print('$*', round(d['ms_per_step']*1e3, 2), 'us/step fbs', round(d['roofline']['kernel_ms_per_launch']*1e3, 2), 'us all_fb', round(d['roofline']['all_fb_kernels_ms_per_step']*1e3, 2))"
}
for v in ${BRK_VARIANTS:-0 1 3 5 8 9}; do run WFSA_FBS_DBG=$v || exit 1; done
