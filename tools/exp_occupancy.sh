# fbs occupancy experiment (GPU box): the fused kernel (118 VGPRs, 1 block/CU)
# vs the bubble-free variant (58 VGPRs) with the bubbles on the side stream,
# at 1 and 2 blocks per CU
set -o pipefail
mkdir -p gpurun_out/occ
run() {
  env "$@" timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/occ/b.json 2> gpurun_out/occ/b.err || { tail -5 gpurun_out/occ/b.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/occ/b.json')); print('$*', round(d['value']/1e9, 2), 'G/s', round(d['ms_per_step']*1e3, 2), 'us/step fbs', round(d['roofline']['kernel_ms_per_launch']*1e3, 2), 'us all_fb', round(d['roofline']['all_fb_kernels_ms_per_step']*1e3, 2))"
}
run WFSA_FBS_DBG=0 && run WFSA_FUSE_BUBBLES=0 && run WFSA_FBS_DBG=10 WFSA_FUSE_BUBBLES=0 WFSA_IPERCU=1 && run WFSA_FBS_DBG=10 WFSA_FUSE_BUBBLES=0 WFSA_IPERCU=2
