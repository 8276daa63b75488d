#!/bin/bash
# tier-2 tests + family B bench probes (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/fb
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier2.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fb/tests.log 2>&1 || { tail -40 gpurun_out/fb/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed|tier2" gpurun_out/fb/tests.log | tail -8
for n in ${NS:-10000 100000}; do
timeout -k 10 300 python -u bench.py --vocab 16 --emissions 4 --strings-per-gpu $n --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/fb/b_$n.json 2>gpurun_out/fb/b_$n.err || { tail gpurun_out/fb/b_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/fb/b_$n.json')); print('B $n', 'strings/s', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'compiled', d['compiled_strings'], 'fallback', d['fallback_strings'], 'tier1', d['tier1_strings'], 'bubbles', d['n_bubbles'], 'prep ms', round(d['prepare_ms']), 'fb ms', d['roofline']['all_fb_kernels_ms_per_step'])"
done
