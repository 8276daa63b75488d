#!/bin/bash
# tier-2 / traversal parity tests + the famB workload (kernel trace) (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/fb
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier2.py tests/test_gpu_rmin.py tests/test_gpu_ranks.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fb/tests.log 2>&1 || { tail -40 gpurun_out/fb/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/fb/tests.log | tail -3
timeout -k 10 300 python -u bench.py --workload famB --no-sub --cpu-sample 0 --boundary-steps 0 > gpurun_out/fb/famb.json 2>gpurun_out/fb/famb.err || { tail gpurun_out/fb/famb.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/fb/famb.json')); print('famB strings/s', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'roofline', d['roofline'])"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/fb/trace" -o run -- \
    python3 "$R/bench.py" --workload famB --no-sub --cpu-sample 0 --boundary-steps 0 --steps 5 > "$R/gpurun_out/fb/trace.log" 2>&1 || { tail -20 "$R/gpurun_out/fb/trace.log"; exit 1; }
head -8 "$R/gpurun_out/fb/trace/run_kernel_stats.csv" | cut -c1-160
