#!/bin/bash
# Full GPU check (GPU box): every -m gpu test, the default bench line (with
# its CPU baseline), a kernel trace of a short bench run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/trace" -o run -- \
    python3 "$R/bench.py" --cpu-sample 0 --steps 20 > "$R/gpurun_out/prof/trace.log" 2>&1 || { tail -20 "$R/gpurun_out/prof/trace.log"; exit 1; }
head -6 "$R/gpurun_out/prof/trace/run_kernel_stats.csv"
