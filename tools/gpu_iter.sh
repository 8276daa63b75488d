#!/bin/bash
# One build->measure iteration on the GPU box: a short bench line, a kernel
# trace of the same command, then every -m gpu test.  Usage: tools/gpu_iter.sh [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--cpu-sample 0)
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u bench.py "${ARGS[@]}" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], (d.get('info_rmin') or {}).get('ms_per_step'))"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/trace" -o run -- \
    python3 "$R/bench.py" "${ARGS[@]}" --steps 20 > "$R/gpurun_out/prof/trace.log" 2>&1 || { tail -20 "$R/gpurun_out/prof/trace.log"; exit 1; }
cut -c1-150 "$R/gpurun_out/prof/trace/run_kernel_stats.csv" | head -12
cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
