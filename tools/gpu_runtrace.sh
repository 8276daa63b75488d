#!/bin/bash
# kernel trace of the bench's timed region (tools/bench_like.py) beside the library's own Run phases
# (WFSA_RUN_TRACE, host steady clock in ns) -- the per-Run fixed cost (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/runtrace"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
BL_REPS=3 WFSA_RUN_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/t" -o run -- \
    python3 "$R/tools/bench_like.py" > "$O/log.txt" 2>&1 || { tail -20 "$O/log.txt"; exit 1; }
grep -E "rep|qn_run 20" "$O/log.txt" | tail -4
