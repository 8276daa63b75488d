#!/bin/bash
# kernel timeline of the QN loop, pipelined (WFSA_PIPE=1) and single-stream (0) (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/pt"
export TMPDIR=/tmp
cd /tmp || exit 1
for p in 1 0; do
  WFSA_PIPE=$p timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pt/p$p" -o run -- \
    python3 "$R/bench.py" --no-sub --cpu-sample 0 --boundary-steps 0 --steps 30 --warmup 2 > "$R/gpurun_out/pt/p$p.log" 2>&1 || { tail -5 "$R/gpurun_out/pt/p$p.log"; exit 1; }
  echo "== WFSA_PIPE=$p"; grep -o '"ms_per_step": [0-9.]*' "$R/gpurun_out/pt/p$p.log" | head -2
  python3 "$R/tools/trace_timeline.py" "$R/gpurun_out/pt/p$p/run_kernel_trace.csv" 24
done
