#!/bin/bash
# QN kernel duration per debug variant from a kernel trace (WFSA_QN_DBG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/qn2"
export TMPDIR=/tmp
cd /tmp || exit 1
for d in ${QN_DBGS:-0 3 7}; do
  WFSA_QN_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/qn2/d$d" -o run -- python3 "$R/bench.py" --cpu-sample 0 --steps 50 > "$R/gpurun_out/qn2/d$d.log" 2>&1 || { tail "$R/gpurun_out/qn2/d$d.log"; exit 1; }
  echo "dbg $d: $(grep -h 'qn_step_kernel\|fbs_kernel<false, true, false, 0, false>' "$R/gpurun_out/qn2/d$d/run_kernel_stats.csv" | cut -d, -f1,4 | tr '\n' ' ')"
done
