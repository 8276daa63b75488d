#!/bin/bash
# the bench's timed region with the loop's kernel timing on / off, and the Run phases (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/tim
for t in 1 0 1 0; do
  WFSA_TIMING=$t BL_REPS=4 WFSA_RUN_TRACE=1 timeout -k 10 200 python -u tools/bench_like.py > gpurun_out/tim/t$t.log 2>&1 || { tail gpurun_out/tim/t$t.log; exit 1; }
  echo "timing=$t: $(grep rep gpurun_out/tim/t$t.log | tail -3 | tr '\n' ' ')"
  grep "qn_run 20" gpurun_out/tim/t$t.log | tail -1
done
