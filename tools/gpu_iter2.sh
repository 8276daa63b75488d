#!/bin/bash
# famB layout variants + the per-Run phases of the c3 loop (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/it2
bash tools/gpu_pull_var.sh || exit 1
WFSA_RUN_TRACE=1 BL_REPS=4 timeout -k 10 200 python -u tools/bench_like.py > gpurun_out/it2/bl.log 2>&1 || { tail gpurun_out/it2/bl.log; exit 1; }
tail -12 gpurun_out/it2/bl.log
