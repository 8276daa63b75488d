#!/bin/bash
# wave_pull_kernel: the traversal-string tests, then famB per-evaluation time with the pull and the push (wide2) kernel (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/pull
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier2.py tests/test_gpu_rmin.py tests/test_gpu_ranks.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pull/tests.log 2>&1 || { tail -40 gpurun_out/pull/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/pull/tests.log | tail -3
for p in 1 0; do
  WFSA_PULL=$p timeout -k 10 300 python -u tools/time_famb.py > gpurun_out/pull/famb_$p.log 2>&1 || { tail gpurun_out/pull/famb_$p.log; exit 1; }
  echo "pull=$p: $(tail -1 gpurun_out/pull/famb_$p.log)"
done
