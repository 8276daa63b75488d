#!/bin/bash
# Timing experiments on the stream kernel (GPU box): kernel trace of a short
# bench under each WFSA_FBS_DBG variant (results of variants 1-3 are wrong by
# design; only the kernel durations matter).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp || exit 1
for v in ${FBS_VARIANTS:-0 1 2 3}; do
    WFSA_FBS_DBG=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/fbsx/v$v" -o run -- \
        python3 "$R/bench.py" --cpu-sample 0 --steps 20 > "$R/gpurun_out/fbsx/v$v.log" 2>&1 || exit 1
    echo "variant $v"; grep -E "fbs_kernel|bubble|tail|qn_" "$R/gpurun_out/fbsx/v$v/run_kernel_stats.csv" | cut -d, -f1-4
done
