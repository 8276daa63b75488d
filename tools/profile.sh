#!/bin/bash
# Kernel trace + PMC passes over a short bench run (GPU box).  Usage:
#   tools/profile.sh OUT_DIR [bench args...]
# Each counter group runs in its own rocprofv3 pass (no --pmc with tracing
# domains other than --kernel-trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(readlink -f "${1:-$R/gpurun_out/prof}"); shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 10 --warmup 2 --cpu-sample 0)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
run() {  # name, rocprofv3 options...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/$name.log" 2>&1
}
run trace --kernel-trace --stats &&
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run sq2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum &&
# calibration of FETCH_SIZE / WRITE_SIZE on a known byte count (same access width)
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calfetch" -o run -- "$R/tools/micro/fetch_calib" > "$OUT/calfetch.log" 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calwrite" -o run -- "$R/tools/micro/fetch_calib" > "$OUT/calwrite.log" 2>&1
