#!/bin/bash
# c5 (dense 4096-state, fp64 MFMA path): parity tests, bench line, kernel
# trace, one PMC pass (GPU box).  Usage: tools/gpu_c5.sh [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
OUT=$R/gpurun_out/c5
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 600 python -u bench.py --workload c5 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --workload c5 --steps 3 --warmup 1 --cpu-sample 0 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
head -8 "$OUT/trace/run_kernel_stats.csv"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/pmc1" -o run -- \
    python3 "$R/bench.py" --workload c5 --steps 1 --warmup 0 --cpu-sample 0 > "$OUT/pmc1.log" 2>&1 || { tail -20 "$OUT/pmc1.log"; exit 1; }
echo done
