#!/bin/bash
# c5 dense per-step GEMM variants (WFSA_DENSE_STEP_CFG 0 / 1 / 2): rocprof
# kernel durations of a short c5 bench run each (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/dcfg
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for v in ${CFGS:-0 1 2}; do
    WFSA_DENSE_STEP_CFG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c$v" -o run -- \
        python3 "$R/bench.py" --workload c5 --steps 3 --warmup 1 --cpu-sample 0 --boundary-steps 0 > "$OUT/c$v.log" 2>&1 || exit 1
    f=$(find "$OUT/c$v" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" <<'PY'
import csv, sys
out = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "dense_gemm" in n:
        out.append(f"{n.split('(')[0].split('::')[-1]} x{r['Calls']} avg {float(r['AverageNs'])/1e3:.1f} us")
print(f"CFG={sys.argv[2]}: " + "; ".join(out), flush=True)
PY
done
