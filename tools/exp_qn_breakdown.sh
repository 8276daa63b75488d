#!/bin/bash
# QN step breakdown from rocprof kernel durations: WFSA_QN_DBG 3 (launch
# only), 1 (launch + first load round), 5 (no bubble slot sums), 0 (all).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/qbrk
mkdir -p "$OUT"
WFSA_VERBOSE=1 timeout -k 10 120 python3 "$R/bench.py" --no-sub --cpu-sample 0 --boundary-steps 0 --steps 20 --warmup 2 > "$OUT/verbose.log" 2>&1 || exit 1
grep "slots per constraint" "$OUT/verbose.log" | head -2
export TMPDIR=/tmp
cd /tmp || exit 1
for v in ${BRK_VARIANTS:-0 3 1 5}; do
    WFSA_QN_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/v$v" -o run -- \
        python3 "$R/bench.py" --no-sub --cpu-sample 0 --boundary-steps 0 --steps 200 --warmup 10 > "$OUT/v$v.log" 2>&1 || exit 1
    f=$(find "$OUT/v$v" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if "fbs_kernel" in n or "qn_step" in n:
        out.append(f"{n.split('(wfsa')[0].split('::')[-1][:48]} x{r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us")
print(f"QN_DBG={sys.argv[2]}: " + "; ".join(out), flush=True)
PY
done
