#!/bin/bash
# fbs_kernel breakdown from rocprof kernel durations against its timing
# variants (the experiments library, make -C w-fsa_amd/csrc exp; WFSA_FBS_DBG:
# 5 launch + finish only, 3 no stream pass, 8 no bubble code, 1 no table
# gathers, 9 stream loads only).  Variant results are wrong by design; only
# durations matter.  c3, 200-step runs of the device QN loop.  BRK_KNOB picks
# the knob (default WFSA_FBS_DBG; WFSA_QN_DBG: 3 launch alone, 1 launch +
# first round, 5 no slot sums), BRK_VARIANTS the values.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/fbrk
mkdir -p "$OUT"
export TMPDIR=/tmp WFSA_LIB=$R/w-fsa_amd/build_exp/libwfsa_amd.so RC_KS=200 RC_REPS=1 RC_RMIN=0
cd /tmp || exit 1
KNOB=${BRK_KNOB:-WFSA_FBS_DBG}
for v in ${BRK_VARIANTS:-0 5 3 8 1 9}; do
    env "$KNOB=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$KNOB$v" -o run -- \
        python3 "$R/tools/run_cost.py" > "$OUT/$KNOB$v.log" 2>&1 || exit 1
    f=$(find "$OUT/$KNOB$v" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" "$KNOB" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if ("fbs_kernel" in n or "qn_step" in n) and int(r["Calls"]) > 50:
        out.append(f"{n.split('(wfsa')[0].split('::')[-1][:48]} x{r['Calls']} avg {float(r['AverageNs'])/1e3:.2f} us")
print(f"{sys.argv[3]}={sys.argv[2]}: " + "; ".join(out), flush=True)
PY
done
