#!/bin/bash
# The default bench line (headline + boundary + info_rmin + dense_c5 + famB sub-records, CPU baselines)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_full.json"))
print("headline", round(d["value"] / 1e9, 2), "G/s", round(d["ms_per_step"] * 1e3, 1), "us; frac", round(d["roofline"]["frac"], 3))
print("boundary", d.get("boundary"))
for k in ("dense_c5", "famB"):
    r = d.get(k) or {}
    if "error" in r: print(k, r); continue
    print(k, round(r.get("value", 0), 1), "strings/s", round(r.get("ms_per_step", 0), 2), "ms; roofline", {x: r["roofline"].get(x) for x in ("kernel", "achieved", "frac", "edge_ops_per_s", "fp64_flops_frac")}, "cpu", (r.get("cpu_baseline") or {}).get("value"))
PY
