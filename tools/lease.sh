#!/bin/bash
# One GPU lease, parameterised: runs the named steps in order, each under its
# own time limit, stopping at the first failure (no retries).  Usage:
#   bash tools/lease.sh OUT_NAME step [step ...]
# Output goes to gpurun_out/OUT_NAME/.  Steps:
#   tests          every GPU test (pytest -m gpu)
#   tests:EXPR     GPU tests selected by -k EXPR
#   smoke          __graft_entry__.smoke()
#   profile        kernel trace + PMC passes over bench.py --steps 50 (tools/profile.sh),
#                  traffic record, PMC summary, kernel stats
#   fbrk           fbs_kernel breakdown over the timing variants (experiments library,
#                  tools/exp_fbs_breakdown.sh; BRK_KNOB / BRK_VARIANTS pass through)
#   trace          rocprof kernel trace + stats of bench.py --steps 200 --no-sub
#   driver         bench.py at the driver's setting (--steps 20 --warmup 5)
#   default        bench.py with no arguments
#   famb           bench.py --workload famB
#   c5             bench.py --workload c5 (our kernels and rocBLAS)
#   runcost        tools/run_cost.py (per-Run fixed cost fit)
#   summary        one line per bench JSON written by this lease
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1; shift
O=$R/gpurun_out/$NAME
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp

step() {
    local s=$1
    echo "== $s $(date +%T)"
    case $s in
    tests)
        timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 180 --timeout-method thread \
            > "$O/gpu_tests.log" 2>&1; local rc=$?; tail -3 "$O/gpu_tests.log"; return $rc ;;
    tests:*)
        timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 180 --timeout-method thread -k "${s#tests:}" \
            > "$O/gpu_tests_k.log" 2>&1; local rc=$?; tail -3 "$O/gpu_tests_k.log"; return $rc ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
        local rc=$?; tail -2 "$O/smoke.log"; return $rc ;;
    profile)
        bash tools/profile.sh "$O/prof" --steps 50 --warmup 10 --cpu-sample 0 --no-sub --boundary-steps 0 || return 1
        python tools/traffic.py "$O/prof" "$O/traffic_latest.json" || return 1
        python tools/pmc_summary.py "$O/prof" fbs_kernel > "$O/pmc.txt" 2>&1
        cp "$(find "$O/prof/trace" -name '*kernel_stats.csv' | head -1)" "$O/kernel_stats.csv" ;;
    fbrk)
        bash tools/exp_fbs_breakdown.sh > "$O/fbrk.txt" 2>&1; local rc=$?; cat "$O/fbrk.txt"; return $rc ;;
    trace)
        (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
            python3 "$R/bench.py" --steps 200 --warmup 20 --cpu-sample 0 --no-sub --boundary-steps 0 \
            > "$O/trace.log" 2>&1) || { tail -20 "$O/trace.log"; return 1; }
        cp "$(find "$O/trace" -name '*kernel_stats.csv' | head -1)" "$O/trace_kernel_stats.csv"
        python - "$O/trace_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 50:
        print(r["Name"][:70], r["Calls"], "avg", round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
        ;;
    driver)
        timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
            || { tail -20 "$O/bench_driver.err"; return 1; } ;;
    default)
        timeout -k 10 600 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" \
            || { tail -20 "$O/bench_default.err"; return 1; } ;;
    famb)
        timeout -k 10 600 python -u bench.py --workload famB > "$O/bench_famb.json" 2> "$O/bench_famb.err" \
            || { tail -20 "$O/bench_famb.err"; return 1; } ;;
    c5)
        timeout -k 10 900 python -u bench.py --workload c5 > "$O/bench_c5.json" 2> "$O/bench_c5.err" \
            || { tail -20 "$O/bench_c5.err"; return 1; } ;;
    runcost)
        timeout -k 10 600 python -u tools/run_cost.py > "$O/runcost.txt" 2>&1; local rc=$?; cat "$O/runcost.txt"; return $rc ;;
    summary)
        python - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e); continue
    sub = {k: (round(v["value"], 4 if v["value"] < 100 else 0), round(v.get("roofline", {}).get("frac", 0), 3))
           for k, v in d.items() if isinstance(v, dict) and "value" in v}
    print(os.path.basename(f), d["metric"][:24], f"{d['value']:.4g}", d["unit"], f"{d['ms_per_step'] * 1e3:.2f} us/step",
          "frac", round(d.get("roofline", {}).get("frac", 0), 3), sub)
PY
        ;;
    *) echo "unknown step $s"; return 2 ;;
    esac
}

for s in "$@"; do
    step "$s" || { echo "step $s failed"; exit 1; }
done
echo "== done $(date +%T)"
