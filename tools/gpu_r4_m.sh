# round 4: the dealer's bubble charges re-swept for the delta rows (rocprof kernel averages over bench_like)
set -o pipefail
mkdir -p gpurun_out/r4m2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" BL_REPS=2 BL_STEPS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4m2/$n -o run -- python tools/bench_like.py > gpurun_out/r4m2/$n.log 2>&1 || { tail -20 gpurun_out/r4m2/$n.log; return 1; }
  python - $n $(find gpurun_out/r4m2/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if "fbs_kernel" in r["Name"]:
        print(sys.argv[1], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
}
for c in 10 14 18 24 30; do run small$c WFSA_SMALL_COST=$c || exit 1; done
for c in 4 12 16; do run big$c WFSA_BIG_COST=$c || exit 1; done
