# round 4: the stream kernel's block geometry re-checked with the delta format (two 512-thread blocks per CU, the
# default, each staging the weight table, vs one 1024-thread block per CU staging it once)
set -o pipefail
mkdir -p gpurun_out/r4q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" BL_REPS=3 BL_STEPS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4q/$n -o run -- python tools/bench_like.py > gpurun_out/r4q/$n.log 2>&1 || { tail -20 gpurun_out/r4q/$n.log; return 1; }
  echo "== $n: $(grep rep gpurun_out/r4q/$n.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4q/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fbs_kernel" in r["Name"] or "qn_step" in r["Name"]:
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
}
run b512 && run b1024 WFSA_IBLOCK=1024 && run b512x WFSA_IPERCU=1 || exit 1
