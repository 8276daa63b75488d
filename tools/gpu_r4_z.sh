# round 4: the QN step kernel's block size (128 / 256 default / 512 threads) re-checked on the final tree
set -o pipefail
mkdir -p gpurun_out/r4z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for nt in 256 128 512; do
  WFSA_QN_BLOCK=$nt BL_REPS=2 BL_STEPS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4z/q$nt -o run -- python tools/bench_like.py > gpurun_out/r4z/q$nt.log 2>&1 || { tail -20 gpurun_out/r4z/q$nt.log; exit 1; }
  echo "== $nt: $(grep rep gpurun_out/r4z/q$nt.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4z/q$nt -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "qn_step" in r["Name"] or "fbs_kernel" in r["Name"]:
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
done
