# round 4: family B pull kernel -- cross-step entry prefetch and the register budget (1024 vs 768-thread blocks), A/B
set -o pipefail
mkdir -p gpurun_out/r4o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4o/$n -o run -- python tools/time_famb.py > gpurun_out/r4o/$n.log 2>&1 || { tail -20 gpurun_out/r4o/$n.log; return 1; }
  echo "== $n: $(grep evaluation gpurun_out/r4o/$n.log)"
  python - $(find gpurun_out/r4o/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pull" in r["Name"]:
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "min", round(float(r["MinNs"]) / 1e3, 1))
PY
}
run pf && run nopf WFSA_LIB=w-fsa_amd/build_var/nopf/libwfsa_amd.so && run b768 WFSA_LIB=w-fsa_amd/build_var/b768/libwfsa_amd.so && run b768nopf WFSA_LIB=w-fsa_amd/build_var/b768nopf/libwfsa_amd.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier2.py tests/test_gpu_dense.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r4o/tests.log 2>&1 || { tail -30 gpurun_out/r4o/tests.log; exit 1; }
tail -2 gpurun_out/r4o/tests.log
