# round 4: split-K RAW GEMM engine -- dense tests on the three engines, then the c5 evaluation per engine
set -o pipefail
mkdir -p gpurun_out/r4n
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -v -x --timeout 180 --timeout-method thread > gpurun_out/r4n/dense_tests.log 2>&1 || { tail -30 gpurun_out/r4n/dense_tests.log; exit 1; }
tail -2 gpurun_out/r4n/dense_tests.log
run() {   # name, env...
  local n=$1; shift
  env "$@" TD_EVALS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n/$n -o run -- python tools/time_dense.py > gpurun_out/r4n/$n.log 2>&1 || { tail -20 gpurun_out/r4n/$n.log; return 1; }
  echo "== $n: $(grep eval gpurun_out/r4n/$n.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4n/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("gemm", "Cijk", "epi", "transpose", "scatter")):
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
}
run split WFSA_DENSE_ENGINE=split && run blas WFSA_DENSE_ENGINE=blas && run fused WFSA_DENSE_ENGINE=fused || exit 1
