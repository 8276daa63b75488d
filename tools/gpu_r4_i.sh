# round 4: GEMM KC operand pitch A/B (odd, the default now, vs round 3's even), dense tests on both engines
set -o pipefail
mkdir -p gpurun_out/r4i
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" TD_EVALS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i/$n -o run -- python tools/time_dense.py > gpurun_out/r4i/$n.log 2>&1 || { tail -20 gpurun_out/r4i/$n.log; return 1; }
  echo "== $n: $(grep eval gpurun_out/r4i/$n.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4i/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm" in r["Name"] or "Cijk" in r["Name"]:
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
}
run odd WFSA_DENSE_BLAS=0 && run even WFSA_DENSE_BLAS=0 WFSA_LIB=w-fsa_amd/build_var/ldkeven/libwfsa_amd.so || exit 1
run grad0 WFSA_DENSE_BLAS=0 WFSA_DENSE_GRAD_CFG=0 && run step2 WFSA_DENSE_BLAS=0 WFSA_DENSE_STEP_CFG=2 || exit 1
WFSA_DENSE_BLAS=0 TD_EVALS=1 timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY --output-format csv -d gpurun_out/r4i/pmc/odd -o run -- python tools/time_dense.py > gpurun_out/r4i/pmc.log 2>&1 || { tail -5 gpurun_out/r4i/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4i/pmc dense_gemm
timeout -k 10 500 python -u -m pytest tests/test_gpu_dense.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r4i/dense_tests.log 2>&1 || { tail -30 gpurun_out/r4i/dense_tests.log; exit 1; }
tail -2 gpurun_out/r4i/dense_tests.log
