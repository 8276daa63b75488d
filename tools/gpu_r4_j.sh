# round 4: delta zero slots on distinct banks (period 511) -- parity, kernel A/B, counters; then the GEMM pitch A/B
set -o pipefail
mkdir -p gpurun_out/r4j
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r4j/tests.log 2>&1 || { tail -30 gpurun_out/r4j/tests.log; exit 1; }
tail -2 gpurun_out/r4j/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" BL_REPS=3 BL_STEPS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4j/$n -o run -- python tools/bench_like.py > gpurun_out/r4j/$n.log 2>&1 || { tail -20 gpurun_out/r4j/$n.log; return 1; }
  echo "== $n: $(grep rep gpurun_out/r4j/$n.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4j/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fbs_kernel" in r["Name"] or "qn_step" in r["Name"]:
        print(r["Name"].split("(wfsa")[0][-44:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "min", round(float(r["MinNs"]) / 1e3, 2))
PY
}
run delta WFSA_DELTA=1 && run b16 WFSA_DELTA=0 || exit 1
WFSA_DELTA=1 BL_REPS=1 BL_STEPS=30 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/r4j/pmc/s1 -o run -- python tools/bench_like.py > gpurun_out/r4j/pmc.log 2>&1 || { tail -5 gpurun_out/r4j/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4j/pmc fbs_kernel
bash tools/gpu_r4_i.sh
