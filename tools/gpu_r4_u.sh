# round 4: the LDS-DMA engine's step GEMMs with raised MFMA priority (and the register-staged gradient GEMM) against the
# split-K default; the delta stream micro at 32 waves per CU
set -o pipefail
mkdir -p gpurun_out/r4u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" TD_EVALS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4u/$n -o run -- python tools/time_dense.py > gpurun_out/r4u/$n.log 2>&1 || { tail -20 gpurun_out/r4u/$n.log; return 1; }
  echo "== $n: $(grep eval gpurun_out/r4u/$n.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4u/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
tot = 0.0
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("gemm", "mm_kernel", "Cijk", "epi", "reduce", "scatter", "transpose", "weights")):
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
}
run split && run dma WFSA_DENSE_ENGINE=dma && run dmaprio WFSA_DENSE_ENGINE=dma WFSA_LIB=w-fsa_amd/build_var/mmprio/libwfsa_amd.so || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -k dma -x -q --timeout 120 --timeout-method thread > gpurun_out/r4u/dma_tests.log 2>&1 || { tail -30 gpurun_out/r4u/dma_tests.log; exit 1; }
tail -1 gpurun_out/r4u/dma_tests.log
bash tools/gpu_r4_t.sh
