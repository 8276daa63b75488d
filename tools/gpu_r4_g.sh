# round 4: counters of the stream kernel (16-bit vs delta format) and of the hand-written dense GEMMs
set -o pipefail
mkdir -p gpurun_out/r4g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4g/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/r4g/counters.txt | sort -u > gpurun_out/r4g/sq_counters.txt || true
wc -l gpurun_out/r4g/sq_counters.txt
pass() {   # name pmc-list env...
  local n=$1 c=$2; shift 2
  env "$@" BL_REPS=1 BL_STEPS=30 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r4g/$n -o run -- python tools/bench_like.py > gpurun_out/r4g/$n.log 2>&1 || { tail -5 gpurun_out/r4g/$n.log; return 1; }
}
for fmt in 0 1; do
  pass f$fmt "FETCH_SIZE" WFSA_DELTA=$fmt || exit 1
  pass s$fmt "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY" WFSA_DELTA=$fmt || exit 1
done
python tools/pmc_summary.py gpurun_out/r4g fbs_kernel
M=$(grep -o "SQ_VALU_MFMA_BUSY_CYCLES\|SQ_INSTS_VALU_MFMA_F64\|SQ_INSTS_MFMA" gpurun_out/r4g/sq_counters.txt | sort -u | tr '\n' ' ')
echo "mfma counters: $M"
WFSA_DENSE_BLAS=0 TD_EVALS=1 timeout -s KILL 180 rocprofv3 --pmc $M SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY --output-format csv -d gpurun_out/r4g/gemm -o run -- python tools/time_dense.py > gpurun_out/r4g/gemm.log 2>&1 || { tail -5 gpurun_out/r4g/gemm.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4g dense_gemm
