# round 4: streaming rate by footprint (Infinity Cache), counter list, GEMM counters on c5 (hand-written kernels)
set -o pipefail
mkdir -p gpurun_out/r4d2
timeout -k 10 120 tools/micro/stream_bw > gpurun_out/r4d2/stream_bw.txt 2>&1 || { cat gpurun_out/r4d2/stream_bw.txt; exit 1; }
cat gpurun_out/r4d2/stream_bw.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4d2/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*\|SQ_INSTS_VALU_MFMA[A-Z0-9_]*" gpurun_out/r4d2/counters.txt | sort -u | head -30
WFSA_DENSE_BLAS=0 timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r4d2/pmc_c5 -o run -- python bench.py --workload c5 --steps 1 --warmup 0 --cpu-sample 0 --boundary-steps 0 > gpurun_out/r4d2/pmc_c5.log 2>&1 || { tail -20 gpurun_out/r4d2/pmc_c5.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4d2 dense_gemm
