# round 4: stream-format micro v4 (+ LDS / fetch counters), then the dense path on both GEMM engines
set -o pipefail
mkdir -p gpurun_out/r4m
timeout -k 10 120 tools/micro/stream_v4 > gpurun_out/r4m/stream_v4.txt 2>&1 || { cat gpurun_out/r4m/stream_v4.txt; exit 1; }
cat gpurun_out/r4m/stream_v4.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/r4m/pmc1 -o run -- tools/micro/stream_v4 > gpurun_out/r4m/pmc1.log 2>&1 || { tail -20 gpurun_out/r4m/pmc1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4m/pmc2 -o run -- tools/micro/stream_v4 > gpurun_out/r4m/pmc2.log 2>&1 || { tail -20 gpurun_out/r4m/pmc2.log; exit 1; }
bash tools/gpu_r4_dense.sh
