# round 4: delta pass prefetch depth A/B (rocprof kernel averages over bench_like), 16-bit for reference; streaming rate by footprint
set -o pipefail
mkdir -p gpurun_out/r4e
timeout -k 10 120 tools/micro/stream_bw > gpurun_out/r4e/stream_bw.txt 2>&1 || { cat gpurun_out/r4e/stream_bw.txt; exit 1; }
cat gpurun_out/r4e/stream_bw.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" BL_REPS=3 BL_STEPS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4e/$n -o run -- python tools/bench_like.py > gpurun_out/r4e/$n.log 2>&1 || { tail -20 gpurun_out/r4e/$n.log; return 1; }
  echo "== $n: $(grep rep gpurun_out/r4e/$n.log | tr '\n' ' ')"
  grep -h "fbs_kernel\|qn_step" $(find gpurun_out/r4e/$n -name "*kernel_stats.csv") | cut -d, -f1-4
}
run d2 WFSA_DELTA=1 && run d3 WFSA_LIB=w-fsa_amd/build_var/d3/libwfsa_amd.so && run d4 WFSA_LIB=w-fsa_amd/build_var/d4/libwfsa_amd.so && run b16 WFSA_DELTA=0 || exit 1

# dense A/B
mkdir -p gpurun_out/r4f
run() {   # name, env...
  local n=$1; shift
  env "$@" TD_EVALS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f/$n -o run -- python tools/time_dense.py > gpurun_out/r4f/$n.log 2>&1 || { tail -20 gpurun_out/r4f/$n.log; return 1; }
  echo "== $n: $(grep eval gpurun_out/r4f/$n.log | tr '\n' ' ')"
  grep -h "gemm\|Cijk\|rocblas" $(find gpurun_out/r4f/$n -name "*kernel_stats.csv") | cut -d, -f1-4 | head -6
}
run mid WFSA_DENSE_BLAS=0 && run end WFSA_DENSE_BLAS=0 WFSA_LIB=w-fsa_amd/build_var/gend/libwfsa_amd.so && run blas WFSA_DENSE_BLAS=1
