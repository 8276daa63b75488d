# round 4: dense GEMM A/B (next-slice stores mid-slice vs at the slice end), rocBLAS for reference; kernel averages
set -o pipefail
mkdir -p gpurun_out/r4f
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" TD_EVALS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f/$n -o run -- python tools/time_dense.py > gpurun_out/r4f/$n.log 2>&1 || { tail -20 gpurun_out/r4f/$n.log; return 1; }
  echo "== $n: $(grep eval gpurun_out/r4f/$n.log | tr '\n' ' ')"
  grep -h "gemm\|Cijk\|rocblas" $(find gpurun_out/r4f/$n -name "*kernel_stats.csv") | cut -d, -f1-4 | head -6
}
run mid WFSA_DENSE_BLAS=0 && run end WFSA_DENSE_BLAS=0 WFSA_LIB=w-fsa_amd/build_var/gend/libwfsa_amd.so && run blas WFSA_DENSE_BLAS=1
