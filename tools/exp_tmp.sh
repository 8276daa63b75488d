export TMPDIR=/tmp
for cfg in "0 0" "0 1" "1 1"; do set -- $cfg
  WFSA_BUBBLE_REG=$1 WFSA_BUBBLE_SKIPBIG=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bx/r$1s$2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 50 > $GRAFT_REPO_ROOT/gpurun_out/bx/r$1s$2.log 2>&1 || exit 1
  echo "reg=$1 skipbig=$2"; grep bubble_kernel $GRAFT_REPO_ROOT/gpurun_out/bx/r$1s$2/run_kernel_stats.csv | cut -d, -f3-5
done
