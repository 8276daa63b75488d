set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_rmin.py -q --timeout 120 --timeout-method thread > gpurun_out/rmin_tests.log 2>&1 || { tail -30 gpurun_out/rmin_tests.log; exit 1; }
tail -1 gpurun_out/rmin_tests.log
timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_rmin.json 2> gpurun_out/bench_rmin.err || { tail -20 gpurun_out/bench_rmin.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_rmin.json')); print(d['value'], d['ms_per_step'])"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/rmin" -o run -- \
    python3 "$R/bench.py" --cpu-sample 0 --steps 20 > "$R/gpurun_out/prof/rmin.log" 2>&1 || { tail -20 "$R/gpurun_out/prof/rmin.log"; exit 1; }
head -12 "$R/gpurun_out/prof/rmin/run_kernel_stats.csv" | cut -c1-160
