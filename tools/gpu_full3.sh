# round-3 evidence, in two calls (each under gpurun's 1200 s limit):
#   bash tools/gpu_full3.sh tests   -- every GPU test
#   bash tools/gpu_full3.sh bench   -- driver-like bench, rocprof kernel trace + PMC passes
set -o pipefail
mkdir -p gpurun_out/full3
case "$1" in
tests)
    timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/full3/tests.log 2>&1 || { tail -60 gpurun_out/full3/tests.log; exit 1; }
    grep -cE "PASSED" gpurun_out/full3/tests.log; tail -2 gpurun_out/full3/tests.log
    ;;
bench)
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 10 > gpurun_out/full3/bench.json 2> gpurun_out/full3/bench.err || { tail -20 gpurun_out/full3/bench.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/full3/bench.json'))
print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'], 'rmin', d['info_rmin']['ms_per_step'])
print('cpu', d['cpu_baseline']['value'], d['ll_rel_err_vs_reference_algorithm'])
for k in ('dense_c5','famB'): print(k, d[k].get('value'), d[k].get('ms_per_step'), d[k].get('roofline',{}).get('frac'))
"
    bash tools/profile.sh gpurun_out/full3/prof --no-sub --cpu-sample 0 --boundary-steps 0 --steps 50 --warmup 5 || exit 1
    find gpurun_out/full3/prof/trace -name "*kernel_stats.csv" | head -1 | xargs head -8
    ;;
*) echo "usage: $0 tests|bench"; exit 2 ;;
esac
