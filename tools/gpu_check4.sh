# stream-format micro, the full bench at the driver's setting, rocprof of the headline
set -o pipefail
mkdir -p gpurun_out/c4
timeout -k 10 120 tools/micro/chain_walk > gpurun_out/c4/chain_walk.txt 2>&1 || { cat gpurun_out/c4/chain_walk.txt; exit 1; }
cat gpurun_out/c4/chain_walk.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 10 > gpurun_out/c4/bench.json 2> gpurun_out/c4/bench.err || { tail -20 gpurun_out/c4/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c4/bench.json'))
print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'], 'rmin', d['info_rmin']['ms_per_step'])
print('boundary', d['boundary']['ms_per_step'], d['boundary']['host_ms_per_step'])
for k in ('dense_c5','famB'): print(k, d[k].get('value'), d[k].get('ms_per_step'), d[k].get('roofline',{}).get('frac'))
"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/c4/prof" -o run -- python3 bench.py --no-sub --cpu-sample 0 --boundary-steps 0 --steps 200 > gpurun_out/c4/prof.log 2>&1 || { tail gpurun_out/c4/prof.log; exit 1; }
find gpurun_out/c4/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
