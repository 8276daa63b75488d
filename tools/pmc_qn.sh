#!/bin/bash
# PMC pass over a short bench run (SQ wave/latency counters), per-kernel rows
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/pmcq"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/gpurun_out/pmcq/sq" -o run -- python3 "$R/bench.py" --cpu-sample 0 --steps 8 --warmup 2 > "$R/gpurun_out/pmcq/sq.log" 2>&1 || { tail "$R/gpurun_out/pmcq/sq.log"; exit 1; }
python3 - "$R/gpurun_out/pmcq/sq/run_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    n = max(cnt[(k, 'SQ_WAVES')], 1)
    print(k, {c: round(v / n) for c, v in d.items()})
PY
