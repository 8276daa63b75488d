#!/bin/bash
# PMC counters of the tier-2 wave kernel on the famB workload (GPU box), one pass per counter set
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/pmc2"
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex wide2 --output-format csv -d "$R/gpurun_out/pmc2/p$i" -o run -- \
     python3 "$R/bench.py" --workload famB --no-sub --cpu-sample 0 --boundary-steps 0 --steps 2 --warmup 1 > "$R/gpurun_out/pmc2/p$i.log" 2>&1 || { tail -5 "$R/gpurun_out/pmc2/p$i.log"; exit 1; }
done
python3 - "$R/gpurun_out/pmc2" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wide2_kernel<false>" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, "per launch", sum(v) / max(1, len(set(v)) and 1) / len(v) * 1.0, "n", len(v))
PY
