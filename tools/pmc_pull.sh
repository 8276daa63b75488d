#!/bin/bash
# PMC counters of wave_pull_kernel on the famB workload (GPU box), one rocprofv3 pass per counter set;
# the kernel's launches of tools/time_famb.py (7 evaluations), summed over XCDs, averaged per launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/pmcpull"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex wave_pull --output-format csv -d "$O/p$i" -o run -- \
     python3 "$R/tools/time_famb.py" > "$O/p$i.log" 2>&1 || { tail -5 "$O/p$i.log"; exit 1; }
  echo "pass $i done"
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wave_pull_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
for k, d in sorted(acc.items()):
    v = list(d.values())
    print(f"{k:32s} {sum(v) / len(v):16.4g} per launch ({len(v)} launches)")
PY
