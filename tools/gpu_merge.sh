#!/bin/bash
# wave-merged bubble slots: every GPU test, then c3 with the merge on and off (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/merge; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in 1 0 1; do
  WFSA_SLOT_MERGE=$m timeout -k 10 300 python -u bench.py --no-sub --cpu-sample 0 --boundary-steps 0 --steps 200 --warmup 20 > $O/c3_$m.json 2> $O/c3_$m.err || { tail $O/c3_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$m.json')); print('merge=$m', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step, fbs', round(d['roofline']['kernel_ms_per_launch']*1e3,2), 'us, rmin', round(d['info_rmin']['ms_per_step']*1e3,2))"
done
WFSA_SLOT_MERGE=1 timeout -k 10 200 python -u tools/slot_stats.py > $O/slots1.log 2>&1 && tail -1 $O/slots1.log
WFSA_SLOT_MERGE=0 timeout -k 10 200 python -u tools/slot_stats.py > $O/slots0.log 2>&1 && tail -1 $O/slots0.log
