#!/bin/bash
# QN step experiments: WFSA_QN_DBG=1 returns after the flags (launch + dispatch cost only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for d in ${QN_DBGS:-0 1}; do
  WFSA_VERBOSE=1 WFSA_QN_DBG=$d timeout -k 10 120 python -u bench.py --cpu-sample 0 > gpurun_out/qn_$d.json 2>gpurun_out/qn_$d.err || { tail gpurun_out/qn_$d.err; exit 1; }
  grep "slots per" gpurun_out/qn_$d.err | head -2
  python -c "import json,sys; d=json.load(open('gpurun_out/qn_$d.json')); print('dbg', $d, 'ms/step', round(d['ms_per_step']*1e3,2), 'us; fbs', round(d['roofline']['kernel_ms_per_launch']*1e3,2))"
done
