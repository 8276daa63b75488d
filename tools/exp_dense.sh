#!/bin/bash
# Timing experiments of the dense path (GPU box): bench c5 under each
# environment setting given as an argument (e.g. WFSA_DENSE_GRAD_CFG=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/exp
i=0
for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python -u bench.py --workload c5 --steps 4 --warmup 1 --cpu-sample 0 > gpurun_out/exp/$i.json 2> gpurun_out/exp/$i.err || { tail gpurun_out/exp/$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/exp/$i.json')); r=d['roofline']; print('$cfg', round(d['value'],1), 'strings/s', round(r['achieved'],2), 'TF', round(r['evaluation_ms'],2), 'ms')"
done
