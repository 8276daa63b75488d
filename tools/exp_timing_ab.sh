#!/bin/bash
# A/B of the per-step timing markers' cost in the device QN loop (c3 bench,
# no sub-records): markers off, every 4th step, every 16th (the default).
set -o pipefail
mkdir -p gpurun_out/tab
for i in 1 2 3; do
  for v in off s4 s16; do
    case $v in off) env="WFSA_TIMING=0";; s4) env="WFSA_TIMING_STRIDE=4";; s16) env="WFSA_TIMING_STRIDE=16";; esac
    env $env timeout -k 10 180 python -u bench.py --no-sub --cpu-sample 0 --boundary-steps 0 --steps 400 > gpurun_out/tab/${v}_$i.json 2>gpurun_out/tab/${v}_$i.err || exit 1
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/tab/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d["roofline"]
    print(f, round(d["ms_per_step"]*1000,2), "us/step", round(r["kernel_ms_per_launch"]*1000,2), "us fbs", r["timed_launches"], "timed")
PY
