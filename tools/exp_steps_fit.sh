set -o pipefail
mkdir -p gpurun_out/sf
for s in 50 200 800; do
  timeout -k 10 180 python -u bench.py --no-sub --cpu-sample 0 --boundary-steps 0 --steps $s > gpurun_out/sf/s$s.json 2>gpurun_out/sf/s$s.err || exit 1
done
python - <<'PY'
import json
for s in (50,200,800):
    d=json.loads(open(f"gpurun_out/sf/s{s}.json").read().strip().splitlines()[-1])
    print(s, "steps:", round(d["ms_per_step"]*s,4), "ms total,", round(d["ms_per_step"]*1000,2), "us/step", "rmin", round(d["info_rmin"]["ms_per_step"]*1000,2))
PY
