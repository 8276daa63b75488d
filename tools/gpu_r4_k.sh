# round 4: the first-Run slowdown (idle device before the warm-up?), every GPU test, the bench at the driver's setting and the default
set -o pipefail
mkdir -p gpurun_out/r4k
bl() { local n=$1; shift; env "$@" timeout -k 10 300 python -u tools/bench_like.py > gpurun_out/r4k/$n.log 2>&1 || { tail -5 gpurun_out/r4k/$n.log; return 1; }; echo "== $n ($*): $(grep rep gpurun_out/r4k/$n.log | tr '\n' ' ')"; }
bl plain BL_REPS=4 BL_STEPS=20 && bl presleep BL_PRESLEEP=1 BL_REPS=3 BL_STEPS=20 && bl presleep_warm200 BL_PRESLEEP=1 BL_WARM=200 BL_REPS=3 BL_STEPS=20 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/r4k/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4k/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh gpurun_out/r4k/prof --steps 50 --warmup 10 --cpu-sample 0 --no-sub --boundary-steps 0 || { echo "profile failed"; exit 1; }
python tools/traffic.py gpurun_out/r4k/prof profiles/traffic_latest.json && cat profiles/traffic_latest.json && cp profiles/traffic_latest.json gpurun_out/r4k/
timeout -k 10 600 python -u bench.py --steps 20 --warmup 10 > gpurun_out/r4k/bench_driver.json 2> gpurun_out/r4k/bench_driver.err || { tail -20 gpurun_out/r4k/bench_driver.err; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r4k/bench_default.json 2> gpurun_out/r4k/bench_default.err || { tail -20 gpurun_out/r4k/bench_default.err; exit 1; }
python - <<'PY'
import json
for n in ("bench_driver", "bench_default"):
    d = json.load(open(f"gpurun_out/r4k/{n}.json"))
    print(n, round(d["value"] / 1e9, 2), "G strings/s", round(d["ms_per_step"] * 1e3, 2), "us/step", "frac", round(d["roofline"]["frac"], 3),
          "boundary", round(d["boundary"]["ms_per_step"] * 1e3, 1) if d.get("boundary") else None,
          "c5", round(d["dense_c5"]["value"], 1) if d.get("dense_c5") else None, "famB", round(d["famB"]["value"] / 1e6, 2) if d.get("famB") else None)
PY
