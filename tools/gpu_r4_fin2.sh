# round 4, last: the bench on the final tree -- the driver's setting and the default, with the sub-records; smoke
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python - <<'PY'
import json
for n in ("bench_driver", "bench_default"):
    d = json.load(open(f"gpurun_out/r4g/{n}.json"))
    g = lambda k, f: (f(d[k]) if isinstance(d.get(k), dict) and "value" in d[k] else d.get(k))
    print(n, round(d["value"] / 1e9, 2), "G strings/s", round(d["ms_per_step"] * 1e3, 2), "us/step", "frac", round(d["roofline"]["frac"], 3),
          "boundary", round(d["boundary"]["ms_per_step"] * 1e3, 1) if d.get("boundary") else None,
          "c5", g("dense_c5", lambda r: (round(r["value"], 1), round(r["roofline"]["frac"], 3))),
          "c5 rocblas", g("dense_c5_rocblas", lambda r: (round(r["value"], 1), round(r["roofline"]["frac"], 3))),
          "famB", g("famB", lambda r: round(r["value"] / 1e6, 2)))
PY
