# round 4: the stream kernel timed by events attached to its dispatch -- every GPU test, the bench's kernel time vs rocprof's
set -o pipefail
O=gpurun_out/r4ev
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 50 --warmup 10 --cpu-sample 0 --no-sub --boundary-steps 0 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python - $(find $O/prof -name "*kernel_stats.csv") <<'PY'
import csv, json, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fbs_kernel" in r["Name"] and r["Name"].endswith("true>(wfsa::CompiledArgs)") or ("fbs_kernel<false, true, false, 0, false, true>" in r["Name"]):
        print("rocprof", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
d = json.load(open("gpurun_out/r4ev/prof.json"))
print("bench events", round(d["roofline"]["kernel_ms_per_launch"] * 1e3, 2), "us, frac", round(d["roofline"]["frac"], 3))
PY
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4ev/bench_default.json'));r=d['roofline'];print('default', round(d['value']/1e9,2), 'G strings/s', round(d['ms_per_step']*1e3,2), 'us/step; events', round(r['kernel_ms_per_launch']*1e3,2), 'us, frac', round(r['frac'],3), '; c5', round(d['dense_c5']['roofline']['frac'],3))"
