# round 4: dense epilogue / reduction reduction batch 16 (default) against 32 (time_dense kernels), and the c5 bench record
set -o pipefail
mkdir -p gpurun_out/r4w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in def rb32; do
  lib=""; [ $v = rb32 ] && lib="WFSA_LIB=w-fsa_amd/build_var/rb32/libwfsa_amd.so"
  env $lib TD_EVALS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4w/$v -o run -- python tools/time_dense.py > gpurun_out/r4w/$v.log 2>&1 || { tail -20 gpurun_out/r4w/$v.log; exit 1; }
  echo "== $v: $(grep eval gpurun_out/r4w/$v.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4w/$v -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("epi", "reduce")):
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
done
timeout -k 10 300 python -u bench.py --workload c5 --cpu-sample 0 --boundary-steps 0 > gpurun_out/r4w/c5.json 2> gpurun_out/r4w/c5.err || { tail -20 gpurun_out/r4w/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4w/c5.json'));r=d['roofline'];print('c5', round(d['value'],1), 'strings/s', round(r['evaluation_ms'],1), 'ms/eval', 'frac', round(r['frac'],3))"
