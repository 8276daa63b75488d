# round 4: the dense epilogues and gamma reduction with batched loads -- dense tests, the c5 evaluation's kernels, the c5 bench record
set -o pipefail
mkdir -p gpurun_out/r4v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4v/dense_tests.log 2>&1 || { tail -30 gpurun_out/r4v/dense_tests.log; exit 1; }
tail -1 gpurun_out/r4v/dense_tests.log
TD_EVALS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4v/split -o run -- python tools/time_dense.py > gpurun_out/r4v/split.log 2>&1 || { tail -20 gpurun_out/r4v/split.log; exit 1; }
grep eval gpurun_out/r4v/split.log | tr '\n' ' '; echo
python - $(find gpurun_out/r4v/split -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("gemm", "epi", "reduce")):
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
timeout -k 10 300 python -u bench.py --workload c5 --cpu-sample 0 --boundary-steps 0 > gpurun_out/r4v/c5.json 2> gpurun_out/r4v/c5.err || { tail -20 gpurun_out/r4v/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4v/c5.json'));r=d['roofline'];print('c5', round(d['value'],1), 'strings/s', round(r['evaluation_ms'],1), 'ms/eval', 'frac', round(r['frac'],3))"
TD_EVALS=2 WFSA_LIB=w-fsa_amd/build_var/gsuper/libwfsa_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4v/gsuper -o run -- python tools/time_dense.py > gpurun_out/r4v/gsuper.log 2>&1 || { tail -20 gpurun_out/r4v/gsuper.log; exit 1; }
echo "== gsuper: $(grep eval gpurun_out/r4v/gsuper.log | tr '\n' ' ')"
python - $(find gpurun_out/r4v/gsuper -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm" in r["Name"]:
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
