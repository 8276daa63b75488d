# round 4: split-K RAW GEMM variants -- next-slice store mid-slice (default) vs at the slice end, K slices of 16 (2 blocks/CU) vs 32 (1 block/CU)
set -o pipefail
mkdir -p gpurun_out/r4p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {   # name, env...
  local n=$1; shift
  env "$@" TD_EVALS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p/$n -o run -- python tools/time_dense.py > gpurun_out/r4p/$n.log 2>&1 || { tail -20 gpurun_out/r4p/$n.log; return 1; }
  echo "== $n: $(grep eval gpurun_out/r4p/$n.log | tr '\n' ' ')"
  python - $(find gpurun_out/r4p/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("gemm", "epi")):
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -k dma -x -q --timeout 120 --timeout-method thread > gpurun_out/r4p/dma_tests.log 2>&1 || { tail -30 gpurun_out/r4p/dma_tests.log; exit 1; }
tail -2 gpurun_out/r4p/dma_tests.log
run dma WFSA_DENSE_ENGINE=dma && run mid && run end WFSA_LIB=w-fsa_amd/build_var/gend/libwfsa_amd.so && run bk32 WFSA_DENSE_STEP_CFG=3 && run frag WFSA_LIB=w-fsa_amd/build_var/gfrag/libwfsa_amd.so && run prio WFSA_LIB=w-fsa_amd/build_var/gprio/libwfsa_amd.so || exit 1
# counters of the RAW GEMM (one evaluation)
TD_EVALS=1 timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r4p/pmc -o run -- python tools/time_dense.py > gpurun_out/r4p/pmc.log 2>&1 || { tail -5 gpurun_out/r4p/pmc.log; exit 1; }
python tools/pmc_summary.py gpurun_out/r4p/pmc dense_gemm
# family B: the next step's source alpha loaded a step early too (variant avpf) vs the default
famb() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p/$n -o run -- python tools/time_famb.py > gpurun_out/r4p/$n.log 2>&1 || { tail -20 gpurun_out/r4p/$n.log; return 1; }
  echo "== $n: $(grep evaluation gpurun_out/r4p/$n.log)"
  python - $(find gpurun_out/r4p/$n -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "wave_pull" in r["Name"]:
        print(r["Name"][:64], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "min", round(float(r["MinNs"]) / 1e3, 1))
PY
}
famb fb_pf && famb fb_avpf WFSA_LIB=w-fsa_amd/build_var/avpf/libwfsa_amd.so || exit 1
bash tools/gpu_r4_q.sh
# the QN loop's Run prologue / tail changes: pipe and parity tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r4p/pipe_tests.log 2>&1 || { tail -30 gpurun_out/r4p/pipe_tests.log; exit 1; }
tail -2 gpurun_out/r4p/pipe_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4p/drv$i.json 2> gpurun_out/r4p/drv$i.err || { tail -20 gpurun_out/r4p/drv$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4p/drv$i.json'));print('driver setting', $i, round(d['ms_per_step']*1e3,2), 'us/step')"
done
timeout -k 10 300 python -u bench.py --cpu-sample 0 --boundary-steps 0 --no-sub > gpurun_out/r4p/d200.json 2> gpurun_out/r4p/d200.err || { tail -20 gpurun_out/r4p/d200.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4p/d200.json'));print('200 steps', round(d['ms_per_step']*1e3,2), 'us/step')"
