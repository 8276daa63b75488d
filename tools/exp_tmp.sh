# timing experiments: avg kernel durations per configuration
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT/gpurun_out/ex
mkdir -p $R
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 40 > $R/$name.log 2>&1 || return 1
  python3 - $R/$name/run_kernel_stats.csv $name <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'fbs_kernel' in n or 'bubble_kernel' in n:
        print(f"{sys.argv[2]:24s} {n[:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:7.1f} us")
PY
  grep -o '"value": [0-9.]*' $R/$name.log
}
run f0 A=1 && run d5 WFSA_FBS_DBG=5 && run nf0 WFSA_FUSE_BUBBLES=0 WFSA_SMALL_COST=0 WFSA_BIG_COST=0 && run nf3 WFSA_FBS_DBG=3 WFSA_FUSE_BUBBLES=0
