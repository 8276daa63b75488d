# round 4: dense epilogue / reduction batch sizes 4 / 8 (default) against 8 / 16, c5 bench record for each
set -o pipefail
mkdir -p gpurun_out/r4w
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in def eb8; do
  lib=""; [ $v = eb8 ] && lib="WFSA_LIB=w-fsa_amd/build_var/eb8/libwfsa_amd.so"
  env $lib timeout -k 10 300 python -u bench.py --workload c5 --cpu-sample 0 --boundary-steps 0 > gpurun_out/r4w/c5_$v.json 2> gpurun_out/r4w/c5_$v.err || { tail -20 gpurun_out/r4w/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4w/c5_$v.json'));r=d['roofline'];print('$v c5', round(d['value'],1), 'strings/s', round(r['evaluation_ms'],1), 'ms/eval', 'frac', round(r['frac'],3))"
done
