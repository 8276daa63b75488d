# famB evaluation time: release pull kernel vs backward/forward unroll variants (make var)
set -o pipefail
mkdir -p gpurun_out/ub
for i in 1 2; do
  for v in release ub3 ub4 uf6; do
    if [ $v = release ]; then L=""; else L=w-fsa_amd/build_var/$v/libwfsa_amd.so; fi
    echo -n "$v " >> gpurun_out/ub/res.txt
    WFSA_LIB=$L timeout -k 10 200 python -u tools/time_famb.py >> gpurun_out/ub/res.txt 2>&1 || exit 1
  done
done
cat gpurun_out/ub/res.txt
