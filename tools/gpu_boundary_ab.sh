# A/B of the host-binding step: release vs w-fsa_amd/build_var/oldsync (GPU box)
set -o pipefail
mkdir -p gpurun_out/bab
for i in 1 2; do
  timeout -k 10 200 python -u tools/boundary_time.py >> gpurun_out/bab/res.txt 2>&1 || exit 1
  WFSA_LIB=w-fsa_amd/build_var/oldsync/libwfsa_amd.so timeout -k 10 200 python -u tools/boundary_time.py >> gpurun_out/bab/res.txt 2>&1 || exit 1
done
cat gpurun_out/bab/res.txt
