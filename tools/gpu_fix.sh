# A/B: the wave kernel's fixed-point conversion (release: magic-number add;
# variant rint: the emulated double -> int64 conversion), famB evaluation time
set -o pipefail
mkdir -p gpurun_out/fix
for i in 1 2; do
  timeout -k 10 200 python -u tools/time_famb.py >> gpurun_out/fix/new.log 2>&1 || exit 1
  WFSA_LIB=w-fsa_amd/build_var/rint/libwfsa_amd.so timeout -k 10 200 python -u tools/time_famb.py >> gpurun_out/fix/rint.log 2>&1 || exit 1
done
echo new; cat gpurun_out/fix/new.log; echo rint; cat gpurun_out/fix/rint.log
