# round 4: the delta stream pass at 32 waves per CU (two 1024-thread blocks, 64-VGPR budget) against 16 (the micro)
set -o pipefail
mkdir -p gpurun_out/r4t
timeout -k 10 180 tools/micro/stream_v4 > gpurun_out/r4t/occ1.txt 2>&1 || { tail -5 gpurun_out/r4t/occ1.txt; exit 1; }
grep -E "delta 10" gpurun_out/r4t/occ1.txt
STREAM_WAVES=8192 timeout -k 10 180 tools/micro/stream_v4 > gpurun_out/r4t/occ2.txt 2>&1 || { tail -5 gpurun_out/r4t/occ2.txt; exit 1; }
grep -E "delta" gpurun_out/r4t/occ2.txt
