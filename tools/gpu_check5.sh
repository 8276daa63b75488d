set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 180 tools/micro/chain_walk > gpurun_out/c5/chain_walk.txt 2>&1 || { cat gpurun_out/c5/chain_walk.txt; exit 1; }
cat gpurun_out/c5/chain_walk.txt
timeout -k 10 600 python -u tools/mp_bench.py > gpurun_out/c5/mp.txt 2> gpurun_out/c5/mp.err || { tail -30 gpurun_out/c5/mp.err; exit 1; }
cat gpurun_out/c5/mp.txt
