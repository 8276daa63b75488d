# round-3 end: every GPU test
set -o pipefail
mkdir -p gpurun_out/full3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread --durations=15 > gpurun_out/full3/tests.log 2>&1 || { tail -60 gpurun_out/full3/tests.log; exit 1; }
grep -cE "PASSED" gpurun_out/full3/tests.log; tail -20 gpurun_out/full3/tests.log
