# round 4: every GPU test (no -x: one run shows every failure), then smoke
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread --durations=20 > gpurun_out/r4/tests.log 2>&1
rc=$?
tail -40 gpurun_out/r4/tests.log
exit $rc
