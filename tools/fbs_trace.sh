#!/bin/bash
# Per-wave timeline of the stream kernel (experiments library, WFSA_FBS_TRACE:
# s_memrealtime stamps per wave of the last launch of each Run -- entry,
# staged, bubbles done, arrived, stream done, QN poll matched, QN done, exit),
# and the c3 step time, for the settings given as "NAME:ENV=V,ENV=V" args.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/fbs_trace
mkdir -p "$OUT"
export WFSA_LIB=$R/w-fsa_amd/build_exp/libwfsa_amd.so WFSA_FBS_TRACE=1 BL_REPS=${BL_REPS:-2} BL_STEPS=${BL_STEPS:-50}
for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    [ "$envs" = "$spec" ] && envs=""
    ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 300 python3 "$R/tools/bench_like.py" > "$OUT/$name.log" 2>&1 ) || { tail -20 "$OUT/$name.log"; exit 1; }
    echo "== $name ($envs)"
    grep "^rep" "$OUT/$name.log" | tr '\n' ' '; echo
    grep "fbs-trace" "$OUT/$name.log" | tail -26
done
