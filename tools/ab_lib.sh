#!/bin/bash
# A/B of library builds on one box: tools/bench_like.py (the bench's timed
# Run, c3, 1M strings) under each library in turn, round-robin over REPS
# rounds so a drifting box shifts every build alike.
# Usage: bash tools/ab_lib.sh REPS name=path/libwfsa_amd.so [name=path ...]   (path "-": the in-tree library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
REPS=$1; shift
for rep in $(seq 1 "$REPS"); do
    for spec in "$@"; do
        name=${spec%%=*}; lib=${spec#*=}
        if [ "$lib" = "-" ]; then unset WFSA_LIB; else export WFSA_LIB=$R/$lib; fi
        out=$(BL_STEPS=${BL_STEPS:-200} BL_REPS=${BL_REPS:-3} timeout -k 10 300 python -u tools/bench_like.py 2>&1) \
            || { echo "$name failed"; echo "$out" | tail -5; exit 1; }
        echo "$name rep $rep: $(echo "$out" | grep 'us/step' | tr '\n' ' ')"
    done
done
