#!/bin/bash
# bench.py's headline alone (no sub-benches, no CPU sample) under several
# environment settings, one line each: name, us/step, stream-kernel us.
# Usage: bash tools/sweep_env.sh [--steps K] name:ENV=V,ENV=V name2: ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/sweep
mkdir -p "$O"
ARGS=()
if [ "$1" = "--steps" ]; then ARGS=(--steps "$2" --warmup 5); shift 2; fi
for spec in "$@"; do
    name=${spec%%:*}
    envs=${spec#*:}
    (
        IFS=',' read -ra kv <<< "$envs"
        for e in "${kv[@]}"; do [ -n "$e" ] && export "${e?}"; done
        timeout -k 10 300 python -u bench.py --no-sub --cpu-sample 0 --boundary-steps 0 "${ARGS[@]}" \
            > "$O/$name.json" 2> "$O/$name.err"
    ) || { echo "$name failed"; tail -5 "$O/$name.err"; exit 1; }
    python - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(f"{sys.argv[2]:<16} {d['ms_per_step'] * 1e3:7.2f} us/step  stream kernel {1e3 * (r.get('kernel_ms_per_launch') or 0):6.2f} us")
PY
done
