#!/bin/bash
# bench.py's headline alone (no sub-benches, no CPU sample) under several
# environment settings, round-robin over REPS rounds (so a drifting box
# shifts every setting alike); one line per run, then each setting's best.
# Usage: bash tools/sweep_env.sh [--steps K] [--reps N] [--workload W] name:ENV=V,ENV=V name2: ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/sweep
mkdir -p "$O"
ARGS=()
REPS=1
while [ "${1:0:2}" = "--" ]; do
    case $1 in
    --steps) ARGS=(--steps "$2" --warmup 5); shift 2 ;;
    --reps) REPS=$2; shift 2 ;;
    --workload) ARGS+=(--workload "$2"); shift 2 ;;
    *) echo "unknown option $1"; exit 2 ;;
    esac
done
for rep in $(seq 1 "$REPS"); do
    for spec in "$@"; do
        name=${spec%%:*}
        envs=${spec#*:}
        (
            IFS=',' read -ra kv <<< "$envs"
            for e in "${kv[@]}"; do [ -n "$e" ] && export "${e?}"; done
            timeout -k 10 300 python -u bench.py --no-sub --cpu-sample 0 --boundary-steps 0 "${ARGS[@]}" \
                > "$O/$name.$rep.json" 2> "$O/$name.$rep.err"
        ) || { echo "$name failed"; tail -5 "$O/$name.$rep.err"; exit 1; }
        python - "$O/$name.$rep.json" "$name" "$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(f"{sys.argv[2]:<16} rep {sys.argv[3]} {d['ms_per_step'] * 1e3:7.2f} us/step  stream kernel "
      f"{1e3 * (r.get('kernel_ms_per_launch') or 0):6.2f} us  frac {r.get('frac') or 0:.3f}", flush=True)
PY
    done
done
python - "$O" "$@" <<'PY'
import glob, json, os, sys
print("best of each setting:")
for spec in sys.argv[2:]:
    name = spec.split(":")[0]
    v = []
    for f in glob.glob(os.path.join(sys.argv[1], name + ".*.json")):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
            v.append((d["ms_per_step"] * 1e3, 1e3 * (d.get("roofline", {}).get("kernel_ms_per_launch") or 0)))
        except Exception:  # noqa: BLE001
            pass
    if v:
        v.sort()
        print(f"  {name:<16} {v[0][0]:7.2f} us/step (median {v[len(v) // 2][0]:.2f}, n {len(v)})  kernel {v[0][1]:.2f} us")
PY
