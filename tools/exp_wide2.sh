#!/bin/bash
# wide2 time breakdown on famB: full, no backward, no edge loops, neither (results wrong except 0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
for d in 0 1 2 3; do
  WFSA_W2_DBG=$d timeout -k 10 200 python -u tools/time_famb.py || exit 1
done
