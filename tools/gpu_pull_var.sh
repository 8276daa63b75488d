#!/bin/bash
# famB per-evaluation time for the release library and the layout variants under w-fsa_amd/build_var (GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/pullvar
for v in release $(ls w-fsa_amd/build_var); do
  lib=w-fsa_amd/build_var/$v/libwfsa_amd.so; [ $v = release ] && lib=w-fsa_amd/wfsa_amd/libwfsa_amd.so
  WFSA_LIB=$R/$lib timeout -k 10 200 python -u tools/time_famb.py > gpurun_out/pullvar/$v.log 2>&1 || { tail gpurun_out/pullvar/$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pullvar/$v.log)"
done
