"""Diagnostic: values of the first Run vs a later one, step by step."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

np.set_printoptions(precision=17, linewidth=200)
syn = W.Synthetic(n_states=256, degree=8, vocab=16, emissions=1, n_strings=40_000, max_len=64, seed=4)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
lrn = W.QuasiNewtonLearner(0)
lrn.set_info_rmin(False)
lrn.BuildFromPacked(fsa, sym, off, wt)
lrn.Finalize()
runs = []
for _ in range(2):
    lrn.Init(7)
    runs.append(np.array(lrn.Run(20, 1.0, -1.0)))
print("stats", {k: v for k, v in lrn.stats().items()
                if k in ("n_bubbles", "compiled_strings", "fallback_strings", "tier1_strings", "n_groups")})
for s in (5, 6, 7, 15, 16, 17):
    print("step", s)
    print("  run0", runs[0][s])
    print("  run1", runs[1][s])
