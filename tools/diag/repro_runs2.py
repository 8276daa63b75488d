"""Diagnostic: is only the very first Run different?  (tier counts printed)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

syn = W.Synthetic(n_states=256, degree=8, vocab=16, emissions=1, n_strings=40_000, max_len=64, seed=4)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
lrn = W.QuasiNewtonLearner(0)
lrn.set_info_rmin(False)
lrn.BuildFromPacked(fsa, sym, off, wt)
lrn.Finalize()
print("stats", {k: v for k, v in lrn.stats().items()
                if k in ("n_bubbles", "compiled_strings", "fallback_strings", "tier1_strings")})
sweeps = []
for sw in range(2):
    xs = []
    for n in (20, 7, 20):
        lrn.Init(7)
        rows = np.array(lrn.Run(n, 1.0, -1.0))
        xs.append((rows, lrn.x()))
    sweeps.append(xs)
for i, n in enumerate((20, 7, 20)):
    for sw in range(2):
        a, b = sweeps[sw][i], sweeps[0][0]
        m = min(len(a[0]), len(b[0]))
        d = sorted(set(int(j) for j in np.argwhere(a[0][:m] != b[0][:m])[:, 0]))
        print(f"sweep {sw} run {i} (n={n}) vs first run: differing steps {d}")
