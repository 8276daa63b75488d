"""Diagnostic: identical device QN runs, where do they differ?"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W
syn = W.Synthetic(n_states=256, degree=8, vocab=16, emissions=1, n_strings=40_000, max_len=64, seed=4)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
lrn = W.QuasiNewtonLearner(0)
lrn.set_info_rmin(False)
lrn.BuildFromPacked(fsa, sym, off, wt)
lrn.Finalize()
runs = []
for _ in range(4):
    lrn.Init(7)
    rows = np.array(lrn.Run(20, 1.0, -1.0))
    runs.append((rows, lrn.x(), lrn.last_grad()))
for r in range(1, 4):
    d = runs[r][0] != runs[0][0]
    steps = sorted(set(int(i) for i in np.argwhere(d)[:, 0]))
    rel = np.max(np.abs(runs[r][0] - runs[0][0]) / np.maximum(np.abs(runs[0][0]), 1e-300))
    print(os.environ.get("WFSA_FIN_HOST", "1"), "run", r, "vs 0: steps", steps, "max rel", rel,
          "x differs", int((runs[r][1] != runs[0][1]).sum()))
