"""Diagnostic: first Run of a fresh learner vs its second Run, after k steps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

syn = W.Synthetic(n_states=256, degree=8, vocab=16, emissions=1, n_strings=40_000, max_len=64, seed=4)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
if os.environ.get("COMPILED_ONLY"):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_fullsize import _compiled_only  # noqa: E402
    sym, off, wt = _compiled_only(W, fsa, sym, off, wt)
    print("compiled strings only:", len(wt))
for k in [int(a) for a in sys.argv[1:]] or [1, 2, 3, 4, 6]:
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(False)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    res = []
    for _ in range(2):
        lrn.Init(7)
        rows = np.array(lrn.Run(k, 1.0, -1.0))
        res.append((rows, lrn.x(), lrn.last_grad()))
    dx = np.flatnonzero(res[0][1] != res[1][1])
    dg = np.flatnonzero(res[0][2] != res[1][2])
    print(f"k={k}: rows equal {np.array_equal(res[0][0], res[1][0])}, x differs at {dx[:8]}, grad differs at {dg[:8]}",
          "grad", res[0][2][dg[:3]], res[1][2][dg[:3]])
    del lrn
