"""Prints the info rows of the in-kernel and the separate QN update over the
sequence tests/test_gpu_qn_inkernel.py runs (diagnostics)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=200_000, max_len=128, seed=1)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)


def mk(v):
    os.environ["WFSA_QN_INKERNEL"] = v
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(False)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    return lrn


a, b = mk("1"), mk("0")
for rep in range(int(os.environ.get("QD_REPS", "1"))):
    a.Init(7)
    b.Init(7)
    ra = np.array(a.Run(3, 1.0, -1.0) + a.Run(4, 1.0, -1.0) + a.Run(1, 1.0, -1.0) + a.Run(12, 1.0, -1.0))
    rb = np.array(b.Run(20, 1.0, -1.0))
    d = np.argwhere(ra != rb)
    print("rep", rep, "differing rows:", sorted(set(int(r) for r, _ in d)), "zero rows a:",
          [i for i in range(len(ra)) if not ra[i].any()], "b:", [i for i in range(len(rb)) if not rb[i].any()], flush=True)
a.Run(1, 1.0, -1.0)
b.Run(1, 1.0, -1.0)
a.Init(7)
b.Init(7)
ra = np.array(a.Run(3, 1.0, -1.0) + a.Run(4, 1.0, -1.0) + a.Run(1, 1.0, -1.0) + a.Run(12, 1.0, -1.0))
rb = np.array(b.Run(20, 1.0, -1.0))
np.set_printoptions(precision=17, linewidth=220)
d = np.argwhere(ra != rb)
print("differing (row, col):", d.tolist())
for r, c in d[:10]:
    print(r, c, ra[r, c], rb[r, c])
print("x equal", np.array_equal(a.x(), b.x()))
