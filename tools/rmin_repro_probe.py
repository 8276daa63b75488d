"""Which path produced each rmin value of a device-loop run (diagnostic):
the fused per-bubble values, or the separate pass the host steps use."""
import sys

import numpy as np

sys.path.insert(0, "w-fsa_amd")
sys.path.insert(0, ".")
import wfsa_amd as W  # noqa: E402

syn = W.Synthetic(n_states=64, degree=8, vocab=16, emissions=1, n_strings=3000, max_len=64, seed=5)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)


def learner():
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(True)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    return lrn


host = learner()
hrows = np.array([host.OptimizationStep(1.0, -1.0)[0] for _ in range(6)])
print("host ", [f"{v:.17g}" for v in hrows[:, 5]], flush=True)
for k in range(4):
    r = np.array(learner().Run(6, 1.0, -1.0))
    print(f"run{k} ", [f"{v:.17g}" for v in r[:, 5]], flush=True)
