"""HessianLearner on the c3 workload (1024-state family A, 1M
strings): n + k = 10,249 unknowns -- the KKT system factored in HBM
(rocSOLVER dsytrf + the dsytrs kernel), H_f from the compiled bubbles.
Prints the time of each Newton epoch and its info row (GPU box)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

n_strings = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=n_strings, max_len=128, seed=1)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
lrn = W.HessianLearner(0)
t = time.time()
lrn.BuildFromPacked(fsa, sym, off, wt)
lrn.Finalize()
inf = lrn.info()
print(f"build {time.time() - t:.2f} s; n = {inf['n_params']}, k = {inf['n_constraints']}", flush=True)
lrn.Init(31)
for e in range(3):
    t = time.time()
    row = lrn.OptimizationStep(1.0, -1.0)
    print(f"epoch {e + 1}: {time.time() - t:.3f} s  info {np.array2string(np.asarray(row[0] if isinstance(row, tuple) else row), precision=6)}",
          flush=True)
