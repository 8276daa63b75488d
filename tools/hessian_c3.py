"""HessianLearner on the c3 workload (1024-state family A, 1M
strings): n + k = 10,249 unknowns, H_f from the compiled bubbles.  The KKT
system through the sparse LDL^T (the default there) and through the dense
Bunch-Kaufman factorisation in HBM (WFSA_KKT=device); prints the time of each
Newton epoch and its info row for both (GPU box)."""
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
for kkt in ("sparse", "device"):
    os.environ["WFSA_KKT"] = kkt
    lrn = W.HessianLearner(0)
    t = time.time()
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    inf = lrn.info()
    print(f"[{kkt}] build {time.time() - t:.2f} s; n = {inf['n_params']}, k = {inf['n_constraints']}", flush=True)
    lrn.Init(31)
    for e in range(3):
        t = time.time()
        row = lrn.OptimizationStep(1.0, -1.0)
        row = np.asarray(row[0] if isinstance(row, tuple) else row)
        print(f"[{kkt}] epoch {e + 1}: {time.time() - t:.3f} s  info {np.array2string(row, precision=12)}", flush=True)
    t = time.time()
    lrn.Renormalize()
    res = lrn.result()
    print(f"[{kkt}] result {time.time() - t:.3f} s  {np.array2string(np.asarray(res), precision=12)}", flush=True)
    del lrn
