"""Dense-path evaluations at c5 size (BASELINE configs[4]: 4096 states,
4096 strings) for GEMM kernel A/B under rocprofv3 --kernel-trace --stats
(WFSA_LIB selects a variant build, WFSA_DENSE_BLAS the GEMM engine)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

syn = W.Synthetic(n_states=4096, degree=1, vocab=16, emissions=16, dense=True, n_strings=4096, max_len=128, seed=2)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
dev = W.Device(0)
dev.load_model(fsa)
dev.load_corpus(sym, off, wt / wt.sum())
assert dev.stats()["dense"] == 1
dev.recognize()
w = np.random.default_rng(11).normal(-8.5, 1.0, size=fsa.counts()["parameters"])
for k in range(int(os.environ.get("TD_EVALS", "3"))):
    t0 = time.perf_counter()
    ll, _, _ = dev.objective_grad(w, want_logq=False)
    print(f"eval {1e3 * (time.perf_counter() - t0):.1f} ms  ll {ll:.12g}", flush=True)
