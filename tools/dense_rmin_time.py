"""Cost of the dense path's rmin column at c5 size (BASELINE configs[4]:
4096 states, 4096 strings): one evaluation, then the (min, +) pass, timed
separately (host clock around synchronous calls)."""
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
for k in range(3):
    t0 = time.perf_counter()
    dev.objective_grad(w, want_logq=False)
    t1 = time.perf_counter()
    r, s = dev.rmin()
    t2 = time.perf_counter()
    st = dev.stats()
    R, T, npad = st["dense_rows"], st["dense_steps"], st["dense_np"]
    ops = 2.0 * npad * npad * R * (T - 1)
    print(f"eval {1e3 * (t1 - t0):.1f} ms  rmin {1e3 * (t2 - t1):.1f} ms  ({ops / (t2 - t1) / 1e12:.1f} T min/add per s, "
          f"R {R} T {T} np {npad})  rmin {r:.6e} string {s}", flush=True)
