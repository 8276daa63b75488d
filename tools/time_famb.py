"""Wall time of one objective/gradient evaluation on the famB workload
(1024 states, out-degree 8, 4 of 16 symbols per state, 100k strings):
wfsa_dev_objective_grad without log q.  For kernel experiments (WFSA_W2_DBG)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
syn = W.Synthetic(n_states=1024, degree=8, vocab=16, emissions=4, n_strings=n, max_len=128, seed=1)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
dev = W.Device(0)
dev.load_model(fsa)
dev.load_corpus(sym, off, wt / wt.sum())
dev.recognize()
w = np.random.default_rng(0).normal(-1.5, 0.3, size=len(fsa.param_names()))
for _ in range(2):
    dev.objective_grad(w, want_logq=False)
t = time.perf_counter()
k = 5
for _ in range(k):
    ll, g, _ = dev.objective_grad(w, want_logq=False)
dt = (time.perf_counter() - t) / k
lib = os.path.basename(os.path.dirname(os.environ.get("WFSA_LIB", "release/x")))
print(f"{lib} dbg {os.environ.get('WFSA_W2_DBG', '0')}: {dt * 1e3:.3f} ms per evaluation, "
      f"{n / dt / 1e6:.2f} M strings/s, ll {ll!r}, grad sum {float(np.sum(g))!r} |g| {float(np.abs(g).sum())!r}")
