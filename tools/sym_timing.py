"""Times the device LDL^T (wfsa_dev_sym_factor / _solve) at KKT sizes (GPU box)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import wfsa_amd as W  # noqa: E402

dev = W.Device(0)
for n in [int(v) for v in sys.argv[1:]] or [1000, 2000, 4000]:
    rng = np.random.default_rng(n)
    a = rng.normal(size=(n, n))
    a = (a + a.T) / 2
    dev.sym_factor(a[:8, :8])
    t = time.time()
    r = dev.sym_factor(a)
    t1 = time.time()
    x = dev.sym_solve(np.ones(n))
    t2 = time.time()
    print(f"n={n}: factor {t1 - t:.3f} s, solve {t2 - t1:.3f} s, inertia {r[0]}", flush=True)
