"""Per-Run fixed cost of the device-resident QN loop (c3, 1M strings).

Times lrn.Run(K) for several K with and without the rmin column, inside the
same barrier + synchronize bracket bench.py uses; with WFSA_RUN_TRACE=1 the
library prints each Run's phases to stderr.  Fit: time(K) = a + b*K.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))


def main():
    import torch
    import wfsa_amd as W
    n = int(os.environ.get("RC_STRINGS", "1000000"))
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=n, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    lrn = W.QuasiNewtonLearner(0)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    ks = [int(k) for k in os.environ.get("RC_KS", "1,2,5,20,50,200").split(",")]
    reps = int(os.environ.get("RC_REPS", "3"))
    for rmin in [bool(int(v)) for v in os.environ.get("RC_RMIN", "0,1").split(",")]:
        lrn.set_info_rmin(rmin)
        lrn.Run(10, 1.0, -1.0)
        res = {}
        for rep in range(reps):
            for k in ks:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                rows = lrn.Run(k, 1.0, -1.0)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                assert len(rows) == k
                res.setdefault(k, []).append(dt * 1e6)
        x = np.array(ks, dtype=float)
        y = np.array([min(res[k]) for k in ks])
        b, a = np.polyfit(x, y, 1) if len(ks) > 1 else (y[0] / x[0], 0.0)
        print(f"rmin={rmin}: " + ", ".join(f"K={k}: {min(res[k]):.0f} us ({min(res[k]) / k:.1f}/step)" for k in ks))
        print(f"rmin={rmin}: fit fixed {a:.1f} us + {b:.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
