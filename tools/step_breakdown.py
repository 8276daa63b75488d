"""Where a QuasiNewton step's time goes (GPU box): full step vs device call
vs kernels.  python tools/step_breakdown.py [n_strings]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
import numpy as np  # noqa: E402
import wfsa_amd as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
syn = W.Synthetic(n_strings=n, seed=1)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
lrn = W.QuasiNewtonLearner(0)
lrn.BuildFromPacked(fsa, sym, off, wt)
lrn.Finalize()
lrn.Init(7)
K = 50


def timed(fn):
    for _ in range(5):
        fn()
    t = time.perf_counter()
    for _ in range(K):
        fn()
    return (time.perf_counter() - t) / K * 1e3


step = timed(lambda: lrn.OptimizationStep(1.0, 1e-6))
st = lrn.stats()
obj = timed(lambda: lrn.objective_grad())
dev = W.Device(0)
dev.load_model(fsa)
p = wt / wt.sum()
dev.load_corpus(sym, off, p)
w = np.full(fsa.counts()["parameters"], -2.0)
dcall = timed(lambda: dev.objective_grad(w, want_logq=False))
ds = dev.stats()
print(f"step {step:.3f} ms | learner objective_grad {obj:.3f} ms | Device.objective_grad {dcall:.3f} ms | "
      f"device-side call {ds['last_call_ms']:.3f} ms | fb kernels {ds['last_fb_kernel_ms']:.3f} ms | "
      f"compiled {ds['last_compiled_ms']:.3f} ms")
