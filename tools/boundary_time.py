"""The bench's `boundary` sub-record alone (c3: QuasiNewtonLearner::
OptimizationStep through wfsa_dev_objective_grad, host QN update), for A/B
of library builds (WFSA_LIB): per-step time and its host phases."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))


def main():
    import torch
    import wfsa_amd as W
    torch.cuda.synchronize()
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=1_000_000, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    lrn = W.QuasiNewtonLearner(0)
    lrn.BuildFromPacked(W.Fsa.read_text(syn.wfsa_text), sym, off, wt)
    lrn.Finalize()
    for rep in range(3):
        lrn.Init(7)
        for _ in range(3):
            lrn.OptimizationStep(1.0, -1.0)
        s0 = lrn.stats()
        k = 50
        t0 = time.perf_counter()
        for _ in range(k):
            lrn.OptimizationStep(1.0, -1.0)
        dt = time.perf_counter() - t0
        s1 = lrn.stats()
        ph = " ".join(f"{f[5:-3]} {1e3 * (s1[f] - s0[f]) / k:.1f}" for f in ("host_begin_ms", "host_overlap_ms",
                                                                         "host_wait_ms", "host_post_ms"))
        print(f"{os.path.basename(os.path.dirname(os.environ.get('WFSA_LIB', 'release/x')))}: "
              f"{dt * 1e6 / k:.1f} us/step ({ph} us)", flush=True)


if __name__ == "__main__":
    main()
