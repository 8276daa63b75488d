"""The bench's timed region, repeated: warmup Run, stats(), barrier, Run(K),
barrier -- every repetition's per-step time (bench.py reports one of them),
with WFSA_RUN_TRACE=1 the library's phases of each Run on stderr."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))


def main():
    import torch
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=int(os.environ.get("BL_STRINGS", "1000000")), max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    lrn = W.QuasiNewtonLearner(0)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    lrn.set_info_rmin(os.environ.get("BL_RMIN") == "1")
    k = int(os.environ.get("BL_STEPS", "20"))
    for rep in range(int(os.environ.get("BL_REPS", "6"))):
        if os.environ.get("BL_PRESLEEP"):   # an idle device before the warm-up (as after the preparation)
            time.sleep(float(os.environ["BL_PRESLEEP"]))
        lrn.Run(int(os.environ.get("BL_WARM", "10")), 1.0, -1.0)
        if os.environ.get("BL_STATS", "1") == "1":
            lrn.stats()
        torch.cuda.synchronize()
        if os.environ.get("BL_SLEEP"):
            time.sleep(float(os.environ["BL_SLEEP"]))
        t0 = time.perf_counter()
        lrn.Run(k, 1.0, -1.0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {rep}: {dt * 1e6 / k:.1f} us/step (in-kernel QN waves {lrn.stats()['qn_inkernel_waves']})", flush=True)


if __name__ == "__main__":
    main()
