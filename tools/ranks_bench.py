"""Multi-rank step cost on ONE GPU, in one process: N contexts form an
in-process group (one thread each) over a c3-like corpus of S strings; with
WFSA_PEER=1 every per-step [LL, grad] sum is the one-shot peer kernel
(stream-ordered, no host step).  The contexts share the device (kernels of
different streams run concurrently), so the N-rank step is about the 1-rank
step of the same corpus plus what the rank combination adds: the reduction
kernel, the peer all-reduce, the non-fused QN step.  (Separate processes on
one GPU take turns on it -- two rank processes measured 349 us per step with
the peer path, 452 with gloo -- so only threads of one process show the
step cost.)"""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

# a hardware queue per context, so no rank's spinning peer kernel sits in
# front of another rank's work (set before HIP starts); a stuck wait gives up
# after 2 s instead of 10
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
os.environ.setdefault("WFSA_PEER_TIMEOUT_S", "2")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))

S = int(os.environ.get("RB_STRINGS", "1000000"))
K = int(os.environ.get("RB_STEPS", "200"))


def main():
    import threading
    import torch
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=S, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    for world, peer in [(1, False), (2, True), (4, True), (8, True)]:
        os.environ["WFSA_PEER"] = "1" if peer else "0"
        gid = W.Device.comm_local_id(world) if world > 1 else None
        bar = threading.Barrier(world)

        def rank(r):
            lrn = W.QuasiNewtonLearner(0)
            if world > 1:
                lrn.SetCommunicator(world, r, gid)
            lrn.BuildFromPacked(fsa, sym, off, wt)
            lrn.Finalize()
            lrn.Init(7)
            lrn.Run(10, 1.0, -1.0)
            torch.cuda.synchronize()
            bar.wait()
            t0 = time.perf_counter()
            rows = lrn.Run(K, 1.0, -1.0)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            st = lrn.stats()
            bar.wait()
            return dt * 1e6 / K, rows[-1][0], st["comm_peer"]

        with ThreadPoolExecutor(max_workers=world) as ex:
            res = list(ex.map(rank, range(world)))
        print(f"ranks {world} peer {peer}: {max(r[0] for r in res):.1f} us/step (max over ranks), "
              f"KL {res[0][1]:.12g}, comm_peer {[r[2] for r in res]}", flush=True)


if __name__ == "__main__":
    main()
