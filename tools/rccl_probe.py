"""Probe: can two processes attach RCCL communicators on the SAME GPU?  If
yes, tests can run the real RCCL transport on a one-GPU box.  Each rank
all-reduces [rank + 1] and prints the sum (expected 3)."""
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, uid, q):
    sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
    import numpy as np
    import wfsa_amd as W
    try:
        dev = W.Device(0)
        dev.comm_init(2, rank, uid)
        q.put((rank, float(dev.allreduce(np.array([rank + 1.0]))[0])))
    except Exception as e:   # report, do not hang the parent
        q.put((rank, repr(e)))


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
    import wfsa_amd as W
    ctx = mp.get_context("spawn")
    uid = W.Device.comm_unique_id()
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, uid, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=60) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    print("rccl same-GPU probe:", sorted(res))
