"""Multi-rank step cost on ONE GPU: N rank processes (spawned, gloo process
group, the host transport) share a c3-like corpus of S strings; each times
Run(K) of the device-resident QN loop.  With WFSA_PEER=1 every per-step
[LL, grad] sum is the one-shot peer kernel (IPC-mapped slots between the
processes); with WFSA_PEER=0 it goes through gloo on the host.  The N=1 run
is the same corpus in one process.  The ranks share the device, so the
step time of N ranks is about the 1-rank step plus what the rank
combination adds (all-reduce, the non-fused QN step, the finish)."""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))

S = int(os.environ.get("MP_STRINGS", "1000000"))
K = int(os.environ.get("MP_STEPS", "200"))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, peer, q):
    os.environ["WFSA_PEER"] = "1" if peer else "0"
    import torch
    import torch.distributed as dist
    import wfsa_amd as W
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=S, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    lrn = W.QuasiNewtonLearner(0)
    if world > 1:
        lrn.SetHostCommunicator(world, rank, W.torch_allreduce)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    lrn.Run(10, 1.0, -1.0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = lrn.Run(K, 1.0, -1.0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = lrn.stats()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    q.put((rank, dt * 1e6 / K, rows[-1][0], st["comm_peer"]))


def main():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    for world, peer in [(1, False), (2, True), (2, False), (4, True)]:
        q = ctx.Queue()
        port = free_port()
        procs = [ctx.Process(target=worker, args=(r, world, port, peer, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = sorted(q.get(timeout=300) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
        us = max(r[1] for r in res)
        print(f"ranks {world} peer {peer}: {us:.1f} us/step (max over ranks), KL {res[0][2]:.12g}, "
              f"comm_peer {[r[3] for r in res]}", flush=True)


if __name__ == "__main__":
    main()
