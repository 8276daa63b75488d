"""The QN step across ranks on ONE GPU, for the 8-GPU projection.

single S: one process, a c3-like corpus of S strings (no communicator).
pairlocal S: the same two processes on this GPU, each with S/2 strings and
          no communicator (independent learners started together): the GPU
          sharing alone, for the exchange's share of the pair's time.
pair S:   two rank processes on this GPU (torch.distributed gloo for the
          set-up, the host transport, WFSA_PEER=1), S strings split in two
          contiguous shards: the in-kernel QN update exchanges each batch's
          member partials through the peer areas (two processes' kernels run
          concurrently on the device: the shards are kept small enough that
          both grids are resident together).
Prints the per-step time (max over ranks) of Run(K) after a warm-up Run, the
in-kernel waves (0: the separate kernels ran) and the last KL."""
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
K = int(os.environ.get("XR_STEPS", "200"))


def corpus(W, n):
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=n, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    return W.Fsa.read_text(syn.wfsa_text), sym, off, wt


def timed(lrn, torch, sync=lambda: None):
    lrn.Run(20, 1.0, -1.0)
    torch.cuda.synchronize()
    sync()
    t0 = time.perf_counter()
    rows = lrn.Run(K, 1.0, -1.0)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6 / K, rows[-1][0], lrn.stats()["qn_inkernel_waves"]


def worker(rank, port, n, rmin, q, comm=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WFSA_PEER="1")
    import torch
    import torch.distributed as dist
    import wfsa_amd as W
    try:
        dist.init_process_group("gloo", rank=rank, world_size=2)
        fsa, sym, off, wt = corpus(W, n)
        lrn = W.QuasiNewtonLearner(0)
        lrn.set_info_rmin(rmin)
        if comm:
            lrn.SetHostCommunicator(2, rank, W.torch_allreduce)
            lrn.BuildFromPacked(fsa, sym, off, wt)
        else:   # this rank's contiguous half, its own learner
            h = (len(off) - 1) // 2
            a, b = rank * h, (rank + 1) * h
            lrn.BuildFromPacked(fsa, sym[off[a]:off[b]], off[a:b + 1] - off[a], wt[a:b])
        lrn.Finalize()
        lrn.Init(7)
        us, kl, waves = timed(lrn, torch, lambda: dist.barrier())
        t = torch.tensor([us], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, float(t.item()), kl, waves))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:   # reported, never a hang
        q.put((rank, -1.0, str(e), 0))


def main():
    mode, n = sys.argv[1], int(sys.argv[2])
    rmin = os.environ.get("XR_RMIN", "0") == "1"
    if mode == "single":
        import torch
        import wfsa_amd as W
        fsa, sym, off, wt = corpus(W, n)
        lrn = W.QuasiNewtonLearner(0)
        lrn.set_info_rmin(rmin)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        us, kl, waves = timed(lrn, torch)
        print(f"single {n} strings rmin {int(rmin)}: {us:.2f} us/step, in-kernel waves {waves}, KL {kl:.12g}", flush=True)
        return
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, n, rmin, q, mode == "pair")) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    print(f"{mode} {n} strings ({n // 2} per rank) rmin {int(rmin)}: {res[0][1]:.2f} us/step (max over ranks), "
          f"in-kernel waves {res[0][3]}/{res[1][3]}, KL {res[0][2]}", flush=True)


if __name__ == "__main__":
    main()
