"""Data parallelism on CPU (gloo, world_size 2): every rank keeps the shard
the product assigns it (wfsa_shard_range, as Learner::BuildFrom does), its
partial [loglik, grad] is computed with globally normalized weights (the CPU
oracle stands in for the device evaluation, which needs a GPU), and the sum
goes through the product's host transport -- the wfsa_host_allreduce_fn
wrapper (wfsa_amd._host_callback around wfsa_amd.torch_allreduce) that
wfsa_dev_comm_init_host calls, invoked here through ctypes exactly as the
library invokes it: a host buffer address, a count and an op code (sum of
doubles for [LL, grad], max of bytes for the used-parameter mask).  The sum
must equal the single-process result.  tests/test_gpu_multiprocess.py runs
the device path itself over the same transport."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _eval_shard(text, sym, off, wt, names_w, b, e):
    """oracle trellis on strings [b, e) with weights normalized over ALL strings"""
    from oracle import Oracle, TRELLIS
    sub_off = off[b:e + 1] - off[b]
    sub_sym = sym[off[b]:off[e]]
    o = Oracle.from_arrays(text, sub_sym, sub_off, wt[b:e], mode=TRELLIS)
    w = np.array([names_w[n] for n in o.full_param_names()])
    ll, logq, grad = o.trellis_eval(w)      # normalized by the shard's own sum
    scale = wt[b:e].sum() / wt.sum()
    by_name = dict(zip(o.full_param_names(), grad * scale))
    return ll * scale, by_name


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
    import wfsa_amd as W
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    syn = W.Synthetic(n_states=32, degree=4, vocab=8, emissions=2, n_strings=400, max_len=16, seed=4)
    sym, off, wt = syn.corpus()
    names = W.Fsa.read_text(syn.wfsa_text).param_names()
    names_w = dict(zip(names, np.random.default_rng(0).normal(-1.2, 0.4, size=len(names))))
    b, e = W.shard_range(off, world, rank)
    ll, g = _eval_shard(syn.wfsa_text, sym, off, wt, names_w, b, e)
    vec = np.array([ll] + [g[n] for n in names] + [float(e - b)], dtype=np.float64)
    cb = W._host_callback(W.torch_allreduce)          # the product's wfsa_host_allreduce_fn
    assert cb(None, vec.ctypes.data, len(vec), 0) == 0          # op 0: sum of doubles
    used = np.zeros(len(names), dtype=np.uint8)                  # a rank's used-parameter mask
    used[rank::world] = 1
    assert cb(None, used.ctypes.data, len(used), 2) == 0        # op 2: max of bytes
    assert used.all()
    if rank == 0:
        full_ll, full_g = _eval_shard(syn.wfsa_text, sym, off, wt, names_w, 0, len(wt))
        q.put((vec, full_ll, np.array([full_g[n] for n in names]), len(wt)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_allreduce_equals_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    vec, full_ll, full_g, n = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert vec[-1] == n                         # every string on exactly one rank
    assert abs(vec[0] - full_ll) <= 1e-12 * abs(full_ll)
    np.testing.assert_allclose(vec[1:-1], full_g, rtol=1e-11, atol=1e-15)
