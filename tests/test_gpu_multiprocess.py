"""The product's data-parallel path across PROCESSES on one GPU: two rank
processes (torch.multiprocessing spawn), a gloo process group, each rank a
QuasiNewtonLearner whose communicator is the host transport
(wfsa_learner_set_comm_host -> torch.distributed.all_reduce over gloo).  The
per-evaluation [LL, grad] sums take the one-shot peer all-reduce
(WFSA_PEER=1): each rank's kernel stores its vector into the other
process's IPC-mapped receive slots and sums them in rank order -- the
cross-process mapping an 8-GPU RCCL job uses, here between two processes on
one device.  Every rank's KL, gradient, epoch rows and final x must equal one
context over the whole corpus; the same with the peer path off (the gloo
transport carries every sum).  The in-process group runs the same peer
kernel between contexts of one process.  All tests need a gfx950 device."""
import os
import socket
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

SPEC = dict(n_states=64, degree=8, vocab=16, emissions=1, n_strings=3000, max_len=64, seed=9)


def _close(a, b, rel, atol=1e-13):
    return abs(a - b) <= max(atol, rel * max(abs(a), abs(b)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _learn(W, fsa, sym, off, wt, setup=None):
    lrn = W.QuasiNewtonLearner(0)
    if setup:
        setup(lrn)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    kl, g, _ = lrn.objective_grad()
    rows = [lrn.OptimizationStep(1.0, -1.0)[0] for _ in range(2)] + lrn.Run(5, 1.0, -1.0)
    return dict(kl=kl, grad=g, rows=[list(r) for r in rows], x=lrn.x(), info=lrn.info(), stats=lrn.stats())


def _worker(rank, world, port, peer, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
    os.environ["WFSA_PEER"] = "1" if peer else "0"
    import torch.distributed as dist
    import wfsa_amd as W
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        syn = W.Synthetic(**SPEC)
        sym, off, wt = syn.corpus()
        fsa = W.Fsa.read_text(syn.wfsa_text)
        res = _learn(W, fsa, sym, off, wt, lambda l: l.SetHostCommunicator(world, rank, W.torch_allreduce))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:   # reported to the parent, never a hang
        import traceback
        q.put((rank, {"error": f"{type(e).__name__}: {e}\n{traceback.format_exc()}"}))


def _one_context():
    import wfsa_amd as W
    syn = W.Synthetic(**SPEC)
    sym, off, wt = syn.corpus()
    return _learn(W, W.Fsa.read_text(syn.wfsa_text), sym, off, wt)


def _compare(res, one):
    assert _close(res["kl"], one["kl"], rel=1e-12)
    np.testing.assert_allclose(res["grad"], one["grad"], rtol=1e-11, atol=1e-15)
    assert len(res["rows"]) == len(one["rows"]) == 7
    for a, b in zip(res["rows"], one["rows"]):
        for u, v in zip(a[:5], b[:5]):
            assert _close(u, v, rel=1e-10, atol=1e-13)
    np.testing.assert_allclose(res["x"], one["x"], rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("peer", [True, False])
def test_two_processes_over_gloo_equal_one_context(peer):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, peer, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, res = q.get(timeout=240)
            got[r] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "error" not in got[r], got[r].get("error")
    one = _one_context()
    for r in range(world):
        assert got[r]["stats"]["comm_ranks"] == world
        assert got[r]["stats"]["comm_peer"] == (1 if peer else 0)
        _compare(got[r], one)


def _in_child(body):
    """run `body` (a function of this module) in a fresh Python process: two
    contexts of one process whose peer kernels spin on each other's flags
    need their streams on distinct hardware queues, which a process that has
    already made and dropped many contexts (this test session) does not
    guarantee -- HIP spreads streams over GPU_MAX_HW_QUEUES queues, and two
    streams on one queue run in order, so one rank's spinning kernel would
    hold back the other's (the wait then gives up: NaN).  The child starts
    with 4 streams on 8 queues."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (f"import sys; sys.path[:0] = [{here!r}, {ROOT!r}, {os.path.join(ROOT, 'w-fsa_amd')!r}]\n"
            f"import test_gpu_multiprocess as t; t.{body}()")
    env = dict(os.environ, WFSA_PEER="1", GPU_MAX_HW_QUEUES="8")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]


def _peer_group_body():
    import wfsa_amd as W
    syn = W.Synthetic(**SPEC)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    gid = W.Device.comm_local_id(2)
    with ThreadPoolExecutor(max_workers=2) as ex:
        futs = [ex.submit(_learn, W, fsa, sym, off, wt, lambda l, r=r: l.SetCommunicator(2, r, gid)) for r in range(2)]
        outs = [f.result(timeout=300) for f in futs]
    one = _one_context()
    for res in outs:
        assert res["stats"]["comm_peer"] == 1
        _compare(res, one)


def test_in_process_group_peer_path():
    """the same peer kernel between two contexts of one process (the
    pointers themselves instead of IPC handles)"""
    _in_child("_peer_group_body")


def _family_a_eval(W):
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=2000, max_len=128, seed=11)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    w = np.random.default_rng(7).normal(-1.5, 0.7, size=len(fsa.param_names()))
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, wt / wt.sum())
    dev.recognize()
    ll, grad, _ = dev.objective_grad(w)
    return ll, np.array(grad)


def _after_group_body():
    import wfsa_amd as W
    os.environ["WFSA_PEER"] = "0"
    ll0, g0 = _family_a_eval(W)
    os.environ["WFSA_PEER"] = "1"
    syn = W.Synthetic(**SPEC)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    for _ in range(2):   # two groups one after the other: the second reuses the first's areas
        gid = W.Device.comm_local_id(2)
        with ThreadPoolExecutor(max_workers=2) as ex:
            futs = [ex.submit(_learn, W, fsa, sym, off, wt, lambda l, r=r: l.SetCommunicator(2, r, gid)) for r in range(2)]
            outs = [f.result(timeout=300) for f in futs]
        assert all(o["stats"]["comm_peer"] == 1 for o in outs)
    for _ in range(3):
        ll1, g1 = _family_a_eval(W)
        assert ll1 == ll0
        np.testing.assert_array_equal(g1, g0)


def test_context_after_peer_group_is_exact():
    """a context made after an in-process peer group is gone evaluates to the
    same bits as one made before it (the group's uncached areas must not
    reach later contexts' allocations: fp64 atomics into them were lost)"""
    _in_child("_after_group_body")
