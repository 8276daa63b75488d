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
# a family-A-like corpus large enough per rank that its bubbles ride in the
# stream kernel -- the in-kernel update's rmin column needs that
SPEC_A = dict(n_states=256, degree=8, vocab=64, emissions=1, n_strings=60000, max_len=64, seed=9)


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


def _worker(rank, world, port, peer, q, late_s=0.0, abort=False, spec=None, rmin=True):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "w-fsa_amd"))
    os.environ["WFSA_PEER"] = "1" if peer else "0"
    os.environ["WFSA_QN_INKERNEL"] = "1"   # (small shards: the cover rule alone would take the two-kernel step)
    if late_s:
        os.environ["WFSA_PEER_TIMEOUT_S"] = "3"
    import torch.distributed as dist
    import wfsa_amd as W
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        syn = W.Synthetic(**(spec or SPEC))
        sym, off, wt = syn.corpus()
        fsa = W.Fsa.read_text(syn.wfsa_text)
        if abort == "d2h":
            q.put((rank, _d2h_learn(W, fsa, sym, off, wt, world, rank)))
            return
        if abort:
            if abort == "stall":
                os.environ["WFSA_COMM_TIMEOUT_S"] = "3"
            q.put((rank, _abort_learn(W, fsa, sym, off, wt, world, rank, abort == "stall")))
            return
        if late_s:   # rank 1 arrives at the device loop after the others' peer waits gave up
            res = _late_learn(W, fsa, sym, off, wt, world, rank, late_s)
            q.put((rank, res))
            return
        def setup(lrn):
            lrn.set_info_rmin(rmin)
            lrn.SetHostCommunicator(world, rank, W.torch_allreduce)
        res = _learn(W, fsa, sym, off, wt, setup)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:   # reported to the parent, never a hang
        import traceback
        q.put((rank, {"error": f"{type(e).__name__}: {e}\n{traceback.format_exc()}"}))


def _late_learn(W, fsa, sym, off, wt, world, rank, late_s):
    """the device QN loop with rank 1 late by late_s: every rank must raise
    (WFSA_ERR_RCCL) -- rank 0 when its peer wait gives up, rank 1 at entry
    of its first peer sum (its area was poisoned) -- and neither may report
    a non-finite halt"""
    import time
    lrn = W.QuasiNewtonLearner(0)
    lrn.SetHostCommunicator(world, rank, W.torch_allreduce)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    lrn.objective_grad()   # the peer path set up and checked while both ranks are here
    assert lrn.stats()["comm_peer"] == 1
    if rank == 1:
        time.sleep(late_s)
    t0 = time.time()
    try:
        rows = lrn.Run(5, 1.0, -1.0)
        return {"raised": None, "rows": [list(r) for r in rows], "s": time.time() - t0}
    except W.WfsaError as e:
        return {"raised": str(e), "code": e.code, "s": time.time() - t0}


def _abort_learn(W, fsa, sym, off, wt, world, rank, stall=False):
    """the host transport (gloo) with the peer path off: rank 1 fails outside
    the library and aborts while rank 0 waits in the per-step gradient sum
    (a non-peer collective); rank 0 must fail at once with the reason, not at
    gloo's 30-minute timeout.  stall: rank 1 stalls instead (no abort) and
    rank 0's wait gives up at WFSA_COMM_TIMEOUT_S (3 s)"""
    import time
    lrn = W.QuasiNewtonLearner(0)
    lrn.SetHostCommunicator(world, rank, W.torch_allreduce)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    lrn.objective_grad()   # both ranks here, healthy
    assert lrn.stats()["comm_peer"] == 0
    t0 = time.time()
    if rank == 1 and stall:
        time.sleep(8.0)    # past rank 0's 3 s limit, without a word
        try:
            lrn.Run(5, 1.0, -1.0)
            return {"raised": None}
        except W.WfsaError as e:
            return {"raised": str(e), "s": time.time() - t0 - 8.0}
    if rank == 1:
        time.sleep(2.0)    # rank 0 is inside Run by now
        lrn.AbortCommunicator("rank 1: injected failure")
        t_abort = time.time() - t0
        try:
            lrn.Run(5, 1.0, -1.0)
            return {"raised": None}
        except W.WfsaError as e:
            return {"raised": str(e), "s": time.time() - t0, "abort_s": t_abort}
    try:
        rows = lrn.Run(50, 1.0, -1.0)
        return {"raised": None, "rows": len(rows)}
    except W.WfsaError as e:
        return {"raised": str(e), "s": time.time() - t0}


def _d2h_learn(W, fsa, sym, off, wt, world, rank):
    """host transport, peer path off; rank 1's 12th payload finds its
    device-to-host copy failed (WFSA_FAULT_HOST_D2H): it must still join that
    payload exchange (poisoned) and fail, so rank 0 is never left in a
    mismatched exchange -- it sees the poison (a non-finite halt) or fails at
    its next header (WFSA_COMM_TIMEOUT_S), within seconds either way"""
    import time
    os.environ["WFSA_COMM_TIMEOUT_S"] = "3"
    if rank == 1:
        os.environ["WFSA_FAULT_HOST_D2H"] = "12"
    t0 = time.time()
    try:
        lrn = W.QuasiNewtonLearner(0)
        lrn.SetHostCommunicator(world, rank, W.torch_allreduce)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        rows = lrn.Run(30, 1.0, -1.0)
        return {"raised": None, "rows": len(rows), "last": list(rows[-1]) if rows else [], "s": time.time() - t0}
    except W.WfsaError as e:
        return {"raised": str(e), "s": time.time() - t0}


def _one_context(spec=None, rmin=True):
    import wfsa_amd as W
    syn = W.Synthetic(**(spec or SPEC))
    sym, off, wt = syn.corpus()
    return _learn(W, W.Fsa.read_text(syn.wfsa_text), sym, off, wt, lambda l: l.set_info_rmin(rmin))


def _compare(res, one):
    assert _close(res["kl"], one["kl"], rel=1e-12)
    np.testing.assert_allclose(res["grad"], one["grad"], rtol=1e-11, atol=1e-15)
    assert len(res["rows"]) == len(one["rows"]) == 7
    for a, b in zip(res["rows"], one["rows"]):
        for u, v in zip(a[:5], b[:5]):
            assert _close(u, v, rel=1e-10, atol=1e-13)
    np.testing.assert_allclose(res["x"], one["x"], rtol=1e-10, atol=1e-12)


def _spawn(world, peer, late_s=0.0, abort=False, spec=None, rmin=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, peer, q, late_s, abort, spec, rmin)) for r in range(world)]
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
    return got


@pytest.mark.parametrize("peer", [True, False])
@pytest.mark.parametrize("corpus", ["small", "familyA"])
def test_two_processes_over_gloo_equal_one_context(peer, corpus):
    """familyA: VERDICT r5 item 4 -- with the peer path the device QN loop
    keeps the update in the stream kernel across ranks: each batch's member
    partials, the log-likelihood and the rmin pair are exchanged through the
    peer areas inside the launch; the rows (rmin included: value and global
    string) still equal one context's.  small: the heavily ambiguous corpus
    whose bubbles do not fit the stream kernel -- the separate kernels"""
    world = 2
    spec = SPEC_A if corpus == "familyA" else SPEC
    got = _spawn(world, peer, spec=spec)
    one = _one_context(spec)
    for r in range(world):
        assert got[r]["stats"]["comm_ranks"] == world
        assert got[r]["stats"]["comm_peer"] == (1 if peer else 0)
        assert (got[r]["stats"]["qn_inkernel_waves"] > 0) == (peer and corpus == "familyA"), got[r]["stats"]
        _compare(got[r], one)
        for a, b in zip(got[r]["rows"], one["rows"]):   # the rmin column: value and (global) string
            assert _close(a[5], b[5], rel=1e-10) and a[6] == b[6], (a, b)


def test_two_processes_inkernel_without_rmin_equal_one_context():
    """the in-kernel update across ranks with the rmin column off (the
    ambiguous corpus: its separate bubble kernel runs before the stream
    kernel, the exchange as above)"""
    got = _spawn(2, True, rmin=False)
    one = _one_context(rmin=False)
    for r in range(2):
        assert got[r]["stats"]["qn_inkernel_waves"] > 0, got[r]["stats"]
        _compare(got[r], one)


def test_two_processes_late_rank_fails_every_rank():
    """rank 1 reaches the device QN loop 8 s late, past WFSA_PEER_TIMEOUT_S
    (3 s): rank 0's peer wait gives up, poisons both areas and raises; rank
    1 raises at its first peer sum without waiting (the timeout
    used to become a NaN gradient and a non-finite halt)"""
    got = _spawn(2, True, late_s=8.0)
    for r in range(2):
        assert got[r]["raised"], f"rank {r} did not fail: {got[r]}"
        assert "peer all-reduce" in got[r]["raised"], got[r]["raised"]
    assert got[0]["s"] < 30          # the 3 s timeout, not a hang
    assert got[1]["s"] < 5           # poisoned: fails at entry


def test_two_processes_abort_over_gloo_fails_every_rank():
    """an abort must reach the other processes over the host
    transport too.  Rank 1 aborts 2 s in; rank 0, waiting in a gloo sum of
    the QN loop, fails within seconds with "aborted the group"; rank 1's own
    next collective fails at entry"""
    got = _spawn(2, False, abort=True)
    assert got[0]["raised"] and "aborted the group" in got[0]["raised"], got[0]
    assert got[0]["s"] < 20, got[0]
    assert got[1]["raised"], got[1]
    assert got[1]["abort_s"] < 20, got[1]


def test_two_processes_stalled_rank_times_out_over_gloo():
    """ADVICE/VERDICT r4 item 6: a member that stalls without aborting.  Rank
    0 waits in a gloo sum; its wait gives up at WFSA_COMM_TIMEOUT_S (3 s) and
    the call fails (the transport is then broken for good); rank 1, back
    8 s later, fails too (rank 0 is gone or its limit ends the wait)"""
    got = _spawn(2, False, abort="stall")
    assert got[0]["raised"] and "callback failed" in got[0]["raised"], got[0]
    assert 2.5 < got[0]["s"] < 15, got[0]
    assert got[1]["raised"], got[1]
    assert got[1]["s"] < 15, got[1]


def test_two_processes_failed_copy_keeps_the_exchange_in_step():
    """a member whose device-to-host copy fails after the header
    exchange joins the payload exchange poisoned and leaves the transport
    broken -- it never sends an 8-byte abort header into the peers' payload
    exchange.  Rank 1 raises with the copy failure; rank 0 ends within
    seconds, with an error or a non-finite halt (the poison), never a
    success on a partial sum"""
    got = _spawn(2, False, abort="d2h")
    assert got[1]["raised"] and "device to host copy failed" in got[1]["raised"], got[1]
    assert got[1]["s"] < 60, got[1]
    r0 = got[0]
    assert r0["s"] < 60, r0
    if not r0["raised"]:   # the poison reached it: the run halted non-finite before 30 steps
        assert r0["rows"] < 30 and not all(np.isfinite(r0["last"][:5])), r0


# ---- the peer kernel on one device, the other members simulated ----------

@pytest.mark.parametrize("nranks,n", [(2, 1), (2, 3000), (3, 1025), (8, 65536)])
def test_peer_kernel_sums_in_rank_order(nranks, n):
    import wfsa_amd as W
    err, status, poisoned, secs = W.Device.peer_selftest(nranks, n, 5.0, 0)
    assert err == 0.0                 # bit for bit the rank-order sum
    assert status == 0 and poisoned == 0
    assert secs < 2


def test_peer_kernel_gives_up_and_poisons_every_area():
    import wfsa_amd as W
    nan, status, poisoned, secs = W.Device.peer_selftest(4, 3000, 0.5, 1)
    assert nan == 3000                # NaN results, never a partial sum
    assert status == 1                # the host-mapped status word (Collective::check)
    assert poisoned == 4              # every member's next call fails at entry
    assert 0.4 < secs < 5


def test_peer_kernel_fails_at_entry_when_poisoned():
    import wfsa_amd as W
    nan, status, poisoned, secs = W.Device.peer_selftest(4, 3000, 10.0, 2)
    assert nan == 3000 and status == 1 and poisoned == 4
    assert secs < 1                   # no wait


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


def test_context_after_peer_selftest_is_exact():
    """contexts made after peer areas were used and handed back evaluate to
    the same bits as one made before (the uncached areas must never reach
    later contexts' allocations: fp64 atomics into them were lost, round 3)"""
    import wfsa_amd as W
    ll0, g0 = _family_a_eval(W)
    for _ in range(3):
        W.Device.peer_selftest(2, 65536, 5.0, 0)
        W.Device.peer_selftest(8, 65536, 5.0, 0)
        ll1, g1 = _family_a_eval(W)
        assert ll1 == ll0
        np.testing.assert_array_equal(g1, g0)


# ---- in-process groups: the peer path refused, failures propagate ---------

def _group(k, fn):
    """run fn(k, rank, gid) on k threads; every rank's result or exception"""
    import wfsa_amd as W
    gid = W.Device.comm_local_id(k)
    with ThreadPoolExecutor(max_workers=k) as ex:
        futs = [ex.submit(fn, k, r, gid) for r in range(k)]
        out = []
        for f in futs:
            try:
                out.append(f.result(timeout=100))
            except Exception as e:   # (a product error, not a test timeout)
                out.append(e)
    return out


def test_in_process_group_on_one_device_refuses_peer(monkeypatch):
    """WFSA_PEER=1 on an in-process group whose members share a device: the
    path is refused (their spinning kernels need not run concurrently), the
    transport carries every sum, and the result equals one context"""
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_PEER", "1")
    syn = W.Synthetic(**SPEC)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    outs = _group(2, lambda k, r, gid: _learn(W, fsa, sym, off, wt, lambda l: l.SetCommunicator(k, r, gid)))
    one = _one_context()
    for res in outs:
        assert not isinstance(res, Exception), res
        assert res["stats"]["comm_peer"] == 0
        _compare(res, one)


def _prepared(W, k, r, gid):
    syn = W.Synthetic(**SPEC)
    sym, off, wt = syn.corpus()
    lrn = W.QuasiNewtonLearner(0)
    lrn.SetCommunicator(k, r, gid)
    lrn.BuildFromPacked(W.Fsa.read_text(syn.wfsa_text), sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    return lrn


def test_aborted_rank_fails_every_rank_promptly():
    """rank 1 fails outside the library and aborts; rank 0, already waiting
    in the device loop's per-step sum, fails at once with the reason"""
    import time
    import wfsa_amd as W

    def body(k, r, gid):
        lrn = _prepared(W, k, r, gid)
        t0 = time.time()
        if r == 1:
            time.sleep(1.0)   # rank 0 is inside Run by now
            lrn.AbortCommunicator("rank 1: injected failure")
            with pytest.raises(W.WfsaError):
                lrn.Run(5, 1.0, -1.0)
            return time.time() - t0
        with pytest.raises(W.WfsaError) as e:
            lrn.Run(5, 1.0, -1.0)
        assert "injected failure" in str(e.value) or "failed" in str(e.value)
        return time.time() - t0

    outs = _group(2, body)
    for o in outs:
        assert not isinstance(o, Exception), o
        assert o < 10


def test_late_rank_times_out_every_rank(monkeypatch):
    """WFSA_GROUP_TIMEOUT_S=2 and rank 1 six seconds late: rank 0's barrier
    gives up after ~2 s and poisons the group; rank 1 fails at its first
    collective without waiting"""
    import time
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_GROUP_TIMEOUT_S", "2")

    def body(k, r, gid):
        lrn = _prepared(W, k, r, gid)
        if r == 1:
            time.sleep(6.0)
        t0 = time.time()
        with pytest.raises(W.WfsaError) as e:
            lrn.Run(5, 1.0, -1.0)
        return time.time() - t0, str(e.value)

    outs = _group(2, body)
    for o in outs:
        assert not isinstance(o, Exception), o
    assert 1.5 < outs[0][0] < 10 and "WFSA_GROUP_TIMEOUT_S" in outs[0][1]
    assert outs[1][0] < 2
