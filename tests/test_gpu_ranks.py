"""The product's multi-rank path on one GPU: K contexts of this process form
an in-process group (wfsa_dev_comm_local_id), one thread per rank, and run
exactly the branches an RCCL job runs on K GPUs -- the shard the rank keeps
(Learner::BuildPaths' Sigma-length split), the corpus statistics all-reduce,
the max-reduced used-parameter mask, the constant trivial gradient reduced
once, the per-step all-reduce of [LL, grad] inside the device QN loop, the
plogp all-reduce of Finalize.  Everything is compared with the one-context
run and, for the first evaluation, with the ENUM oracle (the reference's
algorithm, src/Learner.cpp:276-553).  All tests need a gfx950 device."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b, rel, atol=1e-13):
    return abs(a - b) <= max(atol, rel * max(abs(a), abs(b)))


def _with_unrecognized(sym, off, wt, n_bad=7, seed=0):
    """append strings the automaton cannot produce (byte 0x01) at spread
    positions, so several shards hold auxiliary parameters"""
    rng = np.random.default_rng(seed)
    strings = [bytes(sym[off[i]:off[i + 1]]) for i in range(len(wt))]
    w = list(wt)
    for k in range(n_bad):
        pos = int(rng.integers(0, len(strings) + 1))
        strings.insert(pos, b"\x01" * (1 + k % 3))
        w.insert(pos, float(rng.uniform(0.5, 2.0)))
    off2 = np.concatenate([[0], np.cumsum([len(s) for s in strings])]).astype(np.int64)
    return np.frombuffer(b"".join(strings), dtype=np.uint8).copy(), off2, np.array(w)


def _run_ranks(k, fn):
    import wfsa_amd as W
    gid = W.Device.comm_local_id(k)
    with ThreadPoolExecutor(max_workers=k) as ex:
        futs = [ex.submit(fn, k, r, gid) for r in range(k)]
        return [f.result(timeout=300) for f in futs]


FAMILIES = {
    # compiled streams + bubbles
    "bubbles": dict(n_states=64, degree=8, vocab=16, emissions=1, n_strings=3000, max_len=64, seed=9),
    # ambiguous: traversal tiers 0/1 beside the compiled strings
    "ambiguous": dict(n_states=48, degree=6, vocab=8, emissions=3, n_strings=1200, max_len=24, seed=4),
}


@pytest.mark.parametrize("family", sorted(FAMILIES))
@pytest.mark.parametrize("k", [2, 3])
def test_learner_ranks_equal_one_context(family, k):
    import wfsa_amd as W
    syn = W.Synthetic(**FAMILIES[family])
    sym, off, wt = _with_unrecognized(*syn.corpus())
    fsa = W.Fsa.read_text(syn.wfsa_text)

    def learn(nranks, rank, gid):
        lrn = W.QuasiNewtonLearner(0)
        if nranks > 1:
            lrn.SetCommunicator(nranks, rank, gid)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        kl0, g0, _ = lrn.objective_grad()
        rows = [lrn.OptimizationStep(1.0, -1.0)[0] for _ in range(3)]   # host QN update
        rows += lrn.Run(6, 1.0, -1.0)                                   # device-resident loop
        return lrn.info(), lrn.stats(), kl0, g0, rows, lrn.x(), lrn.trimmed_index()

    one = learn(1, 0, None)
    outs = _run_ranks(k, learn)
    info1, _, kl1, g1, rows1, x1, trim1 = one
    shards = []
    for r, (info, st, kl, g, rows, x, trim) in enumerate(outs):
        b, e = W.shard_range(off, k, r)
        assert (info["shard_begin"], info["shard_end"]) == (b, e)
        shards.append(e - b)
        for key in ("n_params", "n_constraints", "n_strings", "n_paths", "n_full"):
            assert info[key] == info1[key], key
        for key in ("common_support", "plogp", "aux_hessian", "model_volume"):
            assert _close(info[key], info1[key], rel=1e-12), key
        np.testing.assert_array_equal(trim, trim1)           # the OR of the shards' used masks
        assert _close(kl, kl1, rel=1e-12)
        np.testing.assert_allclose(g, g1, rtol=1e-11, atol=1e-14)
        assert len(rows) == len(rows1) == 9
        for a, q in zip(rows, rows1):
            for u, v in zip(a[:7], q[:7]):
                assert _close(u, v, rel=1e-10, atol=1e-13)
        np.testing.assert_allclose(x, x1, rtol=1e-10, atol=1e-12)
    assert sum(shards) == len(wt) and min(shards) > 0
    if family == "ambiguous":   # the traversal tiers ran on some rank
        assert sum(o[1]["fallback_strings"] for o in outs) > 0


def test_learner_ranks_match_enum_oracle():
    """KL and gradient of the first evaluation, summed over 2 ranks, against
    the reference algorithm on the whole corpus"""
    import wfsa_amd as W
    from oracle import ENUM, Oracle
    syn = W.Synthetic(n_states=32, degree=4, vocab=6, emissions=2, n_strings=400, max_len=10, seed=9)
    sym, off, wt = _with_unrecognized(*syn.corpus(), n_bad=3, seed=2)
    fsa = W.Fsa.read_text(syn.wfsa_text)
    o = Oracle.from_arrays(syn.wfsa_text, sym, off, wt, mode=ENUM, max_paths=10_000_000)
    orows = o.qn_run(flags=7, epochs=6)

    def learn(nranks, rank, gid):
        lrn = W.QuasiNewtonLearner(0)
        lrn.SetCommunicator(nranks, rank, gid)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        return lrn.info(), lrn.run(flags=7, epochs=6), lrn.x(), lrn.param_names()

    for info, rows, x, names in _run_ranks(2, learn):
        assert info["n_strings"] == o.info["n_strings"]
        assert info["n_paths"] == o.info["n_paths"]
        assert info["n_params"] == o.info["n_params"]
        assert len(rows) == len(orows)
        for r, q in zip(rows, orows):
            for a, b in zip(r[:5], q[:5]):
                assert _close(a, b, rel=1e-8, atol=1e-11)
        ox = dict(zip(o.param_names(), o.x()))
        for n, v in zip(names, x):
            assert _close(v, ox[n], rel=1e-8, atol=1e-10)


def test_device_ranks_sum_to_the_whole():
    """wfsa_dev_* with an in-process communicator: each context loads its
    shard (p normalised over the whole corpus); objective_grad returns the
    all-reduced [LL, grad] on every rank, recognize the max-reduced used
    mask, allreduce sums host buffers -- all equal to one context"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=64, degree=8, vocab=16, emissions=2, n_strings=2000, max_len=40, seed=3)
    sym, off, wt = syn.corpus()
    p = wt / wt.sum()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    w = np.random.default_rng(1).normal(-1.0, 0.5, size=len(fsa.param_names()))

    def evaluate(nranks, rank, gid):
        dev = W.Device(0)
        if nranks > 1:
            dev.comm_init(nranks, rank, gid)
        b, e = W.shard_range(off, nranks, rank)
        dev.load_model(fsa)
        dev.load_corpus(sym[off[b]:off[e]], off[b:e + 1] - off[b], p[b:e])
        rec, pc, used = dev.recognize()
        ll, grad, logq = dev.objective_grad(w)
        ll2, grad2, _ = dev.objective_grad(w, want_logq=False)   # the fused kernel path
        s = dev.allreduce(np.array([float(e - b), rank + 1.0]))
        return used, ll, grad, logq, ll2, grad2, s, (b, e)

    used1, ll1, g1, logq1, _, _, _, _ = evaluate(1, 0, None)
    outs = _run_ranks(4, evaluate)
    logq_all = np.concatenate([o[3] for o in outs])
    np.testing.assert_allclose(logq_all, logq1, rtol=1e-13)
    for used, ll, grad, logq, ll2, grad2, s, _ in outs:
        np.testing.assert_array_equal(used, used1)
        assert _close(ll, ll1, rel=1e-12)
        assert _close(ll2, ll1, rel=1e-12)
        np.testing.assert_allclose(grad, g1, rtol=1e-11, atol=1e-15)
        np.testing.assert_allclose(grad2, g1, rtol=1e-11, atol=1e-15)
        assert s[0] == len(wt) and s[1] == 10.0
    # a mismatched call is refused, not hung
    def bad(nranks, rank, gid):
        dev = W.Device(0)
        dev.comm_init(nranks, rank, gid)
        with pytest.raises(W.WfsaError):
            dev.allreduce(np.zeros(1 + rank))
        return True
    assert all(_run_ranks(2, bad))


def _recognized(syn):
    """the corpus cut to recognized strings (bubbles and traversal tiers
    alike), and how many of them run on the traversal tiers"""
    import wfsa_amd as W
    sym, off, wt = syn.corpus()
    dev = W.Device(0)
    dev.load_model(W.Fsa.read_text(syn.wfsa_text))
    dev.load_corpus(sym, off, wt / wt.sum())
    rec, pc, _ = dev.recognize()
    keep = np.flatnonzero(rec == 1)
    strings = [bytes(sym[off[i]:off[i + 1]]) for i in keep]
    sym2 = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    off2 = np.concatenate([[0], np.cumsum([len(x) for x in strings])]).astype(np.int64)
    n_trav = int((dev.string_tiers()[keep] >= 0).sum())
    return sym2, off2, wt[keep] / wt[keep].sum(), n_trav


def test_rmin_column_across_ranks():
    """the rmin info column (QuasiNewtonLearner::GetOptimizationInfo,
    src/QuasiNewtonLearner.cpp:80-84) across ranks: value and the global
    index of the string holding the path equal the one-context run, in the
    host steps and the device-resident loop"""
    import wfsa_amd as W
    syn = W.Synthetic(**FAMILIES["ambiguous"])
    sym, off, wt = _with_unrecognized(*syn.corpus())
    fsa = W.Fsa.read_text(syn.wfsa_text)

    def learn(nranks, rank, gid):
        lrn = W.QuasiNewtonLearner(0)
        if nranks > 1:
            lrn.SetCommunicator(nranks, rank, gid)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        rows = [lrn.OptimizationStep(1.0, -1.0)[0] for _ in range(2)]
        return rows + lrn.Run(4, 1.0, -1.0)

    rows1 = learn(1, 0, None)
    assert all(r[6] >= 0 and 0 < r[5] < 1 for r in rows1)   # ambiguous strings exist
    for rows in _run_ranks(3, learn):
        for a, q in zip(rows, rows1):
            for u, v in zip(a[:7], q[:7]):
                assert _close(u, v, rel=1e-10, atol=1e-13)


def test_hessian_across_ranks():
    """HessianLearner with 2 and 3 ranks: the H_f pattern is the union of the
    ranks' patterns (bubbles and traversal strings), the values are
    all-reduced; device values and every
    epoch row (KL, residuals, inertia, lambda_min, rmin) equal one context"""
    import wfsa_amd as W
    syn = W.Synthetic(seed=3, n_states=20, degree=4, vocab=6, emissions=2, n_strings=300, max_len=12)
    sym, off, p, n_trav = _recognized(syn)
    assert n_trav > 0
    fsa = W.Fsa.read_text(syn.wfsa_text)
    w = np.random.default_rng(1).normal(-1.0, 0.3, size=len(fsa.param_names()))
    syn2 = W.Synthetic(seed=3, n_states=16, degree=3, vocab=8, emissions=1, n_strings=2000, max_len=16)
    sym2, off2, p2, _ = _recognized(syn2)
    fsa2 = W.Fsa.read_text(syn2.wfsa_text)

    def hf(nranks, rank, gid):
        dev = W.Device(0)
        if nranks > 1:
            dev.comm_init(nranks, rank, gid)
        b, e = W.shard_range(off, nranks, rank)
        dev.load_model(fsa)
        dev.load_corpus(sym[off[b]:off[e]], off[b:e + 1] - off[b], p[b:e])
        dev.recognize()
        pairs = dev.hf_setup()
        return [tuple(x) for x in pairs], dev.hf_eval(w)

    def learn(nranks, rank, gid):
        lrn = W.HessianLearner(0)
        if nranks > 1:
            lrn.SetCommunicator(nranks, rank, gid)
        lrn.BuildFromPacked(fsa2, sym2, off2, p2)
        lrn.Finalize()
        return np.array(lrn.run(flags=31, epochs=6, tol=1e-13)), lrn.x()

    pairs1, vals1 = hf(1, 0, None)
    rows1, x1 = learn(1, 0, None)
    for k in (2, 3):
        for pairs, vals in _run_ranks(k, hf):
            assert pairs == pairs1
            np.testing.assert_allclose(vals, vals1, rtol=1e-11, atol=1e-15)
        for rows, x in _run_ranks(k, learn):
            assert rows.shape == rows1.shape
            assert len(rows1) == 6
            np.testing.assert_allclose(rows, rows1, rtol=1e-8, atol=1e-10)
            np.testing.assert_allclose(x, x1, rtol=1e-9, atol=1e-11)


_LONG_EDGE_WFSA = "\n".join(
    ["", "^", "$", "^  0", "^ P0 0 Q 0 S 0"]
    + [line for i in range(9) for line in (f"P{i}  0 z 0", f"P{i} P{i + 1} 0 $ 0")]
    + ["P9 a 0 z 0", "P9 R 0 $ 0", "Q a 0 c 0", "Q R 0 $ 0", "R b 0 d 0", "R $ 0 S 0", "S c 0 d 0", "S R 0 $ 0"]
) + "\n"


def test_hf_setup_capacity_on_one_shard_fails_every_rank():
    """the H_f set-up's limit on one shard only: a bubble edge
    through an epsilon chain carries ~20 parameters (more than 8) in the
    last rank's strings alone; every rank fails with WFSA_ERR_CAPACITY and
    none is left waiting in a later collective"""
    import wfsa_amd as W
    fsa = W.Fsa.read_text(_LONG_EDGE_WFSA)
    strings = [b"cb", b"cd", b"db", b"dd", b"ab"]
    sym = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    off = np.concatenate([[0], np.cumsum([len(s) for s in strings])]).astype(np.int64)
    p = np.full(len(strings), 1.0 / len(strings))
    assert W.shard_range(off, 2, 1)[0] > 0 and W.shard_range(off, 2, 1)[1] == len(strings)   # "ab" on rank 1

    def hf(nranks, rank, gid):
        dev = W.Device(0)
        dev.comm_init(nranks, rank, gid)
        b, e = W.shard_range(off, nranks, rank)
        dev.load_model(fsa)
        dev.load_corpus(sym[off[b]:off[e]], off[b:e + 1] - off[b], p[b:e])
        dev.recognize()
        with pytest.raises(W.WfsaError) as err:
            dev.hf_setup()
        return err.value.code, str(err.value)

    import time
    t0 = time.time()
    outs = _run_ranks(2, hf)
    assert time.time() - t0 < 60
    codes = [c for c, _ in outs]
    assert codes[0] == codes[1] and codes[0] != 0
    assert "another rank" in outs[0][1] and "parameters" in outs[1][1]


def test_dense_path_across_ranks_with_rmin(monkeypatch):
    """the dense fp64 path across 2 ranks (each rank's row slots hold its
    shard; [LL, grad] summed per step) with the rmin column on -- its (min, +)
    pass per rank, then the global minimum and string index: the host steps
    and the device loop equal one context"""
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_DENSE", "1")
    syn = W.Synthetic(n_states=16, degree=1, vocab=8, emissions=2, dense=True, n_strings=300, max_len=9, seed=21)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)

    def learn(nranks, rank, gid):
        lrn = W.QuasiNewtonLearner(0)
        if nranks > 1:
            lrn.SetCommunicator(nranks, rank, gid)
        lrn.set_info_rmin(True)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        assert lrn.stats()["dense"] == 1
        rows = [lrn.OptimizationStep(1.0, -1.0)[0] for _ in range(2)]
        return rows + lrn.Run(4, 1.0, -1.0), lrn.x()

    rows1, x1 = learn(1, 0, None)
    assert all(r[6] >= 0 and 0 < r[5] < 1 for r in rows1)
    for rows, x in _run_ranks(2, learn):
        assert len(rows) == len(rows1) == 6
        for a, q in zip(rows, rows1):
            for u, v in zip(a[:7], q[:7]):
                assert _close(u, v, rel=1e-10, atol=1e-13)
        np.testing.assert_allclose(x, x1, rtol=1e-10, atol=1e-12)
