"""BASELINE configs[3] ("c4": the 1024-state family-A WFSA, 10M strings
sharded over 8 GPUs, one all-reduce of [LL, grad] per step) at its full size
on one GPU.

Eight contexts of this process form an in-process group
(wfsa_dev_comm_local_id), one thread per rank, each keeping its 1.25M-string
shard of the 10M-string corpus -- exactly the rank code an 8-GPU RCCL job
runs (Learner::BuildPaths' Sigma-length split, the statistics and used-mask
all-reduces, the constant trivial gradient reduced once, the per-step
all-reduce inside the device QN loop).  The result must equal one context
holding the whole corpus, and both must equal the ENUM oracle (the
reference's BuildPaths + SpMV chain, src/Learner.cpp:276-553 and
src/QuasiNewtonLearner.cpp:93-201) on the same 10M strings.  The loop being
sharded is the reference's per-string loop, src/Learner.cpp:332-343."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_RANKS = 8
STRINGS = 10_000_000
STEPS = 5


def _close(a, b, rel, atol=1e-13):
    return abs(a - b) <= max(atol, rel * max(abs(a), abs(b)))


@pytest.fixture(scope="module")
def c4():
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=STRINGS, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    return syn, sym, off, wt, W.Fsa.read_text(syn.wfsa_text)


def _learn(c4, nranks, rank, gid):
    import wfsa_amd as W
    syn, sym, off, wt, fsa = c4
    lrn = W.QuasiNewtonLearner(0)
    if nranks > 1:
        lrn.SetCommunicator(nranks, rank, gid)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    kl, g, _ = lrn.objective_grad()
    rows = lrn.Run(STEPS, 1.0, -1.0)   # the device-resident loop (per-step all-reduce across ranks)
    out = dict(info=lrn.info(), kl=kl, grad=g, rows=rows, x=lrn.x(), trim=lrn.trimmed_index(),
               names=lrn.param_names(), stats=lrn.stats())
    del lrn
    return out


@pytest.fixture(scope="module")
def one_context(c4):
    return _learn(c4, 1, 0, None)


@pytest.fixture(scope="module")
def ranks(c4):
    import wfsa_amd as W
    gid = W.Device.comm_local_id(N_RANKS)
    with ThreadPoolExecutor(max_workers=N_RANKS) as ex:
        futs = [ex.submit(_learn, c4, N_RANKS, r, gid) for r in range(N_RANKS)]
        return [f.result(timeout=600) for f in futs]


def test_c4_eight_ranks_equal_one_context(c4, one_context, ranks):
    import wfsa_amd as W
    syn, sym, off, wt, fsa = c4
    one = one_context
    sizes = []
    for r, o in enumerate(ranks):
        b, e = W.shard_range(off, N_RANKS, r)
        assert (o["info"]["shard_begin"], o["info"]["shard_end"]) == (b, e)
        sizes.append(e - b)
        for key in ("n_params", "n_constraints", "n_strings", "n_paths", "n_full"):
            assert o["info"][key] == one["info"][key], key
        # corpus statistics are 10M-term sums: per shard, then across the
        # ranks, against one sequential sum -- a different order, n*eps ~ 1e-9
        for key in ("common_support", "plogp", "model_volume"):
            assert _close(o["info"][key], one["info"][key], rel=2e-9), key
        np.testing.assert_array_equal(o["trim"], one["trim"])   # the OR of the shards' used masks
        assert _close(o["kl"], one["kl"], rel=1e-10)
        np.testing.assert_allclose(o["grad"], one["grad"], rtol=1e-10, atol=1e-15)
        assert len(o["rows"]) == len(one["rows"]) == STEPS
        for a, q in zip(o["rows"], one["rows"]):
            for u, v in zip(a[:5], q[:5]):
                assert _close(u, v, rel=1e-10, atol=1e-13)
        np.testing.assert_allclose(o["x"], one["x"], rtol=1e-10, atol=1e-12)
        assert o["stats"]["compiled_strings"] > 0
    assert sum(sizes) == STRINGS
    # ~1.25M strings per rank: the shards are balanced on total length
    assert min(sizes) > 0.95 * STRINGS / N_RANKS and max(sizes) < 1.05 * STRINGS / N_RANKS
    assert sum(o["stats"]["compiled_strings"] + o["stats"]["fallback_strings"] for o in ranks) <= STRINGS


def test_c4_matches_enum_oracle(c4, one_context, ranks):
    """KL and the full gradient at the initial point, and the QuasiNewton
    epochs, against the reference algorithm on the whole 10M-string corpus"""
    from oracle import ENUM, Oracle
    syn, sym, off, wt, fsa = c4
    o = Oracle.from_arrays(syn.wfsa_text, sym, off, wt, mode=ENUM, max_paths=100_000_000)
    o.set_threads(16)
    assert o.info["n_strings"] == one_context["info"]["n_strings"]
    assert o.info["n_paths"] == one_context["info"]["n_paths"]
    assert o.info["n_params"] == one_context["info"]["n_params"]
    o.qn_init(7)
    kl_ref, ll_ref = o.objective_grad()
    g_ref = dict(zip(o.param_names(), o.grad()))
    for res in [one_context, ranks[0], ranks[-1]]:
        assert _close(res["kl"], kl_ref, rel=1e-9)   # (plogp: 10M-term sums in different orders)
        g = np.array([g_ref[n] for n in res["names"]])
        np.testing.assert_allclose(res["grad"], g, rtol=1e-9, atol=1e-14)
    orows = o.qn_run(flags=7, epochs=STEPS, tol=-1.0)
    assert len(orows) == STEPS
    ox = dict(zip(o.param_names(), o.x()))
    for res in [one_context, ranks[0], ranks[-1]]:
        for r, q in zip(res["rows"], orows):
            for a, b in zip(r[:5], q[:5]):
                assert _close(a, b, rel=1e-8, atol=1e-11)
        for n, v in zip(res["names"], res["x"]):
            assert _close(v, ox[n], rel=1e-8, atol=1e-10)
