"""The timed path at BASELINE size, and determinism.

* c3 (BASELINE.json configs[2]): 1M family-A strings through the
  path bench.py times -- the device-resident QN loop (stream kernel with the
  bubbles fused, then the fused QN step that sums the bubble slots itself) --
  against the reference algorithm restated (ENUM: BFS path enumeration + the
  P/M SpMV chain, src/Learner.cpp:276-348,515-553,
  src/QuasiNewtonLearner.cpp:93-125): KL and the full gradient by name at the
  initial weights, the QN update's x, and then log q of every string and the
  host-binding objective_grad (wfsa_dev_objective_grad without log q) at the
  updated weights.
* determinism: the same evaluation twice, and the same 20-step run twice,
  give the same bits (the reference, mkl_sequential, is deterministic).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b, rel, atol=1e-13):
    return abs(a - b) <= max(atol, rel * max(abs(a), abs(b)))


def _by_name(names, values):
    return dict(zip(names, values))


@pytest.fixture(scope="module")
def c3():
    import wfsa_amd as W
    from oracle import ENUM, Oracle
    syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=1_000_000, max_len=128, seed=1)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    o = Oracle.from_arrays(syn.wfsa_text, sym, off, wt, mode=ENUM, max_paths=10_000_000)
    return syn, fsa, sym, off, wt, o


def test_c3_full_size_timed_path_matches_enum(c3):
    import wfsa_amd as W
    syn, fsa, sym, off, wt, o = c3
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(False)   # the bench's headline step
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    o.qn_init(7)
    st = lrn.stats()
    assert st["compiled_strings"] == len(wt) and st["n_bubbles"] > 100_000   # bubbles exercised
    dn, on = lrn.param_names(), o.param_names()
    assert sorted(dn) == sorted(on)
    # one device-resident step: row 0 is evaluated at the initial weights
    rows = lrn.Run(1, 1.0, -1.0)
    kl_o, ll_o = o.objective_grad()
    g_o = _by_name(on, o.grad())
    info_o = o.qn_step(1.0)
    assert _close(rows[0][0], kl_o, rel=1e-11)
    for a, b in zip(rows[0][:5], info_o[:5]):
        assert _close(a, b, rel=1e-9, atol=1e-12)
    g_d = _by_name(dn, lrn.last_grad())
    keys = sorted(g_o)
    np.testing.assert_allclose([g_d[k] for k in keys], [g_o[k] for k in keys], rtol=1e-10, atol=1e-15)
    x_d, x_o = _by_name(dn, lrn.x()), _by_name(on, o.x())
    np.testing.assert_allclose([x_d[k] for k in keys], [x_o[k] for k in keys], rtol=1e-10, atol=1e-13)
    # at the updated weights: every string's log q, and the host binding's
    # objective_grad (fused bubbles + reduction kernel)
    kl1_o, ll1_o = o.objective_grad()
    g1_o = _by_name(on, o.grad())
    kl1, g1, _ = lrn.objective_grad()
    assert _close(kl1, kl1_o, rel=1e-11)
    g1_d = _by_name(dn, g1)
    np.testing.assert_allclose([g1_d[k] for k in keys], [g1_o[k] for k in keys], rtol=1e-10, atol=1e-15)
    kl2, _, logq = lrn.objective_grad(want_logq=True)
    np.testing.assert_allclose(logq, o.logq(), rtol=1e-12, atol=1e-12)
    assert _close(kl2, kl1_o, rel=1e-11)


def _compiled_only(W, fsa, sym, off, wt):
    """the strings that compile (stream + bubbles; the traversal strings have
    their own bitwise test below)"""
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, wt / wt.sum())
    dev.recognize()
    dev.objective_grad(np.full(len(fsa.param_names()), -1.0), want_logq=False)
    keep = np.flatnonzero(dev.string_tiers() < 0)
    lens = np.diff(off)[keep]
    noff = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nsym = np.concatenate([sym[off[i]:off[i + 1]] for i in keep]).astype(np.uint8)
    return nsym, noff, wt[keep]


def _ambiguous_learner(W, seed=4):
    syn = W.Synthetic(n_states=256, degree=8, vocab=16, emissions=1, n_strings=40_000, max_len=64, seed=seed)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    sym, off, wt = _compiled_only(W, fsa, sym, off, wt)
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(False)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    return lrn


def test_evaluations_and_runs_are_bitwise_reproducible():
    import wfsa_amd as W
    lrn = _ambiguous_learner(W)
    lrn.Init(7)
    st = lrn.stats()
    assert st["n_bubbles"] > 1000
    assert st["fallback_strings"] == 0 and st["tier1_strings"] == 0
    kl_a, g_a, _ = lrn.objective_grad()
    kl_b, g_b, _ = lrn.objective_grad()
    assert kl_a == kl_b
    assert np.array_equal(g_a, g_b)
    runs = []
    for _ in range(2):
        lrn.Init(7)
        rows = lrn.Run(20, 1.0, -1.0)
        runs.append((np.array(rows), lrn.x(), lrn.last_grad()))
    assert np.array_equal(runs[0][0], runs[1][0])
    assert np.array_equal(runs[0][1], runs[1][1])
    assert np.array_equal(runs[0][2], runs[1][2])
    # a second context over the same corpus (a fresh compilation) agrees bitwise too
    other = _ambiguous_learner(W)
    other.Init(7)
    kl_c, g_c, _ = other.objective_grad()
    assert kl_c == kl_a and np.array_equal(g_c, g_a)


def test_halting_run_leaves_consistent_state():
    """after a run that halts, an evaluation at the final x equals a fresh one"""
    import wfsa_amd as W
    lrn = _ambiguous_learner(W, seed=6)
    lrn.Init(7)
    rows = lrn.Run(200, 1.0, 1e-3)
    assert 0 < len(rows) < 200
    x = lrn.x()
    kl, g, _ = lrn.objective_grad()
    fresh = _ambiguous_learner(W, seed=6)
    fresh.Init(7)
    fresh.set_x(x)
    kl_f, g_f, _ = fresh.objective_grad()
    assert kl == kl_f and np.array_equal(g, g_f)


def test_traversal_strings_are_bitwise_reproducible():
    """family B strings run on the wave kernel, whose waves draw strings from a
    work counter; its gradient and log-likelihood are fixed-point sums, so the
    evaluation and a QN run give the same bits every time and in a second
    context"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=8, vocab=16, emissions=4, n_strings=3000, max_len=128, seed=2)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)

    def learner():
        lrn = W.QuasiNewtonLearner(0)
        lrn.set_info_rmin(False)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        return lrn

    lrn = learner()
    st = lrn.stats()
    assert st["wave_strings"] > 1000
    evals = [lrn.objective_grad() for _ in range(3)]
    for kl, g, _ in evals[1:]:
        assert kl == evals[0][0]
        assert np.array_equal(g, evals[0][1])
    runs = []
    for _ in range(2):
        lrn.Init(7)
        rows = lrn.Run(5, 1.0, -1.0)
        runs.append((np.array(rows), lrn.x()))
    assert np.array_equal(runs[0][0], runs[1][0])
    assert np.array_equal(runs[0][1], runs[1][1])
    other = learner()
    kl_c, g_c, _ = other.objective_grad()
    assert kl_c == evals[0][0] and np.array_equal(g_c, evals[0][1])
