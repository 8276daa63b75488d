"""GPU parity of traversal tier 2 (wide_kernel: one block per string, alpha
in global scratch) -- the tier for strings whose trellis overflows every LDS
slab, e.g. SURVEY.md 8d "family B" (ambiguous: 1024 states, out-degree 8,
4 of 16 symbols per state).  All tests need a gfx950 device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _close(a, b, rel, atol=1e-13):
    return abs(a - b) <= max(atol, rel * max(abs(a), abs(b)))


def _oracle(text, sym, off, wt, w_by_name):
    from oracle import Oracle, TRELLIS
    o = Oracle.from_arrays(text, sym, off, wt, mode=TRELLIS)
    names = o.full_param_names()
    ll, logq, grad = o.trellis_eval(np.array([w_by_name[n] for n in names]))
    return ll, logq, dict(zip(names, grad))


def _eval(text, sym, off, p, w, monkeypatch, force):
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_TIER2", "1" if force else "0")
    monkeypatch.setenv("WFSA_DENSE", "0")
    fsa = W.Fsa.read_text(text)
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, p)
    rec, pc, used = dev.recognize()
    ll, grad, logq = dev.objective_grad(w)
    return rec, pc, used, ll, grad, logq, dev.stats()


@pytest.mark.parametrize("family", [
    dict(n_states=64, degree=8, vocab=16, emissions=1, n_strings=800, max_len=64),
    dict(n_states=48, degree=6, vocab=8, emissions=3, n_strings=500, max_len=24),
])
def test_tier2_forced_equals_lds_tiers(family, monkeypatch):
    """every string forced onto tier 2 == the LDS tiers / compiled streams"""
    import wfsa_amd as W
    syn = W.Synthetic(seed=17, **family)
    sym, off, wt = syn.corpus()
    p = wt / wt.sum()
    names = W.Fsa.read_text(syn.wfsa_text).param_names()
    w = np.random.default_rng(4).normal(-1.2, 0.6, size=len(names))
    r0, pc0, u0, ll0, g0, lq0, st0 = _eval(syn.wfsa_text, sym, off, p, w, monkeypatch, False)
    r2, pc2, u2, ll2, g2, lq2, st2 = _eval(syn.wfsa_text, sym, off, p, w, monkeypatch, True)
    assert st2["tier2_strings"] == len(wt) and st0["tier2_strings"] == 0
    np.testing.assert_array_equal(r2, r0)
    np.testing.assert_array_equal(pc2, pc0)
    np.testing.assert_array_equal(u2, u0)
    np.testing.assert_allclose(lq2, lq0, rtol=1e-12)
    assert _close(ll2, ll0, rel=1e-12)
    np.testing.assert_allclose(g2, g0, rtol=1e-10, atol=1e-16)


def test_family_b_against_oracle(monkeypatch):
    """family B strings overflow the LDS slabs and run on tier 2"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=8, vocab=16, emissions=4, n_strings=300, max_len=128, seed=2)
    sym, off, wt = syn.corpus()
    p = wt / wt.sum()
    names = W.Fsa.read_text(syn.wfsa_text).param_names()
    w = np.random.default_rng(6).normal(-1.5, 0.5, size=len(names))
    rec, pc, used, ll, grad, logq, st = _eval(syn.wfsa_text, sym, off, p, w, monkeypatch, False)
    assert rec.all()
    assert st["tier2_strings"] > 0
    print(f"tier2 {st['tier2_strings']} of {len(wt)}, compiled {st['compiled_strings']}")
    oll, ologq, ograd = _oracle(syn.wfsa_text, sym, off, wt, dict(zip(names, w)))
    np.testing.assert_allclose(logq, ologq, rtol=1e-11)
    assert _close(ll, oll, rel=1e-11)
    np.testing.assert_allclose(grad, [ograd[n] for n in names], rtol=1e-9, atol=1e-15)


def test_tier2_path_counts_match_enumeration(monkeypatch):
    import wfsa_amd as W
    from oracle import ENUM, Oracle
    syn = W.Synthetic(n_states=48, degree=6, vocab=8, emissions=3, n_strings=400, max_len=12, seed=5)
    sym, off, wt = syn.corpus()
    names = W.Fsa.read_text(syn.wfsa_text).param_names()
    rec, pc, used, *_ = _eval(syn.wfsa_text, sym, off, wt / wt.sum(), np.zeros(len(names)), monkeypatch, True)
    o = Oracle.from_arrays(syn.wfsa_text, sym, off, wt, mode=ENUM, max_paths=10_000_000)
    np.testing.assert_array_equal(pc, o.path_counts().astype(np.float64))
    oused = {n for n, t in zip(o.full_param_names(), o.trimmed_index()) if t != -2}
    assert {n for n, u in zip(names, used) if u} == oused


@pytest.mark.parametrize("family", [
    dict(n_states=256, degree=8, vocab=16, emissions=4, n_strings=600, max_len=48),    # D up to ~80: 4 nodes/lane
    dict(n_states=1024, degree=8, vocab=16, emissions=4, n_strings=300, max_len=40),   # famB shape: 6 nodes/lane
])
def test_wave_pull_equals_push_and_repeats(family, monkeypatch):
    """the traversal strings' pull kernel (wave_pull_kernel, the default) and
    round 2's push kernel (wide2_kernel, WFSA_PULL=0) give the same log q,
    log-likelihood and gradient; the pull kernel's evaluation repeats bit for
    bit (fixed-order node sums, fixed-point gradient)"""
    import wfsa_amd as W
    syn = W.Synthetic(seed=23, **family)
    sym, off, wt = syn.corpus()
    p = wt / wt.sum()
    names = W.Fsa.read_text(syn.wfsa_text).param_names()
    w = np.random.default_rng(8).normal(-1.4, 0.4, size=len(names))
    monkeypatch.setenv("WFSA_PULL", "0")
    *_, llp, gp, lqp, stp = _eval(syn.wfsa_text, sym, off, p, w, monkeypatch, False)
    assert stp["wave_strings"] > 0 and stp["wave_pull"] == 0
    monkeypatch.setenv("WFSA_PULL", "1")
    import wfsa_amd as W2
    fsa = W2.Fsa.read_text(syn.wfsa_text)
    dev = W2.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, p)
    dev.recognize()
    ll1, g1, lq1 = dev.objective_grad(w)
    ll2, g2, lq2 = dev.objective_grad(w)
    st = dev.stats()
    assert st["wave_strings"] == stp["wave_strings"] and st["wave_pull"] in (4, 6, 8)
    assert ll1 == ll2 and np.array_equal(g1, g2) and np.array_equal(lq1, lq2)
    np.testing.assert_allclose(lq1, lqp, rtol=1e-12)
    assert _close(ll1, llp, rel=1e-12)
    np.testing.assert_allclose(g1, gp, rtol=1e-10, atol=1e-16)


@pytest.mark.parametrize("n_strings,max_len", [(10_000, 128), (2_000, 600)])
def test_wave_pull_fixed_point_gradient_at_scale(n_strings, max_len, monkeypatch):
    """family B at scale: the pull kernel's 64-bit fixed-point gradient
    (resolution 2^-F, F from max_len and parameters per edge) against tier 2's
    fp64 sums (WFSA_WIDE2=0: block per string, pinned to the oracle by the
    tests above) element by element.  Every credit is -p * posterior <= 0, so
    no entry cancels: a relative bound holds for each nonzero entry, and the
    zero entries must agree exactly."""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=8, vocab=16, emissions=4, n_strings=n_strings, max_len=max_len, seed=31)
    sym, off, wt = syn.corpus()
    p = wt / wt.sum()
    names = W.Fsa.read_text(syn.wfsa_text).param_names()
    w = np.random.default_rng(9).normal(-1.5, 0.5, size=len(names))
    monkeypatch.setenv("WFSA_WIDE2", "0")
    *_, ll0, g0, lq0, st0 = _eval(syn.wfsa_text, sym, off, p, w, monkeypatch, False)
    monkeypatch.setenv("WFSA_WIDE2", "1")
    *_, ll1, g1, lq1, st1 = _eval(syn.wfsa_text, sym, off, p, w, monkeypatch, False)
    assert st0["wave_strings"] == 0 and st1["wave_strings"] > 0.9 * n_strings
    assert (g0 <= 0).all() and (g1 <= 0).all()
    nz = g0 != 0
    np.testing.assert_array_equal(g1[~nz], 0.0)
    rel = np.abs(g1[nz] - g0[nz]) / np.abs(g0[nz])
    print(f"{n_strings} strings, max len {int(np.diff(off).max())}: worst rel {rel.max():.2e}, "
          f"{int(nz.sum())} nonzero entries, smallest |g| {np.abs(g0[nz]).min():.2e}")
    assert rel.max() <= 1e-9
    np.testing.assert_allclose(lq1, lq0, rtol=1e-12)
    assert _close(ll1, ll0, rel=1e-12)
