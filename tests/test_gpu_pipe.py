"""The pipelined device QN loop (wfsa_dev_qn_run when every string is
compiled, one rank, no rmin column): bubbles + QN update on one stream, the
stream pass + the step's finish on a second one, weights double-buffered by
step parity.  It must give the same trajectory as the single-stream loop
(WFSA_PIPE=0): bitwise in x and the gradient columns (the same bubble slots
and summation order), the KL column to rounding (the log-likelihood partials
are grouped differently); halting at the same epoch; and the weights after a
run equal to those of x.  All tests need a gfx950 device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _learner(monkeypatch, pipe, syn, halt_tol=-1.0, steps=12):
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_PIPE", "1" if pipe else "0")   # (opt-in path vs the default)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(False)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    rows = np.array(lrn.Run(steps, 1.0, halt_tol))
    return lrn, rows


@pytest.mark.parametrize("family", [
    dict(n_states=64, degree=8, vocab=16, emissions=1, n_strings=3000, max_len=64, seed=5),
    dict(n_states=256, degree=8, vocab=64, emissions=1, n_strings=20000, max_len=96, seed=2),
])
def test_pipelined_loop_equals_single_stream(family, monkeypatch):
    import wfsa_amd as W
    syn = W.Synthetic(**family)
    a, ra = _learner(monkeypatch, True, syn)
    b, rb = _learner(monkeypatch, False, syn)
    st = a.stats()
    assert st["fallback_strings"] == 0 and st["n_bubbles"] > 0
    assert ra.shape == rb.shape == (12, a.width)
    np.testing.assert_array_equal(ra[:, 1:5], rb[:, 1:5])    # graderr, g_min, g_max, lambda_min
    np.testing.assert_allclose(ra[:, 0], rb[:, 0], rtol=1e-13)  # KL
    np.testing.assert_array_equal(a.x(), b.x())
    # the weights left on the device are x's: the next evaluation equals a fresh one
    kl_a, g_a, _ = a.objective_grad()
    kl_b, g_b, _ = b.objective_grad()
    assert abs(kl_a - kl_b) <= 1e-13 * abs(kl_b)
    np.testing.assert_allclose(g_a, g_b, rtol=1e-13, atol=1e-16)
    # a second run continues from there
    ra2 = np.array(a.Run(4, 1.0, -1.0))
    rb2 = np.array(b.Run(4, 1.0, -1.0))
    np.testing.assert_array_equal(ra2[:, 1:5], rb2[:, 1:5])
    np.testing.assert_array_equal(a.x(), b.x())


def test_pipelined_loop_halts_at_the_same_epoch(monkeypatch):
    import wfsa_amd as W
    syn = W.Synthetic(n_states=64, degree=8, vocab=16, emissions=1, n_strings=3000, max_len=64, seed=5)
    a, ra = _learner(monkeypatch, True, syn, halt_tol=1e-3, steps=60)
    b, rb = _learner(monkeypatch, False, syn, halt_tol=1e-3, steps=60)
    assert len(ra) == len(rb) < 60
    np.testing.assert_array_equal(ra[:, 1:5], rb[:, 1:5])
    np.testing.assert_array_equal(a.x(), b.x())
