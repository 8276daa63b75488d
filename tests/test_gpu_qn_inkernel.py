"""The QN update inside the stream kernel (fb_kernels.hpp QnWave).

The device-resident QN loop (src/main.cpp:276-303 run natively; one
QuasiNewtonLearner::OptimizationStep per step, src/QuasiNewtonLearner.cpp:
162-201) runs each step's update in the stream kernel's QN waves, which wait
for every block's bubble slots by an arrival counter and read them
write-through.  It must give the same bits as the separate qn_step_kernel
(WFSA_QN_INKERNEL=0) -- rows, x, lambda-dependent trajectory, the last
gradient -- over runs of any length (the weights alternate between two
buffers by step parity), across consecutive runs, and through a halt.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


# where step e's finish (its log-likelihood sum, halt test and info row) runs:
# "last" (default): in launch e + 1's finish wave, the Run's last launch
# finishing its own step; "next": always in the next launch, the Run's last
# step by a finish kernel of its own (WFSA_QN_LAST_SELF=0)
FINISH = ["last", "next"]


def _learner(W, fsa, sym, off, wt, monkeypatch, inkernel, finish="last", rmin=False):
    if inkernel is None:   # the cover rule decides (the product default)
        monkeypatch.delenv("WFSA_QN_INKERNEL", raising=False)
    else:
        monkeypatch.setenv("WFSA_QN_INKERNEL", "1" if inkernel else "0")
    monkeypatch.setenv("WFSA_QN_LAST_SELF", "0" if finish == "next" else "1")
    lrn = W.QuasiNewtonLearner(0)
    lrn.set_info_rmin(rmin)
    lrn.BuildFromPacked(fsa, sym, off, wt)
    lrn.Finalize()
    lrn.Init(7)
    return lrn


def _corpus(W, compiled_only=False, **kw):
    syn = W.Synthetic(**kw)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    if compiled_only:   # the strings that compile (the others make the loop take the separate kernel)
        dev = W.Device(0)
        dev.load_model(fsa)
        dev.load_corpus(sym, off, wt / wt.sum())
        dev.recognize()
        dev.objective_grad(np.full(len(fsa.param_names()), -1.0), want_logq=False)
        keep = np.flatnonzero(dev.string_tiers() < 0)
        lens = np.diff(off)[keep]
        off_k = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        sym = np.concatenate([sym[off[i]:off[i + 1]] for i in keep]).astype(np.uint8)
        off, wt = off_k, wt[keep]
    return fsa, sym, off, wt


FAMILIES = {
    # family A at c3's shape, fewer strings: every string compiles, bubbles at cuts
    "familyA": dict(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=200_000, max_len=128, seed=1),
    # many bubbles per string and popular parameters (large slot chunks per member)
    "ambiguous": dict(n_states=256, degree=8, vocab=16, emissions=1, n_strings=8_000, max_len=64, seed=4,
                      compiled_only=True),
}


@pytest.mark.parametrize("rmin", [False, True], ids=["", "rmin"])
@pytest.mark.parametrize("finish", FINISH)
@pytest.mark.parametrize("family", sorted(FAMILIES))
def test_inkernel_update_equals_qn_step_kernel(family, finish, rmin, monkeypatch):
    """finish: where each step's finish runs (FINISH above); the runs of odd
    and even length below exercise the Run's last launch finishing itself.
    rmin: the info rows' rmin column (the product default), folded into the
    stream kernel (RminFold: one-bubble strings' candidates at once, a
    multi-bubble string's sum by its last bubble's arrival) against the
    separate strings pass -- the same (value, string) in every row"""
    import wfsa_amd as W
    fsa, sym, off, wt = _corpus(W, **FAMILIES[family])
    a = _learner(W, fsa, sym, off, wt, monkeypatch, True, finish, rmin)
    b = _learner(W, fsa, sym, off, wt, monkeypatch, False, rmin=rmin)
    # runs of odd and even length, back to back: the weight parity and the
    # arrival counters carry across runs
    # one step first: the gradient the update used and the updated x
    r1a, r1b = a.Run(1, 1.0, -1.0), b.Run(1, 1.0, -1.0)
    np.testing.assert_array_equal(a.last_grad(), b.last_grad())
    np.testing.assert_array_equal(a.x(), b.x())
    np.testing.assert_array_equal(np.array(r1a), np.array(r1b))
    a.Init(7)
    b.Init(7)
    ra = a.Run(3, 1.0, -1.0) + a.Run(4, 1.0, -1.0) + a.Run(1, 1.0, -1.0) + a.Run(12, 1.0, -1.0)
    sa = a.stats()
    rb = b.Run(20, 1.0, -1.0)
    # (the rmin column rides in the stream kernel only with the bubbles fused
    # into it: the heavily ambiguous family's bubbles outnumber its waves)
    if not (rmin and family == "ambiguous"):
        assert sa["qn_inkernel_waves"] > 0 and sa["qn_batches"] > 0, "the in-kernel update did not run"
    assert b.stats()["qn_inkernel_waves"] == 0
    ra, rb = np.array(ra), np.array(rb)
    if rmin:   # an ambiguous corpus: the column is a real minimum, not the no-string default
        assert (ra[:, 6] >= 0).all() and (ra[:, 5] > 0).all(), ra[:, 5:7]
    bad = sorted(set(int(r) for r, _ in np.argwhere(ra != rb)))
    assert not bad, f"rows {bad} differ: {ra[bad].tolist()} vs {rb[bad].tolist()}"
    np.testing.assert_array_equal(a.x(), b.x())
    np.testing.assert_array_equal(a.last_grad(), b.last_grad())
    # the weights after the run (parity buffers folded back): the next
    # evaluation agrees with the other learner's bit for bit
    kl_a, g_a, _ = a.objective_grad()
    kl_b, g_b, _ = b.objective_grad()
    assert kl_a == kl_b and np.array_equal(g_a, g_b)


def test_inkernel_update_matches_host_steps(monkeypatch):
    """the in-kernel loop against the host QN update (OptimizationStep one by
    one: wfsa_dev_objective_grad + QuasiNewtonLearner.cpp's update on the host)"""
    import wfsa_amd as W
    fsa, sym, off, wt = _corpus(W, **FAMILIES["ambiguous"])
    a = _learner(W, fsa, sym, off, wt, monkeypatch, True)
    b = _learner(W, fsa, sym, off, wt, monkeypatch, True)
    rows_a = a.Run(8, 1.0, -1.0)
    assert a.stats()["qn_inkernel_waves"] > 0
    rows_b = [b.OptimizationStep(1.0, -1.0)[0] for _ in range(8)]
    for r, q in zip(rows_a, rows_b):
        for u, v in zip(r[:5], q[:5]):
            assert abs(u - v) <= max(1e-14, 1e-11 * max(abs(u), abs(v)))
    np.testing.assert_allclose(a.x(), b.x(), rtol=1e-11, atol=1e-13)


@pytest.mark.parametrize("rmin", [False, True], ids=["", "rmin"])
@pytest.mark.parametrize("finish", FINISH)
def test_inkernel_halting_run(finish, rmin, monkeypatch):
    """a halting run stops at the same epoch with the same rows and state as
    the separate kernel; the steps enqueued after the halt are skipped and
    the next run starts cleanly"""
    import wfsa_amd as W
    fsa, sym, off, wt = _corpus(W, **FAMILIES["ambiguous"])
    a = _learner(W, fsa, sym, off, wt, monkeypatch, True, finish, rmin)
    b = _learner(W, fsa, sym, off, wt, monkeypatch, False, rmin=rmin)
    ra = a.Run(200, 1.0, 1e-3)
    rb = b.Run(200, 1.0, 1e-3)
    assert 0 < len(ra) < 200
    assert np.array_equal(np.array(ra), np.array(rb))
    assert np.array_equal(a.x(), b.x())
    kl_a, g_a, _ = a.objective_grad()
    kl_b, g_b, _ = b.objective_grad()
    assert kl_a == kl_b and np.array_equal(g_a, g_b)
    # after the halt: a fresh start runs in-kernel again and matches
    a.Init(7)
    b.Init(7)
    assert np.array_equal(np.array(a.Run(5, 1.0, -1.0)), np.array(b.Run(5, 1.0, -1.0)))
    assert np.array_equal(a.x(), b.x())


MIXED = {
    # strings that do not compile (traversal kernels) beside compiled ones
    "mixed": dict(n_states=256, degree=8, vocab=16, emissions=1, n_strings=8_000, max_len=64, seed=4),
    # (single-emission states: the delta stream format, which the in-kernel update needs)
    "mixedA": dict(n_states=1024, degree=8, vocab=16, emissions=1, n_strings=50_000, max_len=128, seed=2),
}


@pytest.mark.parametrize("rmin", [False, True], ids=["", "rmin"])
@pytest.mark.parametrize("family", sorted(MIXED))
def test_inkernel_update_with_traversal_strings(family, rmin, monkeypatch):
    """a corpus with traversal strings keeps the one-launch
    step.  The traversal kernels run before the stream kernel (the per-edge
    weights from the edge-weights kernel), their gradient in `out` joins each
    member's sum in the QN waves in qn_step_kernel's order (traversal part,
    trivial words, slots) and their ll partials keep their slots -- so every
    row, x and the last gradient equal the separate kernel's bit for bit"""
    import wfsa_amd as W
    fsa, sym, off, wt = _corpus(W, **MIXED[family])
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, wt / wt.sum())
    dev.recognize()
    dev.objective_grad(np.full(len(fsa.param_names()), -1.0), want_logq=False)
    tiers = dev.string_tiers()
    assert (tiers >= 0).any() and (tiers < 0).any(), "the corpus must mix compiled and traversal strings"
    del dev
    a = _learner(W, fsa, sym, off, wt, monkeypatch, True, rmin=rmin)
    b = _learner(W, fsa, sym, off, wt, monkeypatch, False, rmin=rmin)
    ra = a.Run(3, 1.0, -1.0) + a.Run(6, 1.0, -1.0)
    rb = b.Run(9, 1.0, -1.0)
    if not rmin:
        assert a.stats()["qn_inkernel_waves"] > 0, "the in-kernel update did not run"
    assert b.stats()["qn_inkernel_waves"] == 0
    ra, rb = np.array(ra), np.array(rb)
    bad = sorted(set(int(r) for r, _ in np.argwhere(ra != rb)))
    assert not bad, f"rows {bad} differ: {ra[bad].tolist()} vs {rb[bad].tolist()}"
    np.testing.assert_array_equal(a.x(), b.x())
    np.testing.assert_array_equal(a.last_grad(), b.last_grad())


def test_poll_timeout_fails_the_run(monkeypatch):
    """a QN wave whose arrival wait gives up must not let
    the step pass as updated.  WFSA_FAULT_QN_POLL=1 makes the first QN wave
    wait for one arrival too many and give up after a few polls: its
    constraints keep x / lambda while the other waves update theirs, so the
    run must fail with the timeout (the finish used to drop the wave's NaN
    partials in fmin / fmax and report the step as run)"""
    import wfsa_amd as W
    fsa, sym, off, wt = _corpus(W, **FAMILIES["familyA"])
    monkeypatch.setenv("WFSA_FAULT_QN_POLL", "1")
    a = _learner(W, fsa, sym, off, wt, monkeypatch, True)
    with pytest.raises(W.WfsaError, match="timed out"):
        a.Run(4, 1.0, -1.0)
    assert a.stats()["qn_inkernel_waves"] > 0   # the in-kernel update was the one that ran


def test_cover_rule_takes_two_kernels_for_short_streams(monkeypatch):
    """with WFSA_QN_INKERNEL unset the one-launch step is taken only when the
    deal's mean stream rows per wave cover the bubble tail (wfsa_dev.hip
    qw_cover): a 200k-string family-A corpus (~3 rows per wave) steps with
    the two kernels, bit for bit what the forced one-launch step gives"""
    import wfsa_amd as W
    fsa, sym, off, wt = _corpus(W, **FAMILIES["familyA"])
    a = _learner(W, fsa, sym, off, wt, monkeypatch, None)
    ra = a.Run(4, 1.0, -1.0)
    assert a.stats()["qn_inkernel_waves"] == 0
    b = _learner(W, fsa, sym, off, wt, monkeypatch, True)
    rb = b.Run(4, 1.0, -1.0)
    assert b.stats()["qn_inkernel_waves"] > 0
    assert np.array_equal(np.array(ra), np.array(rb))
    np.testing.assert_array_equal(a.x(), b.x())
