"""GPU tests of the rmin info column (QuasiNewtonLearner::GetOptimizationInfo,
src/QuasiNewtonLearner.cpp:80-84; HessianLearner :313-317): the smallest
relative path probability over all paths, from the device's (min, x) passes
(compiled bubbles, traversal tiers 0/1 in min mode, tier 2 in min mode),
against the oracle's enumerated paths (oracle/hessian.py).  The index column
is the string holding that path; the reference's BFS path index is mapped to
its string through the oracle's M rows.  Needs a gfx950 device."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu


def _oracle_rmin(h, x):
    """(min relative path prob, string of that path) from the path matrices"""
    h.x = np.array(x, dtype=np.float64)
    _, rpp = h.modeled()
    amb = np.repeat(np.diff(h.mrow) > 1, np.diff(h.mrow))
    r = np.where(amb, rpp, np.inf)
    i = int(np.argmin(r))
    s = int(np.searchsorted(h.mrow, i, side="right") - 1)
    return float(r[i]), s, rpp


def _setup(wfsa_text, sym, off, wt, monkeypatch, tier2=False):
    """device with the recognized strings (corpus order) + the oracle"""
    import wfsa_amd as W
    from oracle import Oracle
    from oracle.hessian import HessianOracle
    monkeypatch.setenv("WFSA_TIER2", "1" if tier2 else "0")
    o = Oracle.from_arrays(wfsa_text, sym, off, wt)
    h = HessianOracle(o)
    fsa = W.Fsa.read_text(wfsa_text)
    dev = W.Device(0)
    dev.load_model(fsa)
    p = wt / wt.sum()
    dev.load_corpus(sym, off, p)
    rec, _, _ = dev.recognize()
    keep = np.flatnonzero(rec)
    strings = [bytes(sym[off[i]:off[i + 1]]) for i in keep]
    sym2 = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    off2 = np.concatenate([[0], np.cumsum([len(s) for s in strings])]).astype(np.int64)
    dev.load_corpus(sym2, off2, p[keep])
    # the device numbers parameters as the reference does (its hash-map
    # order), the oracle by state order: match them by name
    names = {n: j for j, n in enumerate(o.full_param_names())}
    dev.perm = np.array([names[n] for n in fsa.param_names()], dtype=np.int64)
    return o, h, dev


def _check(o, h, dev, seed):
    rng = np.random.default_rng(seed)
    for _ in range(3):
        x = rng.normal(-1.0, 0.5, size=o.n)
        o.set_x(x)
        dev.objective_grad(o.w_full()[dev.perm], want_logq=False)
        r, s = dev.rmin()
        want, ws, rpp = _oracle_rmin(h, x)
        assert abs(r - want) <= 1e-12 * want, (r, want)
        # ties (equal path probabilities in different strings) may pick either
        a, b = h.mrow[s], h.mrow[s + 1]
        assert b - a > 1 and abs(rpp[a:b].min() - want) <= 1e-12 * want
        if np.sum(np.abs(np.where(np.repeat(np.diff(h.mrow) > 1, np.diff(h.mrow)), rpp, np.inf) - want)
                  <= 1e-12 * want) == 1:
            assert s == ws


def _files(wfsa, corpus):
    import wfsa_amd as W
    text = open(os.path.join(DATA, wfsa + ".wfsa"), "rb").read().decode("latin-1")
    sym, off, wt = W.Corpus.read_file(os.path.join(DATA, corpus + ".corpus")).packed()
    return text, sym, off, wt


@pytest.mark.parametrize("case", [("talk", "talk"), ("test3", "test"), ("test5", "test5"), ("test5_2", "test5")],
                         ids=lambda c: c[0])
@pytest.mark.parametrize("tier2", [False, True], ids=["auto", "tier2"])
def test_rmin_golden_cases(case, tier2, monkeypatch):
    """talk / test3: compiled bubbles; test5: one 20-node ambiguity region on
    a traversal tier; tier2: every string forced onto the wide kernel"""
    text, sym, off, wt = _files(*case)
    o, h, dev = _setup(text, sym, off, wt, monkeypatch, tier2)
    _check(o, h, dev, seed=5)


@pytest.mark.parametrize("family", [
    dict(n_states=12, degree=3, vocab=3, emissions=2, n_strings=150, max_len=8),
    dict(n_states=64, degree=4, vocab=16, emissions=1, n_strings=400, max_len=10),
])
@pytest.mark.parametrize("tier2", [False, True], ids=["auto", "tier2"])
def test_rmin_synthetic(family, tier2, monkeypatch):
    """family 0: mostly traversal tiers 0/1 (ambiguous); family 1: compiled"""
    import wfsa_amd as W
    syn = W.Synthetic(seed=3, **family)
    sym, off, wt = syn.corpus()
    o, h, dev = _setup(syn.wfsa_text, sym, off, wt, monkeypatch, tier2)
    tiers = dev.string_tiers()
    if not tier2:
        assert (tiers == -1).any() or (tiers >= 0).any()
    _check(o, h, dev, seed=7)


@pytest.mark.parametrize("source", ["test3", "family0", "family0_tier2"])
def test_rmin_column_in_quasinewton_device_loop(source, monkeypatch):
    """the device-resident QN loop fills columns 5/6 at each step's x: the
    oracle's QN trajectory (same steps) gives the x before each step.
    family0's strings run on the traversal tiers, whose weighted passes carry
    the min forward in the loop (family0_tier2: all on the wide kernel)"""
    import wfsa_amd as W
    from oracle import Oracle
    from oracle.hessian import HessianOracle
    monkeypatch.setenv("WFSA_TIER2", "1" if source.endswith("tier2") else "0")
    lrn = W.QuasiNewtonLearner(0, optimizer="QuasiNewton")
    if source == "test3":
        wpath, cpath = os.path.join(DATA, "test3.wfsa"), os.path.join(DATA, "test.corpus")
        o = Oracle.from_files(wpath, cpath)
        lrn.BuildFrom(W.Fsa.read_file(wpath), W.Corpus.read_file(cpath))
    else:
        syn = W.Synthetic(n_states=12, degree=3, vocab=3, emissions=2, n_strings=150, max_len=8, seed=3)
        sym, off, wt = syn.corpus()
        o = Oracle.from_arrays(syn.wfsa_text, sym, off, wt)
        lrn.BuildFromPacked(W.Fsa.read_text(syn.wfsa_text), sym, off, wt)
    h = HessianOracle(o)
    o.qn_init(7)
    want = []
    for _ in range(8):
        r, s, _ = _oracle_rmin(h, o.x())
        want.append((r, s))
        o.qn_step(1.0)
        if o.qn_halt(1e-6):
            break
    lrn.Finalize()
    rows = np.array(lrn.run(flags=7, epochs=len(want), tol=1e-6))
    assert len(rows) == len(want)
    np.testing.assert_allclose(rows[:, 5], [w[0] for w in want], rtol=1e-9)
    np.testing.assert_array_equal(rows[:, 6], [w[1] for w in want])


def test_rmin_column_bitwise_reproducible_on_bubbles():
    """the bubble passes (fused into the stream kernel, or the bubble kernel
    beside it, as here) store each bubble's log(min path / Z) at its list
    position and the strings kernel sums them per string in bubble order (no
    atomics): two device-loop runs give the same rmin column bit for bit,
    equal to the separate rmin pass (host steps) to rounding"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=64, degree=8, vocab=16, emissions=1, n_strings=3000, max_len=64, seed=5)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    runs = []
    for _ in range(2):
        lrn = W.QuasiNewtonLearner(0)
        lrn.set_info_rmin(True)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        runs.append(np.array(lrn.Run(6, 1.0, -1.0)))
    assert lrn.stats()["n_bubbles"] > 0 and lrn.stats()["fallback_strings"] == 0
    assert (runs[0][:, 6] >= 0).all()
    np.testing.assert_array_equal(runs[0][:, 5:7], runs[1][:, 5:7])
    host = W.QuasiNewtonLearner(0)
    host.set_info_rmin(True)
    host.BuildFromPacked(fsa, sym, off, wt)
    host.Finalize()
    host.Init(7)
    rows = np.array([host.OptimizationStep(1.0, -1.0)[0] for _ in range(6)])
    np.testing.assert_allclose(rows[:, 5], runs[0][:, 5], rtol=1e-11)
    np.testing.assert_array_equal(rows[:, 6], runs[0][:, 6])
