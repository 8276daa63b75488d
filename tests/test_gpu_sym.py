"""GPU tests of the dense symmetric-indefinite factorisation in HBM that the
HessianLearner uses for large KKT systems (wfsa_dev_sym_factor / _solve:
rocSOLVER dsytrf + the dsytrs kernel) -- inertia, log|det| and sign against
numpy's eigenvalues / slogdet, the solve against numpy -- and the learner
with the device factorisation forced (WFSA_KKT=device) against the dense
restatement.  Needs a gfx950 device."""
import os

import numpy as np
import pytest

from conftest import DATA

pytestmark = pytest.mark.gpu


def _kkt(rng, n, k):
    """an indefinite KKT-like matrix [[H, J], [J^T, 0]] (2x2 pivots needed)"""
    a = rng.normal(size=(n, n))
    h = (a + a.T) / 2
    j = np.zeros((n, k))
    for i in range(n):
        j[i, i % k] = rng.uniform(0.5, 1.5)
    return np.block([[h, j], [j.T, np.zeros((k, k))]])


@pytest.mark.parametrize("n,k", [(1, 0), (2, 1), (7, 3), (64, 5), (500, 40), (1500, 200)])
def test_sym_factor_and_solve(n, k):
    import wfsa_amd as W
    rng = np.random.default_rng(n)
    a = _kkt(rng, n, k) if k else np.array([[rng.normal()]])
    dev = W.Device(0)
    (pos, neg, zero), lad, sign = dev.sym_factor(a)
    ev = np.linalg.eigvalsh(a)
    assert (pos, neg, zero) == (int(np.sum(ev > 0)), int(np.sum(ev < 0)), 0)
    s, l = np.linalg.slogdet(a)
    assert sign == int(s)
    assert abs(lad - l) <= 1e-9 * max(1.0, abs(l))
    b = rng.normal(size=a.shape[0])
    x = dev.sym_solve(b)
    want = np.linalg.solve(a, b)
    np.testing.assert_allclose(x, want, rtol=1e-8, atol=1e-8 * np.abs(want).max())


@pytest.mark.parametrize("case", [("talk", "talk"), ("test3", "test"), ("test4", "test")], ids=lambda c: c[0])
def test_hessian_learner_with_device_factorisation(case, monkeypatch):
    import wfsa_amd as W
    from oracle import Oracle
    from oracle.hessian import HessianOracle
    monkeypatch.setenv("WFSA_KKT", "device")
    wpath, cpath = os.path.join(DATA, case[0] + ".wfsa"), os.path.join(DATA, case[1] + ".corpus")
    h = HessianOracle(Oracle.from_files(wpath, cpath))
    want = np.array(h.run(flags=31, epochs=20, tol=1e-6))
    lrn = W.HessianLearner(0)
    lrn.BuildFrom(W.Fsa.read_file(wpath), W.Corpus.read_file(cpath))
    lrn.Finalize()
    got = np.array(lrn.run(flags=31, epochs=20, tol=1e-6))
    assert got.shape == want.shape
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-10, atol=1e-13)
    np.testing.assert_array_equal(got[:, 4:6], want[:, 4:6])


def test_hessian_learner_host_and_device_factorisations_agree(monkeypatch):
    """a compiled synthetic family whose KKT system (n + k ~ 1.2k) takes the
    device path by default: three Newton epochs, host vs device"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=128, degree=8, vocab=64, emissions=1, n_strings=5000, max_len=24, seed=2)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    rows = {}
    for side in ("host", "device"):
        monkeypatch.setenv("WFSA_KKT", side)
        lrn = W.HessianLearner(0)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        rows[side] = np.array(lrn.run(flags=31, epochs=3, tol=-1.0))
    assert rows["host"].shape == rows["device"].shape == (3, 9)
    np.testing.assert_allclose(rows["device"][:, 0], rows["host"][:, 0], rtol=1e-9)
    np.testing.assert_array_equal(rows["device"][:, 4:6], rows["host"][:, 4:6])


def _upper_entries(a, rng):
    """upper-triangle coordinates of a (i <= j); a tenth of the entries split
    in two parts (duplicates add, as SymEntries emits them)"""
    i, j = np.nonzero(np.triu(a))
    v = a[i, j]
    dup = np.flatnonzero(rng.random(len(v)) < 0.1)
    part = rng.uniform(0.2, 0.8, size=len(dup))
    extra = v[dup] * (1 - part)
    v = v.copy()
    v[dup] *= part
    return np.concatenate([i, i[dup]]), np.concatenate([j, j[dup]]), np.concatenate([v, extra])


@pytest.mark.parametrize("n,k", [(5, 2), (120, 10), (300, 30), (1000, 100), (2600, 300)])
def test_blocked_factor_from_entries(n, k):
    """wfsa_dev_sym_factor_coo: KKT-shaped systems (zero-diagonal constraint
    rows, several 128-column panels) factored blockwise -- inertia, log|det|,
    sign against numpy, the refined solve against numpy.linalg.solve"""
    import wfsa_amd as W
    rng = np.random.default_rng(100 + n)
    a = _kkt(rng, n, k)
    i, j, v = _upper_entries(a, rng)
    dev = W.Device(0)
    b = rng.normal(size=a.shape[0])
    (pos, neg, zero), lad, sign, method, x = dev.sym_factor_coo(a.shape[0], i, j, v, b)
    assert method == 1   # the blocked factorisation held up
    ev = np.linalg.eigvalsh(a)
    assert (pos, neg, zero) == (int(np.sum(ev > 0)), int(np.sum(ev < 0)), 0)
    s, l = np.linalg.slogdet(a)
    assert sign == int(s)
    assert abs(lad - l) <= 1e-8 * max(1.0, abs(l))
    want = np.linalg.solve(a, b)
    np.testing.assert_allclose(x, want, rtol=1e-8, atol=1e-9 * np.abs(want).max())
    # sym_solve after it: the same factor, refined
    b2 = rng.normal(size=a.shape[0])
    np.testing.assert_allclose(dev.sym_solve(b2), np.linalg.solve(a, b2), rtol=1e-8,
                               atol=1e-9 * np.abs(np.linalg.solve(a, b2)).max())


def test_blocked_factor_falls_back_to_full_pivoting():
    """a diagonal block no pivot inside it can serve (zero block, coupled only
    to rows below): the restricted pivoting gives up and the full
    Bunch-Kaufman answers"""
    import wfsa_amd as W
    rng = np.random.default_rng(7)
    n = 300
    a = np.zeros((n, n))
    a[128:, 128:] = rng.normal(size=(n - 128, n - 128))
    a[128:, 128:] = (a[128:, 128:] + a[128:, 128:].T) / 2
    c = rng.normal(size=(n - 128, 128))
    a[128:, :128] = c
    a[:128, 128:] = c.T
    i, j = np.nonzero(np.triu(a))
    b = rng.normal(size=n)
    dev = W.Device(0)
    (pos, neg, zero), lad, sign, method, x = dev.sym_factor_coo(n, i, j, a[i, j], b)
    assert method == 2
    ev = np.linalg.eigvalsh(a)
    assert (pos, neg, zero) == (int(np.sum(ev > 0)), int(np.sum(ev < 0)), 0)
    want = np.linalg.solve(a, b)
    np.testing.assert_allclose(x, want, rtol=1e-7, atol=1e-8 * np.abs(want).max())
