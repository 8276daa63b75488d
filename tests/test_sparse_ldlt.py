"""The HessianLearner's sparse LDL^T (w-fsa_amd/csrc/SparseLdlt.cpp, MKL DSS's
role in src/HessianLearner.cpp:28-57,100-113) through the host C ABI
(wfsa_sym_sparse_solve): solution, inertia and log|det| against numpy on
KKT-shaped systems like the learner's (H_g + H_f over the parameters, one
J_g entry per parameter row, the zero constraint block), in the three orders
(the identity -- the reference's MKL_DSS_MY_ORDER --, exact minimum degree,
and approximate minimum degree for init flag 16, the reference's METIS), with
the multifrontal supernodal Bunch-Kaufman pivots (2x2 blocks where a zero
diagonal comes first).  Host only: no device."""
import numpy as np
import pytest

import wfsa_amd as W


def _kkt(n, k, seed, indefinite=False, pairs=3):
    rng = np.random.default_rng(seed)
    C = rng.integers(0, k, size=n)
    C[:k] = np.arange(k)                      # every constraint has a parameter
    ex = np.exp(rng.normal(-1.0, 0.5, size=n))
    lam = rng.uniform(0.5, 2.0, size=k)
    ent = {}

    def add(a, b, v):
        a, b = min(a, b), max(a, b)
        ent[(a, b)] = ent.get((a, b), 0.0) + v

    for i in range(n):
        add(i, i, ex[i] * lam[C[i]])
        add(i, n + C[i], ex[i])
    # H_f: -cov over random groups of parameters (negative semidefinite blocks)
    for _ in range(pairs * n // 4):
        g = rng.choice(n, size=4, replace=False)
        c = rng.normal(size=4) * 0.3
        for a in range(4):
            for b in range(a, 4):
                add(g[a], g[b], -(c[a] * c[b]) * (3.0 if indefinite else 0.2))
    i, j = np.array([e[0] for e in ent], dtype=np.int32), np.array([e[1] for e in ent], dtype=np.int32)
    v = np.array(list(ent.values()))
    N = n + k
    A = np.zeros((N, N))
    A[i, j] += v
    A[j, i] += np.where(i != j, v, 0.0)
    return i, j, v, A


@pytest.mark.parametrize("order", [0, 1, 2])
@pytest.mark.parametrize("n,k,seed,indef", [(40, 6, 1, False), (300, 30, 2, False), (300, 30, 3, True),
                                             (1500, 120, 4, True)])
def test_kkt_solve_inertia_logdet(order, n, k, seed, indef):
    i, j, v, A = _kkt(n, k, seed, indef)
    b = np.random.default_rng(seed + 100).normal(size=n + k)
    x, st = W.sym_sparse_solve(i, j, v, n + k, b, order=order)
    want = np.linalg.solve(A, b)
    np.testing.assert_allclose(x, want, rtol=1e-8, atol=1e-10 * np.abs(want).max())
    ev = np.linalg.eigvalsh(A)
    assert (st["positive"], st["negative"]) == (int((ev > 0).sum()), int((ev < 0).sum()))
    sign, logdet = np.linalg.slogdet(A)
    assert st["det_sign"] == int(sign)
    assert abs(st["log_abs_det"] - logdet) <= 1e-9 * max(1.0, abs(logdet))
    assert st["ordered"]


def test_minimum_degree_avoids_arrow_fill():
    """an arrow matrix whose dense row comes first fills L completely in the
    identity order; minimum degree eliminates the leaves first (no fill)"""
    n = 200
    i = np.concatenate([np.arange(n), np.zeros(n - 1)]).astype(np.int32)
    j = np.concatenate([np.arange(n), np.arange(1, n)]).astype(np.int32)
    v = np.concatenate([[float(n)], np.full(n - 1, 2.0), np.full(n - 1, 1.0)])
    b = np.arange(n, dtype=float)
    x0, s0 = W.sym_sparse_solve(i, j, v, n, b, order=0)
    x1, s1 = W.sym_sparse_solve(i, j, v, n, b, order=1)
    x2, s2 = W.sym_sparse_solve(i, j, v, n, b, order=2)
    assert s0["nnz_l"] == n * (n - 1) // 2
    assert s0["supernodes"] == 1 and s0["max_front"] == n   # (the dense chain is one supernode)
    assert s1["nnz_l"] == n - 1 and s2["nnz_l"] == n - 1
    np.testing.assert_allclose(x0, x1, rtol=1e-12)
    np.testing.assert_allclose(x2, x1, rtol=1e-12)
    A = np.zeros((n, n))
    A[i, j] = v
    A[j, i] = v
    np.testing.assert_allclose(x1, np.linalg.solve(A, b), rtol=1e-10)


def test_duplicates_add_and_factor_only():
    i = np.array([0, 0, 1, 0, 1], dtype=np.int32)
    j = np.array([0, 0, 1, 1, 1], dtype=np.int32)
    v = np.array([1.0, 2.0, 1.0, 1.0, 3.0])           # A = [[3, 1], [1, 4]]
    x, st = W.sym_sparse_solve(i, j, v, 2)
    assert x is None
    assert st["positive"] == 2 and abs(st["log_abs_det"] - np.log(11.0)) < 1e-14


def test_two_by_two_pivot_and_singular():
    """[[0, 1], [1, 0]] needs a 2x2 pivot: one supernode, one 2x2 block, inertia
    (1, 1); a singular matrix is reported (the learner falls back to the dense
    factorisation then)"""
    x, st = W.sym_sparse_solve(np.array([0, 0, 1], np.int32), np.array([0, 1, 1], np.int32), np.array([0.0, 1.0, 0.0]),
                               2, np.array([2.0, 3.0]))
    assert (st["positive"], st["negative"], st["two_by_two"]) == (1, 1, 1)
    np.testing.assert_allclose(x, [3.0, 2.0], rtol=1e-15)
    assert st["det_sign"] == -1 and abs(st["log_abs_det"]) < 1e-15
    with pytest.raises(W.WfsaError, match="singular"):
        W.sym_sparse_solve(np.array([0, 0, 1], np.int32), np.array([0, 1, 1], np.int32), np.array([1.0, 1.0, 1.0]),
                           2, np.ones(2))
    x, st = W.sym_sparse_solve(np.array([0, 0, 1], np.int32), np.array([0, 1, 1], np.int32),
                               np.array([1e-3, 1.0, 0.0]), 2, np.ones(2))
    assert (st["positive"], st["negative"]) == (1, 1)
    np.testing.assert_allclose(x, np.linalg.solve([[1e-3, 1.0], [1.0, 0.0]], np.ones(2)), rtol=1e-12)


def _constraints_first(n, k, seed):
    """the KKT system with the constraint rows numbered first: their zero
    diagonals come first in the identity order, so the pivots there are 2x2
    blocks (or swaps) inside the supernodes"""
    i, j, v, A = _kkt(n, k, seed, True)
    N = n + k
    p = np.concatenate([np.arange(n, N), np.arange(n)])   # new -> old
    q = np.empty(N, dtype=np.int64)
    q[p] = np.arange(N)                                   # old -> new
    a, b = q[i], q[j]
    lo, hi = np.minimum(a, b).astype(np.int32), np.maximum(a, b).astype(np.int32)
    return lo, hi, v, A[np.ix_(p, p)]


@pytest.mark.parametrize("order", [0, 1, 2])
@pytest.mark.parametrize("n,k,seed", [(60, 12, 5), (400, 40, 6)])
def test_zero_diagonals_first(order, n, k, seed):
    i, j, v, A = _constraints_first(n, k, seed)
    b = np.random.default_rng(seed).normal(size=n + k)
    x, st = W.sym_sparse_solve(i, j, v, n + k, b, order=order)
    want = np.linalg.solve(A, b)
    np.testing.assert_allclose(x, want, rtol=1e-7, atol=1e-9 * np.abs(want).max())
    ev = np.linalg.eigvalsh(A)
    assert (st["positive"], st["negative"]) == (int((ev > 0).sum()), int((ev < 0).sum()))
    sign, logdet = np.linalg.slogdet(A)
    assert st["det_sign"] == int(sign)
    assert abs(st["log_abs_det"] - logdet) <= 1e-8 * max(1.0, abs(logdet))
    if order == 0:   # the zero diagonals lead: 2x2 blocks or delayed columns
        assert st["two_by_two"] + st["delayed"] > 0


def test_fill_reducing_orders_on_a_grid():
    """a 2-D grid Laplacian (+ shift): approximate minimum degree cuts the
    identity order's band fill, forms supernodes, and solves the same"""
    m = 30
    n = m * m
    ii, jj, vv = [], [], []
    for r in range(m):
        for c in range(m):
            u = r * m + c
            ii.append(u); jj.append(u); vv.append(4.5)
            if c + 1 < m:
                ii.append(u); jj.append(u + 1); vv.append(-1.0)
            if r + 1 < m:
                ii.append(u); jj.append(u + m); vv.append(-1.0)
    i, j, v = np.array(ii, np.int32), np.array(jj, np.int32), np.array(vv)
    b = np.random.default_rng(0).normal(size=n)
    x0, s0 = W.sym_sparse_solve(i, j, v, n, b, order=0)
    x1, s1 = W.sym_sparse_solve(i, j, v, n, b, order=1)
    x2, s2 = W.sym_sparse_solve(i, j, v, n, b, order=2)
    assert s2["nnz_l"] < 0.5 * s0["nnz_l"] and s1["nnz_l"] < 0.5 * s0["nnz_l"]
    assert s2["supernodes"] < n
    for x in (x1, x2):
        np.testing.assert_allclose(x, x0, rtol=1e-11, atol=1e-12)
    assert s0["positive"] == s1["positive"] == s2["positive"] == n
    assert abs(s2["log_abs_det"] - s0["log_abs_det"]) < 1e-9 * abs(s0["log_abs_det"])


@pytest.mark.parametrize("order", [0, 1, 2])
def test_edge_cases(order):
    """empty and 1x1 systems, a zero diagonal entry with no coupling
    (singular), and a forest (two independent blocks, one needing a 2x2 pivot)"""
    x, st = W.sym_sparse_solve(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0), 0, np.zeros(0), order=order)
    assert x.size == 0 and st["positive"] == st["negative"] == 0 and st["supernodes"] == 0
    x, st = W.sym_sparse_solve(np.array([0], np.int32), np.array([0], np.int32), np.array([2.0]), 1, np.array([4.0]),
                               order=order)
    assert x[0] == 2.0 and st["positive"] == 1 and abs(st["log_abs_det"] - np.log(2.0)) < 1e-15
    with pytest.raises(W.WfsaError, match="singular"):
        W.sym_sparse_solve(np.array([0, 1], np.int32), np.array([0, 1], np.int32), np.array([1.0, 0.0]), 2, np.ones(2),
                           order=order)
    i = np.array([0, 0, 1, 2, 2, 3], np.int32)
    j = np.array([0, 1, 1, 2, 3, 3], np.int32)
    v = np.array([2.0, 1.0, 3.0, 0.0, 1.0, 0.0])
    A = np.zeros((4, 4))
    A[i, j] += v
    A[j, i] += np.where(i != j, v, 0.0)
    b = np.arange(4.0)
    x, st = W.sym_sparse_solve(i, j, v, 4, b, order=order)
    np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-14)
    assert st["two_by_two"] == 1 and (st["positive"], st["negative"]) == (3, 1)
