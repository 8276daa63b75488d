"""GPU tests of the HessianLearner path (the reference's default optimizer):
the count-covariance kernel against finite differences of the device
gradient, the CLI on every CTest case (CMakeLists.txt:34-57: default Hessian
optimizer, -n -eval -e 20 -i 31) with the reference's exit codes, and the
talk -eval Result vector of SURVEY.md Appendix A.  Needs a gfx950 device."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import DATA, ROOT

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "appendix_a.json")))
CLI = os.path.join(ROOT, "w-fsa_amd", "wfsa_amd", "wfsa")


@pytest.mark.parametrize("family", [
    dict(n_states=8, degree=2, vocab=4, emissions=1, n_strings=200, max_len=8),
    dict(n_states=20, degree=4, vocab=6, emissions=2, n_strings=300, max_len=12),
    dict(n_states=64, degree=4, vocab=16, emissions=1, n_strings=400, max_len=10),
])
def test_count_covariance_equals_gradient_derivative(family):
    """sum_s p_s Cov_s(c_j, c_k) = -d grad_j / d w_k (grad_j = -sum p E[c_j]):
    central differences of the device gradient, every pattern pair; and the
    pairs outside the pattern have no derivative.  Second-order terms exist
    for strings compiled into bubbles only, so the corpus is cut to those."""
    import wfsa_amd as W
    syn = W.Synthetic(seed=3, **family)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    nf = len(fsa.param_names())
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, wt / wt.sum())
    rec, pc, used = dev.recognize()
    tiers = dev.string_tiers()
    keep = np.flatnonzero((tiers == -1) & (rec == 1))
    assert len(keep) >= 10, (len(keep), np.bincount(tiers + 1))
    strings = [bytes(sym[off[i]:off[i + 1]]) for i in keep]
    sym2 = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    off2 = np.concatenate([[0], np.cumsum([len(x) for x in strings])]).astype(np.int64)
    dev.load_corpus(sym2, off2, wt[keep] / wt.sum())
    rec, pc, used = dev.recognize()
    assert rec.all() and (pc > 1).any()
    pairs = dev.hf_setup()
    w = np.random.default_rng(1).normal(-1.0, 0.3, size=nf)
    cov = dev.hf_eval(w)
    assert len(pairs) > 0
    h = 1e-5
    jac = np.zeros((nf, nf))
    for k in range(nf):
        if not used[k]:
            continue
        wp, wm = w.copy(), w.copy()
        wp[k] += h
        wm[k] -= h
        jac[:, k] = -(dev.objective_grad(wp, want_logq=False)[1] - dev.objective_grad(wm, want_logq=False)[1]) / (2 * h)
    dense = np.zeros((nf, nf))
    for (j, k), v in zip(pairs, cov):
        dense[j, k] = v
        dense[k, j] = v
    scale = np.abs(jac).max()
    np.testing.assert_allclose(dense, jac, rtol=0, atol=1e-7 * scale)
    assert np.abs(jac - (jac + jac.T) / 2).max() <= 1e-7 * scale


def _run_cli(wfsa, corpus, *extra):
    r = subprocess.run([CLI, "-a", os.path.join(DATA, wfsa + ".wfsa"), "-c", os.path.join(DATA, corpus + ".corpus"),
                        *extra], capture_output=True, text=True, timeout=120)
    return r


CTESTS = [("test", "test"), ("test.list", "test"), ("test2", "test"), ("test3", "test"), ("test4", "test"),
          ("test.loop", "test"), ("talk", "talk"), ("talk", "test")]
CTEST_NAMES = ["test1", "testlist", "test2", "test3", "test4", "test_loop", "test_talk", "test_talk2"]


@pytest.mark.parametrize("case,name", list(zip(CTESTS, CTEST_NAMES)), ids=CTEST_NAMES)
@pytest.mark.parametrize("verbose", [False, True], ids=["", "v"])
def test_ctest_exit_codes(case, name, verbose):
    extra = (["-p"] if verbose else []) + ["-n", "-eval", "-e", "20", "-i", "31"]
    r = _run_cli(case[0], case[1], *extra)
    assert r.returncode == GOLD["ctest_exit_codes"][name], r.stderr[-2000:]
    if r.returncode == 0:
        assert "Result:" in r.stderr


def _check_talk_result(got, want):
    """every entry but logdetH (index 4) to 5e-13; talk's weight-space
    Hessian is exactly singular (tests/test_oracle.py), so logdetH is the log
    of a rounding residue: only 'numerically singular' is pinned"""
    keep = [0, 1, 2, 3, 5, 6, 7]
    np.testing.assert_allclose(got[keep], want[keep], rtol=5e-13, atol=1e-14)
    assert got[4] == np.inf or got[4] < -15.0


def test_talk_eval_result_matches_reference():
    """`wfsa -a talk.wfsa -c talk.corpus -n -eval -e 20 -i 31` Result line
    (KL, mxlogx(support), LogModelVolume, LogAuxVolume, logdetH, LogDetAuxH,
    n-k, aux-1) == the reference's printout (15 significant digits)"""
    r = _run_cli("talk", "talk", "-n", "-eval", "-e", "20", "-i", "31", "-s")
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stderr.splitlines() if l.startswith("Result:")][-1]
    got = [float(v) for v in line.split()[1:]]
    want = np.array(GOLD["talk_hessian_result"]["result"])
    assert len(got) == len(want)
    _check_talk_result(np.array(got), want)


def test_hessian_learner_api_talk():
    """the same through the C ABI (wfsa_learner_create("Hessian"))"""
    import wfsa_amd as W
    fsa = W.Fsa.read_file(os.path.join(DATA, "talk.wfsa"))
    corpus = W.Corpus.read_file(os.path.join(DATA, "talk.corpus"))
    lrn = W.HessianLearner(0)
    assert lrn.width == 9
    lrn.BuildFrom(fsa, corpus)
    lrn.Finalize()
    rows = lrn.run(flags=31, epochs=20, tol=1e-6)
    assert 1 <= len(rows) <= 20
    lrn.Renormalize()
    _check_talk_result(np.array(lrn.result()), np.array(GOLD["talk_hessian_result"]["result"]))


HCASES = [("talk", "talk"), ("test3", "test"), ("test4", "test"), ("test.list", "test"), ("test2", "test"),
          ("test.loop", "test"), ("test5", "test5"), ("test5_2", "test5")]


def _fd_check(dev, nf, used, seed=1):
    pairs = dev.hf_setup()
    w = np.random.default_rng(seed).normal(-1.0, 0.3, size=nf)
    cov = dev.hf_eval(w)
    assert len(pairs) > 0
    h = 1e-5
    jac = np.zeros((nf, nf))
    for k in range(nf):
        if not used[k]:
            continue
        wp, wm = w.copy(), w.copy()
        wp[k] += h
        wm[k] -= h
        jac[:, k] = -(dev.objective_grad(wp, want_logq=False)[1] - dev.objective_grad(wm, want_logq=False)[1]) / (2 * h)
    dense = np.zeros((nf, nf))
    for (j, k), v in zip(pairs, cov):
        dense[j, k] = v
        dense[k, j] = v
    scale = np.abs(jac).max()
    np.testing.assert_allclose(dense, jac, rtol=0, atol=1e-7 * scale)


TRAV_FAMILIES = [
    dict(n_states=12, degree=3, vocab=3, emissions=2, n_strings=150, max_len=24, seed=3),
    dict(n_states=16, degree=3, vocab=4, emissions=2, n_strings=100, max_len=12, seed=3),
]


@pytest.mark.parametrize("family", TRAV_FAMILIES)
def test_count_covariance_on_traversal_strings(family):
    """strings whose ambiguity region no compiled bubble (<= 32 nodes) holds
    run on the traversal tiers; their second-order terms come from
    hf_trav_kernel (E[c c^T] = D + A + A^T over the string's trellis, on its
    equivocal parameters).  The whole recognized corpus, bubbles and
    traversal strings together, against central differences of the gradient."""
    import wfsa_amd as W
    syn = W.Synthetic(**family)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    nf = len(fsa.param_names())
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, wt / wt.sum())
    rec, _, _ = dev.recognize()
    keep = np.flatnonzero(rec == 1)
    strings = [bytes(sym[off[i]:off[i + 1]]) for i in keep]
    sym2 = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    off2 = np.concatenate([[0], np.cumsum([len(x) for x in strings])]).astype(np.int64)
    dev.load_corpus(sym2, off2, wt[keep] / wt.sum())
    rec, pc, used = dev.recognize()
    assert rec.all()
    assert (dev.string_tiers() >= 0).sum() >= 5, np.bincount(dev.string_tiers() + 1)
    _fd_check(dev, nf, used)


def _trav_learner(fam):
    import wfsa_amd as W
    syn = W.Synthetic(**fam)
    sym, off, wt = syn.corpus()
    lrn = W.HessianLearner(0)
    lrn.BuildFromPacked(W.Fsa.read_text(syn.wfsa_text), sym, off, wt)
    lrn.Finalize()
    return syn, (sym, off, wt), lrn


def test_hessian_learner_on_traversal_strings_matches_restatement():
    """HessianLearner epochs on a corpus with 16 traversal-tier strings (the
    rest in bubbles), against oracle/hessian.py on the oracle's enumerated
    paths (<= 144 per string)"""
    from oracle import Oracle
    from oracle.hessian import HessianOracle
    fam = dict(n_states=16, degree=2, vocab=4, emissions=2, n_strings=200, max_len=16, seed=4)
    syn, (sym, off, wt), lrn = _trav_learner(fam)
    h = HessianOracle(Oracle.from_arrays(syn.wfsa_text, sym, off, wt, max_paths=3_000_000))
    want = np.array(h.run(flags=31, epochs=20, tol=1e-6))
    got = np.array(lrn.run(flags=31, epochs=20, tol=1e-6))
    assert lrn.stats()["fallback_strings"] > 0
    assert got.shape[0] == want.shape[0]
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(got[:, 1:4], want[:, 1:4], rtol=1e-6, atol=1e-10)
    np.testing.assert_array_equal(got[:, 4:6], want[:, 4:6])
    names = {n: i for i, n in enumerate(h.o.param_names())}
    order = [names[n] for n in lrn.param_names()]
    np.testing.assert_allclose(lrn.x(), h.x[order], rtol=0, atol=1e-8)


def test_hessian_learner_degenerate_step_like_restatement():
    """a family whose Newton step goes non-finite: both sides stop with
    "Unable to continue!" (HaltCondition, src/HessianLearner.cpp:374-379)
    after the same epochs; the factorisation of the NaN system stays in
    bounds (a fresh learner runs after it)"""
    import wfsa_amd as W
    from oracle import Oracle
    from oracle.hessian import HessianOracle
    from oracle.oracle import OracleError
    fam = dict(n_states=16, degree=3, vocab=4, emissions=2, n_strings=100, max_len=12, seed=3)
    syn, (sym, off, wt), lrn = _trav_learner(fam)
    h = HessianOracle(Oracle.from_arrays(syn.wfsa_text, sym, off, wt, max_paths=3_000_000))
    with pytest.raises(OracleError, match="Unable to continue"):
        h.run(flags=31, epochs=20, tol=1e-6)
    with pytest.raises(W.WfsaError, match="Unable to continue"):
        lrn.run(flags=31, epochs=20, tol=1e-6)
    del lrn
    _, _, lrn2 = _trav_learner(dict(fam, seed=4))
    lrn2.Init(31)


@pytest.mark.parametrize("kkt,flags", [("", 31), ("sparse", 31), ("sparse", 15)], ids=["dense", "sparse-md", "sparse-id"])
@pytest.mark.parametrize("case", HCASES, ids=lambda c: f"{c[0]}+{c[1]}")
def test_hessian_learner_epochs_match_restatement(case, kkt, flags, monkeypatch):
    """HessianLearner through the C ABI, epoch by epoch (KL, graderr, g_min,
    g_max, inertia +/-, lambda_min) and its Result vector, against the dense
    restatement oracle/hessian.py on the oracle's enumerated paths.  logdetH is
    compared where the Hessian is well conditioned (talk's is singular).  The
    KKT system through the dense Bunch-Kaufman LDL^T and through the sparse
    LDL^T (WFSA_KKT=sparse) in approximate-minimum-degree order (flag 16, the reference's
    METIS) and in the identity order (the reference's MKL_DSS_MY_ORDER)."""
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_KKT", kkt)
    from oracle import Oracle
    from oracle.hessian import HessianOracle
    wpath, cpath = os.path.join(DATA, case[0] + ".wfsa"), os.path.join(DATA, case[1] + ".corpus")
    h = HessianOracle(Oracle.from_files(wpath, cpath))
    want = np.array(h.run(flags=flags, epochs=20, tol=1e-6))
    h.renormalize()
    want_res = h.result()
    lrn = W.HessianLearner(0)
    lrn.BuildFrom(W.Fsa.read_file(wpath), W.Corpus.read_file(cpath))
    lrn.Finalize()
    got = np.array(lrn.run(flags=flags, epochs=20, tol=1e-6))
    assert got.shape[0] == want.shape[0]
    # KL and residuals; the residuals shrink to ~1e-12, so an absolute floor
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(got[:, 1:4], want[:, 1:4], rtol=1e-6, atol=1e-10)
    np.testing.assert_array_equal(got[:, 4:6], want[:, 4:6])
    np.testing.assert_allclose(got[:, 6], want[:, 6], rtol=1e-9, atol=1e-12)
    # rmin: the value, and the string holding the reference's min path
    np.testing.assert_allclose(got[:, 7], want[:, 7], rtol=1e-9, atol=1e-300)
    strings = np.searchsorted(h.mrow, want[:, 8].astype(np.int64), side="right") - 1
    np.testing.assert_array_equal(got[:, 8], np.where(h.unique, 0, strings))
    lrn.Renormalize()
    # same parameters, possibly another order: match them by name.  On a
    # singular Hessian (talk: a one-dimensional set of optima) the last Newton
    # steps move along the flat direction by rounding-sized amounts
    ev = np.abs(np.linalg.eigvalsh(h.weight_hessian()))
    well = ev.min() > 1e-8 * ev.max()
    names = {n: i for i, n in enumerate(h.o.param_names())}
    order = [names[n] for n in lrn.param_names()]
    np.testing.assert_allclose(lrn.x(), h.x[order], rtol=0, atol=1e-8 if well else 1e-4)
    res = np.array(lrn.result())
    keep = [0, 1, 2, 3, 5, 6, 7]
    np.testing.assert_allclose(res[keep], want_res[keep], rtol=1e-10, atol=1e-13)
    if well:
        if np.isinf(want_res[4]):
            assert np.isinf(res[4])
        else:
            np.testing.assert_allclose(res[4], want_res[4], rtol=1e-8, atol=1e-10)


def test_hessian_learner_sparse_and_dense_kkt_agree(monkeypatch):
    """a mid-size sparse family (n + k > 1024, so the host-dense size is
    exceeded): the default choice between the sparse LDL^T and the dense
    factorisation in HBM against WFSA_KKT=device -- the same epochs (inertia
    exactly, the rest to rounding) and the same Result vector"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=256, degree=8, vocab=64, emissions=1, n_strings=20000, max_len=64, seed=2)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)

    def run(kkt):
        monkeypatch.setenv("WFSA_KKT", kkt)
        lrn = W.HessianLearner(0)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        inf = lrn.info()
        rows = np.array(lrn.run(flags=31, epochs=4, tol=1e-12))
        lrn.Renormalize()
        return inf, rows, np.array(lrn.result())

    inf, ra, resa = run("")
    assert inf["n_params"] + inf["n_constraints"] > 1024
    _, rb, resb = run("device")
    assert ra.shape == rb.shape
    np.testing.assert_allclose(ra[:, 0], rb[:, 0], rtol=1e-10)
    np.testing.assert_allclose(ra[:, 1:4], rb[:, 1:4], rtol=1e-6, atol=1e-10)
    np.testing.assert_array_equal(ra[:, 4:6], rb[:, 4:6])
    keep = [0, 1, 2, 3, 5, 6, 7]
    np.testing.assert_allclose(resa[keep], resb[keep], rtol=1e-9, atol=1e-12)
    if np.isfinite(resb[4]):
        np.testing.assert_allclose(resa[4], resb[4], rtol=1e-8)
