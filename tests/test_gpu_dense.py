"""GPU parity of the dense-automaton path (fp64 MFMA GEMMs, dense_path.hip;
BASELINE.json configs[4], SURVEY.md 8d "c5") against the CPU oracle's
trellis restatement and against the sparse trellis kernels on the same
inputs.  All tests need a gfx950 device."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["fused", "split", "dma", "blas"])
def gemm_engine(request, monkeypatch):
    """every test on the four GEMM engines of the dense path: our fused
    v_mfma_f64_16x16x4f64 kernels, our split-K RAW kernels and our LDS-DMA
    pipelined kernels with the epilogue kernels, and rocBLAS dgemm with the
    epilogue kernels (WFSA_DENSE_ENGINE)"""
    monkeypatch.delenv("WFSA_DENSE_BLAS", raising=False)
    monkeypatch.setenv("WFSA_DENSE_ENGINE", request.param)
    return request.param


def _close(a, b, rel, atol=1e-13):
    return abs(a - b) <= max(atol, rel * max(abs(a), abs(b)))


def _device(fsa, sym, off, p, monkeypatch, dense):
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_DENSE", "1" if dense else "0")
    dev = W.Device(0)
    dev.load_model(fsa)
    dev.load_corpus(sym, off, p)
    assert dev.stats()["dense"] == (1 if dense else 0)
    return dev


def _oracle(text, sym, off, wt, w_by_name):
    from oracle import Oracle, TRELLIS
    o = Oracle.from_arrays(text, sym, off, wt, mode=TRELLIS)
    names = o.full_param_names()
    ll, logq, grad = o.trellis_eval(np.array([w_by_name[n] for n in names]))
    return ll, logq, dict(zip(names, grad))


@pytest.mark.parametrize("spec", [
    dict(n_states=64, vocab=8, emissions=3, n_strings=400, max_len=24),     # partial emission sets
    dict(n_states=100, vocab=16, emissions=16, n_strings=300, max_len=40),  # every state emits every symbol; np padded
    dict(n_states=200, vocab=5, emissions=2, n_strings=700, max_len=70),    # two row tiles, ragged slots
])
def test_dense_matches_oracle_random_weights(spec, monkeypatch):
    import wfsa_amd as W
    syn = W.Synthetic(degree=1, dense=True, seed=13, **spec)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    names = fsa.param_names()
    p = wt / wt.sum()
    w = np.random.default_rng(5).normal(-1.0, 0.8, size=len(names))
    dev = _device(fsa, sym, off, p, monkeypatch, dense=True)
    rec, pc, used = dev.recognize()
    assert rec.all() and used.all()
    ll, grad, logq = dev.objective_grad(w)
    oll, ologq, ograd = _oracle(syn.wfsa_text, sym, off, wt, dict(zip(names, w)))
    np.testing.assert_allclose(logq, ologq, rtol=1e-12)
    assert _close(ll, oll, rel=1e-12)
    np.testing.assert_allclose(grad, [ograd[n] for n in names], rtol=1e-10, atol=1e-17)


def test_dense_equals_sparse_kernels(monkeypatch):
    """same model, same inputs: the MFMA path and the trellis kernels agree on
    recognition, path counts, used parameters, log q and the gradient"""
    import wfsa_amd as W
    # small enough for the trellis kernels' LDS slab (a dense 64-state model
    # is not: it fails there with WFSA_ERR_CAPACITY)
    syn = W.Synthetic(n_states=16, degree=1, vocab=6, emissions=2, dense=True, n_strings=500, max_len=9, seed=3)
    sym, off, wt = syn.corpus()
    # a few strings the automaton cannot emit (a byte nobody emits) and an empty one
    extra = [b"\x01", b"", syn_bad := b"zz\x02"]
    lens = np.diff(off)
    strings = [bytes(sym[off[i]:off[i + 1]]) for i in range(len(lens))] + extra
    sym2 = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    off2 = np.concatenate([[0], np.cumsum([len(s) for s in strings])]).astype(np.int64)
    wt2 = np.concatenate([wt, [3.0, 2.0, 1.0]])
    p2 = wt2 / wt2.sum()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    names = fsa.param_names()
    w = np.random.default_rng(2).normal(-0.7, 0.5, size=len(names))
    sp = _device(fsa, sym2, off2, p2, monkeypatch, dense=False)
    dn = _device(fsa, sym2, off2, p2, monkeypatch, dense=True)
    r_s, pc_s, u_s = sp.recognize()
    r_d, pc_d, u_d = dn.recognize()
    np.testing.assert_array_equal(r_d, r_s)
    assert list(r_d[-3:]) == [0, 0, 0] and syn_bad
    np.testing.assert_allclose(pc_d, pc_s, rtol=1e-12)
    np.testing.assert_array_equal(u_d, u_s)
    # weighted pass over the recognized strings only (as the Learner does)
    keep = np.flatnonzero(r_s)
    ks = [strings[i] for i in keep]
    sym3 = np.frombuffer(b"".join(ks), dtype=np.uint8).copy()
    off3 = np.concatenate([[0], np.cumsum([len(s) for s in ks])]).astype(np.int64)
    for d in (sp, dn):
        d.load_corpus(sym3, off3, p2[keep])
    ll_s, g_s, lq_s = sp.objective_grad(w)
    ll_d, g_d, lq_d = dn.objective_grad(w)
    np.testing.assert_allclose(lq_d, lq_s, rtol=1e-12)
    assert _close(ll_d, ll_s, rel=1e-12)
    np.testing.assert_allclose(g_d, g_s, rtol=1e-10, atol=1e-17)


def test_dense_learner_qn_equals_sparse(monkeypatch):
    """QuasiNewtonLearner end to end (BuildFrom, Trim, device-resident QN loop)"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=16, degree=1, vocab=8, emissions=2, dense=True, n_strings=300, max_len=9, seed=21)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    rows = {}
    xs = {}
    for dense in (False, True):
        monkeypatch.setenv("WFSA_DENSE", "1" if dense else "0")
        lrn = W.QuasiNewtonLearner(0)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        assert lrn.stats()["dense"] == (1 if dense else 0)
        rows[dense] = [lrn.OptimizationStep(1.0, -1.0)[0] for _ in range(2)] + lrn.Run(4, 1.0, -1.0)
        xs[dense] = lrn.x()
    assert len(rows[True]) == len(rows[False]) == 6
    for r, q in zip(rows[True], rows[False]):
        for a, b in zip(r[:5], q[:5]):
            assert _close(a, b, rel=1e-9, atol=1e-12)
    np.testing.assert_allclose(xs[True], xs[False], rtol=1e-9, atol=1e-11)


def test_dense_chosen_automatically(monkeypatch):
    import wfsa_amd as W
    monkeypatch.delenv("WFSA_DENSE", raising=False)
    syn = W.Synthetic(n_states=128, degree=1, vocab=4, emissions=4, dense=True, n_strings=50, max_len=8, seed=1)
    sym, off, wt = syn.corpus()
    dev = W.Device(0)
    dev.load_model(W.Fsa.read_text(syn.wfsa_text))
    dev.load_corpus(sym, off, wt / wt.sum())
    assert dev.stats()["dense"] == 1
    sparse = W.Synthetic(n_states=128, degree=8, vocab=4, emissions=1, n_strings=50, max_len=8, seed=1)
    dev2 = W.Device(0)
    dev2.load_model(W.Fsa.read_text(sparse.wfsa_text))
    assert dev2.stats()["dense"] == 0


def test_dense_1024_properties(monkeypatch):
    """c5 shape at 1024 states (every state emits every symbol of 16):
    posterior counts add up (one start and one end edge per path, L emissions
    and L-1 transitions), LL = p . log q, a string subset against the oracle"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=1024, degree=1, vocab=16, emissions=16, dense=True, n_strings=1500, max_len=64,
                      seed=4)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    names = fsa.param_names()
    p = wt / wt.sum()
    dev = _device(fsa, sym, off, p, monkeypatch, dense=True)
    rec, pc, used = dev.recognize()
    assert rec.all()
    rng = np.random.default_rng(9)
    w = rng.normal(-7.0, 1.0, size=len(names))
    ll, grad, logq = dev.objective_grad(w)
    assert np.isfinite(logq).all()
    assert _close(ll, float(np.dot(p, logq)), rel=1e-12)
    L = np.diff(off).astype(np.float64)
    kind = np.array([0 if n[1] == "E" else (1 if n[0] == "^" else (2 if n[2] == "$" else 3)) for n in names])
    assert _close(grad[kind == 1].sum(), -1.0, rel=1e-11)                       # ^ -> T
    assert _close(grad[kind == 2].sum(), -1.0, rel=1e-11)                       # S -> $
    assert _close(grad[kind == 0].sum(), -float(np.dot(p, L)), rel=1e-11)       # emissions
    assert _close(grad[kind == 3].sum(), -float(np.dot(p, L - 1)), rel=1e-11)   # S -> T
    idx = np.sort(rng.choice(len(wt), size=8, replace=False))
    sub_off = np.concatenate([[0], np.cumsum(np.diff(off)[idx])])
    sub_sym = np.concatenate([sym[off[i]:off[i + 1]] for i in idx])
    _, ologq, _ = _oracle(syn.wfsa_text, sub_sym, sub_off, wt[idx], dict(zip(names, w)))
    np.testing.assert_allclose(logq[idx], ologq, rtol=1e-12)


def test_dense_device_qn_large_groups_equals_host_update(monkeypatch):
    """device-resident QN (constraint groups of 101 members: the strided
    qn_update path) == the host QN update (QuasiNewtonLearner.cpp) step by step"""
    import wfsa_amd as W
    monkeypatch.setenv("WFSA_DENSE", "1")
    syn = W.Synthetic(n_states=100, degree=1, vocab=4, emissions=2, dense=True, n_strings=200, max_len=12, seed=8)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    a, b = W.QuasiNewtonLearner(0), W.QuasiNewtonLearner(0)
    for lrn in (a, b):
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        assert lrn.stats()["dense"] == 1
    rows_a = a.Run(5, 1.0, -1.0)
    rows_b = [b.OptimizationStep(1.0, -1.0)[0] for _ in range(5)]
    for r, q in zip(rows_a, rows_b):
        for u, v in zip(r[:5], q[:5]):
            assert _close(u, v, rel=1e-10, atol=1e-13)
    np.testing.assert_allclose(a.x(), b.x(), rtol=1e-10, atol=1e-12)


def _dense_tables(fsa, w, with_index=False):
    """exp-weights of a dense synthetic model from its flat description:
    A[S][T] (transitions), E[T][c] (1-byte emissions), the start row and the
    end column; kind of every Fsa parameter (0 emission, 1 start transition,
    2 end transition, 3 interior transition).  Unequivocal groups (-1) weigh 1."""
    import ctypes as C
    d = fsa.desc()
    ns = d.n_states

    def arr(ptr, n, ct):
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy()

    tr_ptr = arr(d.tr_ptr, ns + 1, C.c_int32)
    tr_dst = arr(d.tr_dst, int(tr_ptr[-1]), C.c_int32)
    tr_par = arr(d.tr_param, int(tr_ptr[-1]), C.c_int32)
    em_ptr = arr(d.em_ptr, ns + 1, C.c_int32)
    n_em = int(em_ptr[-1])
    em_off = arr(d.em_off, n_em, C.c_int64)
    em_len = arr(d.em_len, n_em, C.c_int32)
    em_par = arr(d.em_param, n_em, C.c_int32)
    em_bytes = arr(d.em_bytes, int((em_off + em_len).max()) if n_em else 1, C.c_uint8)
    ew = np.where(np.asarray(tr_par) >= 0, np.exp(w[np.maximum(tr_par, 0)]), 1.0)
    src = np.repeat(np.arange(ns), np.diff(tr_ptr))
    A = np.zeros((ns, ns))
    A[src, tr_dst] = ew
    E = np.zeros((ns, 256))
    esrc = np.repeat(np.arange(ns), np.diff(em_ptr))
    one = em_len == 1
    E[esrc[one], em_bytes[em_off[one]]] = np.where(em_par[one] >= 0, np.exp(w[np.maximum(em_par[one], 0)]), 1.0)
    kind = np.full(len(w), -1)
    kind[em_par[em_par >= 0]] = 0
    tk = np.where(src == d.start, 1, np.where(tr_dst == d.end, 2, 3))
    kind[tr_par[tr_par >= 0]] = tk[tr_par >= 0]
    if not with_index:
        return A, E, d.start, d.end, kind
    # every parameter's (row, column) in A or E
    index = dict(tr=(src, tr_dst, tr_par), em=(esrc[one], em_bytes[em_off[one]], em_par[one]))
    return A, E, d.start, d.end, kind, index


def _dense_logq(A, E, start, end, s):
    """scaled forward: alpha_1 = A[start] E[:, s0]; alpha_{i+1} = (alpha_i A) E[:, s_i]"""
    a = A[start] * E[:, s[0]]
    lg = 0.0
    for c in s[1:]:
        z = a.sum()
        lg += np.log(z)
        a = (a / z) @ A * E[:, c]
    return lg + np.log(a @ A[:, end])


def test_dense_c5_4096_states(monkeypatch):
    """c5 at its BASELINE size (BASELINE.json configs[4]: 4096 states, full
    transition matrix, every state emits every one of 16 symbols; 4096
    strings, L ~ 32): the posterior count identities of the 1024-state test,
    LL = p . log q, 8 strings against a numpy restatement of the forward
    (the C oracle's trellis takes minutes per string at this size), and the
    device-resident QN loop (4096 constraints of 4097 members: the strided
    QN path) against the host QN update for two steps"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=4096, degree=1, vocab=16, emissions=16, dense=True, n_strings=4096, max_len=128,
                      seed=2)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    n_par = fsa.counts()["parameters"]
    p = wt / wt.sum()
    dev = _device(fsa, sym, off, p, monkeypatch, dense=True)
    rec, pc, used = dev.recognize()
    assert rec.all()
    rng = np.random.default_rng(11)
    w = rng.normal(-8.5, 1.0, size=n_par)
    ll, grad, logq = dev.objective_grad(w)
    assert np.isfinite(logq).all()
    assert _close(ll, float(np.dot(p, logq)), rel=1e-12)
    A, E, start, end, kind = _dense_tables(fsa, w)
    assert (kind >= 0).all()
    L = np.diff(off).astype(np.float64)
    assert _close(grad[kind == 1].sum(), -1.0, rel=1e-10)
    assert _close(grad[kind == 2].sum(), -1.0, rel=1e-10)
    assert _close(grad[kind == 0].sum(), -float(np.dot(p, L)), rel=1e-10)
    assert _close(grad[kind == 3].sum(), -float(np.dot(p, L - 1)), rel=1e-10)
    for i in np.sort(rng.choice(len(wt), size=8, replace=False)):
        assert _close(logq[i], _dense_logq(A, E, start, end, sym[off[i]:off[i + 1]]), rel=1e-11)
    del dev, A, E
    a, b = W.QuasiNewtonLearner(0), W.QuasiNewtonLearner(0)
    for lrn in (a, b):
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        assert lrn.stats()["dense"] == 1
    rows_a = a.Run(2, 1.0, -1.0)
    rows_b = [b.OptimizationStep(1.0, -1.0)[0] for _ in range(2)]
    for r, q in zip(rows_a, rows_b):
        for u, v in zip(r[:5], q[:5]):
            assert _close(u, v, rel=1e-9, atol=1e-12)
    np.testing.assert_allclose(a.x(), b.x(), rtol=1e-9, atol=1e-11)


def _dense_expected_counts(A, E, start, end, s):
    """log q and the expected transition / emission counts of one string
    (numpy forward-backward, per-position scaling):
    C_A[S][T] = sum_i P(S at i, T at i+1), C_E[T][c] = sum_i P(T at i) [s_i = c]"""
    L = len(s)
    al = np.zeros((L, A.shape[0]))
    z = np.zeros(L)
    a = A[start] * E[:, s[0]]
    for i in range(L):
        if i > 0:
            a = al[i - 1] @ A * E[:, s[i]]
        z[i] = a.sum()
        al[i] = a / z[i]
    fin = al[L - 1] @ A[:, end]
    logq = np.log(z).sum() + np.log(fin)
    be = A[:, end] / fin          # beta_{L-1}, in the scale where al[i] * be[i] sums to 1
    CA = np.zeros_like(A)
    CE = np.zeros_like(E)
    CA[:, end] += al[L - 1] * A[:, end] / fin
    for i in range(L - 1, -1, -1):
        g = al[i] * be
        CE[:, s[i]] += g
        if i == 0:
            CA[start] += g
            break
        nxt = E[:, s[i]] * be / z[i]   # message into T at position i
        CA += np.outer(al[i - 1], nxt) * A
        be = A @ nxt
    return logq, CA, CE


def test_dense_c5_4096_gradient_per_element(monkeypatch):
    """per-parameter gradient at the c5 size (4096 states, full transition
    matrix, 16 symbols): 6 strings as their own corpus on the dense MFMA path
    against a numpy forward-backward of the same strings -- every transition
    (start, interior, end) and emission parameter, rel 1e-9"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=4096, degree=1, vocab=16, emissions=16, dense=True, n_strings=6, max_len=40, seed=5)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    n_par = fsa.counts()["parameters"]
    p = wt / wt.sum()
    w = np.random.default_rng(12).normal(-8.5, 1.0, size=n_par)
    dev = _device(fsa, sym, off, p, monkeypatch, dense=True)
    rec, _, _ = dev.recognize()
    assert rec.all()
    ll, grad, logq = dev.objective_grad(w)
    A, E, start, end, kind, index = _dense_tables(fsa, w, with_index=True)
    CA = np.zeros_like(A)
    CE = np.zeros_like(E)
    ll_ref = 0.0
    for i in range(len(wt)):
        lq, ca, ce = _dense_expected_counts(A, E, start, end, sym[off[i]:off[i + 1]])
        assert _close(logq[i], lq, rel=1e-11)
        ll_ref += p[i] * lq
        CA += p[i] * ca
        CE += p[i] * ce
    assert _close(ll, ll_ref, rel=1e-11)
    ref = np.zeros(n_par)
    src, dst, par = index["tr"]
    ok = par >= 0
    ref[par[ok]] -= CA[src[ok], dst[ok]]
    es, ec, ep = index["em"]
    ok = ep >= 0
    ref[ep[ok]] -= CE[es[ok], ec[ok]]
    assert (kind >= 0).all()
    for k in range(4):   # start, interior, end transitions and emissions all compared
        assert (kind == k).any()
    np.testing.assert_allclose(grad, ref, rtol=1e-9, atol=1e-15)


def test_dense_evaluation_is_bitwise_reproducible(monkeypatch):
    """the dense path's sums run in a fixed order -- the library GEMMs with
    atomics off, the epilogue row sums as fixed block trees: two evaluations
    of the same weights agree bit for bit"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=512, degree=1, vocab=16, emissions=16, dense=True, n_strings=600, max_len=40, seed=6)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    dev = _device(fsa, sym, off, wt / wt.sum(), monkeypatch, dense=True)
    dev.recognize()
    w = np.random.default_rng(3).normal(-6.0, 1.0, size=len(fsa.param_names()))
    ll1, g1, lq1 = dev.objective_grad(w)
    ll2, g2, lq2 = dev.objective_grad(w)
    assert ll1 == ll2
    np.testing.assert_array_equal(g1, g2)
    np.testing.assert_array_equal(lq1, lq2)


def _dense_min_rpp(A, E, start, end, s, logq):
    """the string's smallest relative path probability: a (min, +) forward
    in the log domain (missing edges +inf) over the same model"""
    with np.errstate(divide="ignore"):
        lA = np.where(A > 0, np.log(np.where(A > 0, A, 1.0)), np.inf)
        lE = np.where(E > 0, np.log(np.where(E > 0, E, 1.0)), np.inf)
    m = lA[start] + lE[:, s[0]]
    for c in s[1:]:
        m = np.min(m[:, None] + lA, axis=0) + lE[:, c]
    return float(np.exp(np.min(m + lA[:, end]) - logq))


def test_dense_rmin_matches_path_enumeration(monkeypatch):
    """the rmin info column on the dense path (its (min, +) trellis) against
    the oracle's enumerated paths (src/QuasiNewtonLearner.cpp:80-84, the
    reference's idamin over relative_path_probs), a 5-state model forced
    dense: value and the string holding the path"""
    from test_gpu_rmin import _check, _setup
    import wfsa_amd as W
    syn = W.Synthetic(n_states=5, degree=1, vocab=3, emissions=2, dense=True, n_strings=60, max_len=5, seed=9)
    sym, off, wt = syn.corpus()
    monkeypatch.setenv("WFSA_DENSE", "1")
    o, h, dev = _setup(syn.wfsa_text, sym, off, wt, monkeypatch)
    assert dev.stats()["dense"] == 1
    _check(o, h, dev, seed=3)


def test_dense_rmin_equals_sparse_kernels(monkeypatch):
    """same model and strings: the dense path's rmin equals the trellis
    kernels' (min, x) passes (traversal tiers), value and string"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=16, degree=1, vocab=6, emissions=2, dense=True, n_strings=400, max_len=9, seed=4)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    names = fsa.param_names()
    p = wt / wt.sum()
    sp = _device(fsa, sym, off, p, monkeypatch, dense=False)
    dn = _device(fsa, sym, off, p, monkeypatch, dense=True)
    rec, _, _ = dn.recognize()
    assert rec.all()
    with pytest.raises(Exception):   # structural pass only: no weights yet
        dn.rmin()
    rng = np.random.default_rng(6)
    for _ in range(3):
        w = rng.normal(-0.8, 0.6, size=len(names))
        sp.objective_grad(w)
        dn.objective_grad(w)
        (rs, ss), (rd, sd) = sp.rmin(), dn.rmin()
        assert _close(rd, rs, rel=1e-12) and 0.0 < rd < 1.0
        assert sd == ss


def test_dense_rmin_two_column_tiles_against_numpy(monkeypatch):
    """200 states (np 256: two column tiles, padded states), ragged row
    slots: the device's rmin equals a numpy (min, +) restatement per string"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=200, degree=1, vocab=5, emissions=2, dense=True, n_strings=300, max_len=40, seed=12)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    p = wt / wt.sum()
    dev = _device(fsa, sym, off, p, monkeypatch, dense=True)
    dev.recognize()
    w = np.random.default_rng(8).normal(-1.5, 0.9, size=len(fsa.param_names()))
    _, _, logq = dev.objective_grad(w)
    r, s = dev.rmin()
    A, E, start, end, _ = _dense_tables(fsa, w)
    want = np.array([_dense_min_rpp(A, E, start, end, sym[off[i]:off[i + 1]], logq[i]) for i in range(len(wt))])
    i = int(np.argmin(want))
    assert _close(r, want[i], rel=1e-11)
    assert s == i or _close(want[s], want[i], rel=1e-11)


def test_dense_rmin_column_in_quasinewton_device_loop(monkeypatch):
    """QuasiNewtonLearner with the rmin column on: the dense path's device
    loop fills columns 5/6 as the trellis kernels' loop does"""
    import wfsa_amd as W
    syn = W.Synthetic(n_states=16, degree=1, vocab=8, emissions=2, dense=True, n_strings=300, max_len=9, seed=21)
    sym, off, wt = syn.corpus()
    fsa = W.Fsa.read_text(syn.wfsa_text)
    rows = {}
    for dense in (False, True):
        monkeypatch.setenv("WFSA_DENSE", "1" if dense else "0")
        lrn = W.QuasiNewtonLearner(0)
        lrn.set_info_rmin(True)
        lrn.BuildFromPacked(fsa, sym, off, wt)
        lrn.Finalize()
        lrn.Init(7)
        assert lrn.stats()["dense"] == (1 if dense else 0)
        rows[dense] = np.array([lrn.OptimizationStep(1.0, -1.0)[0] for _ in range(2)] + lrn.Run(4, 1.0, -1.0))
    assert (rows[True][:, 6] >= 0).all() and (rows[True][:, 5] < 1.0).all()
    np.testing.assert_allclose(rows[True][:, 5], rows[False][:, 5], rtol=1e-9)
    np.testing.assert_array_equal(rows[True][:, 6], rows[False][:, 6])
