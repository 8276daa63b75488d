"""CLI output parity through the wfsa binary:
  * -m >prefix after -a/-c: the path matrices enumerated on the host
    (Paths.hpp) equal the oracle's (the reference's BuildPaths + Trim,
    src/Learner.cpp:276-425) entry for entry, and reload through -m <prefix;
  * -p: the recognized-path listing (src/main.cpp:178-203) and the C / M / P
    printout (:231-239, PrintCsrMtx src/Utils.cpp:157-182) against the oracle's
    path matrices; the Hessian's KKT printout (PrintEq / PrintH);
  * -o: Dump after RewriteWeights (src/Fsa.cpp:47-71, src/Learner.cpp:45-58)
    against the weights the oracle's optimisation implies;
  * the CRLF automaton data/test.wfsa.win fails to parse, as the reference's
    tokenizer makes it.
The binary runs BuildFrom on the GPU: these tests need a gfx950 device."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import DATA, ROOT
from matrix_io import read_csr

pytestmark = pytest.mark.gpu

CLI = os.path.join(ROOT, "w-fsa_amd", "wfsa_amd", "wfsa")
PAIRS = [("talk", "talk"), ("test3", "test"), ("test.loop", "test"), ("test4", "test"), ("test5", "test5")]


def _run(*args):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=120)
    return r.returncode, r.stdout, r.stderr


def _files(wfsa, corpus):
    return os.path.join(DATA, wfsa + ".wfsa"), os.path.join(DATA, corpus + ".corpus")


def _oracle(wfsa, corpus):
    from oracle import ENUM, Oracle
    a, c = _files(wfsa, corpus)
    return Oracle.from_files(a, c, mode=ENUM, max_paths=10_000_000)


def _our_names(wfsa, corpus):
    """trimmed parameter index -> (state, kind, label) in this build's numbering
    (the reference's: Fsa::AssignIndices over its hash-map order)"""
    import wfsa_amd as W
    a, c = _files(wfsa, corpus)
    lrn = W.QuasiNewtonLearner(0)
    lrn.BuildFrom(W.Fsa.read_file(a), W.Corpus.read_file(c))
    return lrn.param_names()


def _strings(prow, pcol, pdata, mrow, p, names):
    """multiset over recognized strings of (p_s, its paths as name -> count);
    the oracle numbers parameters and orders strings its own way, so the
    comparison is by name"""
    out = []
    for s in range(len(mrow) - 1):
        paths = []
        for l in range(mrow[s], mrow[s + 1]):
            paths.append(tuple(sorted((names[int(pcol[q])], float(pdata[q])) for q in range(prow[l], prow[l + 1]))))
        out.append((round(float(p[s]), 12), tuple(sorted(paths))))
    return sorted(out)


def _groups(ccol, names):
    g = {}
    for j, c in enumerate(ccol):
        g.setdefault(int(c), set()).add(names[j])
    return sorted(sorted(v) for v in g.values())


@pytest.mark.parametrize("wfsa,corpus", PAIRS)
def test_save_matrices_after_buildfrom(wfsa, corpus, tmp_path):
    a, c = _files(wfsa, corpus)
    prefix = str(tmp_path / "m")
    rc, _, err = _run("-a", a, "-c", c, "-opt", "QuasiNewton", "-e", "0", "-s", "-m", ">" + prefix)
    assert rc == 0, err
    assert f'Saving matrices "{prefix}" ... Done' in err
    names = _our_names(wfsa, corpus)
    o = _oracle(wfsa, corpus)
    onames = o.param_names()
    prow, pcol, pdata = read_csr(prefix + ".P")
    mrow, mcol, _ = read_csr(prefix + ".M")
    np.testing.assert_array_equal(mcol, np.arange(mrow[-1]))   # path l is column l
    prob = np.loadtxt(prefix + ".prob", ndmin=1)
    assert _strings(prow, pcol, pdata, mrow, prob, names) == _strings(*o.paths(), o.p(), onames)
    crow, ccol, _ = read_csr(prefix + ".C")
    np.testing.assert_array_equal(crow, np.arange(o.n + 1))
    assert _groups(ccol, names) == _groups(o.ccol(), onames)
    aux = open(prefix + ".aux").read().split()
    i = o.info
    for got, want in zip(aux[:4], (i["common_support"], i["plogp"], i["model_volume"], i["aux_hessian"])):
        assert math.isclose(float(got), want, rel_tol=1e-13, abs_tol=1e-15)
    assert int(aux[4]) == i["aux_params"]
    # and back: the saved files drive the matrix-file mode through the same epochs
    # (-i 1: uniform start on both sides -- matrix files carry no weights)
    rc1, _, e1 = _run("-a", a, "-c", c, "-opt", "QuasiNewton", "-e", "3", "-i", "1", "-s")
    rc2, _, e2 = _run("-m", "<" + prefix, "-opt", "QuasiNewton", "-e", "3", "-i", "1", "-s")
    assert rc1 == rc2 == 0, (e1, e2)
    # (all columns but the last: the rmin index is the string holding the path
    # from an automaton, the reference's path index from matrices -- DESIGN 3d)
    table = lambda e: [ln.split()[:-1] for ln in e.splitlines() if re.match(r"^\d+\t", ln)]
    assert table(e1) == table(e2) and len(table(e1)) > 0


def _section(err, name, stop):
    lines = err.splitlines()
    i = lines.index(name + ":")
    out = []
    for ln in lines[i + 1:]:
        if ln.startswith(stop):
            break
        out.append(ln)
    return out


def _dense(lines, ncols):
    """PrintCsrMtx rows back to a dense matrix: 8 characters per column"""
    m = np.zeros((len(lines), ncols))
    for r, ln in enumerate(lines):
        for j in range(0, len(ln), 8):
            tok = ln[j:j + 7].strip()
            if tok:
                m[r, j // 8] = float(tok)
    return m


def _csr(dense):
    rows, cols, data = [0], [], []
    for r in dense:
        nz = np.flatnonzero(r)
        cols += list(nz)
        data += list(r[nz])
        rows.append(len(cols))
    return np.array(rows), np.array(cols), np.array(data)


@pytest.mark.parametrize("wfsa,corpus", [("talk", "talk"), ("test3", "test"), ("test5", "test5")])
def test_print_paths_and_matrices(wfsa, corpus):
    a, c = _files(wfsa, corpus)
    rc, _, err = _run("-a", a, "-c", c, "-opt", "QuasiNewton", "-e", "1", "-s", "-p")
    assert rc == 0, err
    names = _our_names(wfsa, corpus)
    o = _oracle(wfsa, corpus)
    oprow, opcol, opdata, omrow = o.paths()
    n_paths, n, S = len(oprow) - 1, o.n, len(omrow) - 1
    # the listing: one line per accepting path, "<emitted>: <start> -> <state>"<emission>" ..."
    listing = [ln for ln in err.splitlines() if re.match(r'^[^\t]*: \^( -> |$)', ln)]
    assert len(listing) == n_paths
    counts = {}
    for ln in listing:
        assert ln.endswith(" -> $")
        w = ln.split(": ", 1)[0]
        counts[w] = counts.get(w, 0) + 1
    assert sorted(counts.values()) == sorted(int(v) for v in np.diff(omrow))
    # C, M, P (PrintCsrMtx), against the oracle's matrices by parameter name
    C = _dense(_section(err, "C", "M:"), o.info["n_constraints"])
    assert (C.sum(axis=1) == 1).all()
    assert _groups(C.argmax(axis=1), names) == _groups(o.ccol(), onames := o.param_names())
    M = _dense(_section(err, "M", "P:"), n_paths)
    assert M.shape == (S, n_paths) and (M.sum(axis=0) == 1).all()
    mrow = np.concatenate([[0], np.cumsum(M.sum(axis=1))]).astype(int)
    for s in range(S):   # each string's paths are consecutive columns
        assert (M[s, mrow[s]:mrow[s + 1]] == 1).all()
    prow, pcol, pdata = _csr(_dense(_section(err, "P", "Initialize"), n))
    p_ours = np.zeros(S)   # the string identity is carried by the path sets themselves
    p_or = np.zeros(S)
    assert _strings(prow, pcol, pdata, mrow, p_ours, names) == _strings(oprow, opcol, opdata, omrow, p_or, onames)


def test_print_recognize_depth_first_and_hessian_kkt():
    a, c = _files("test5", "test5")
    rc, _, bfs = _run("-a", a, "-c", c, "-opt", "QuasiNewton", "-e", "0", "-s", "-pr")
    rc2, _, dfs = _run("-a", a, "-c", c, "-opt", "QuasiNewton", "-e", "0", "-s", "-pr", "-r", "1")
    assert rc == rc2 == 0
    pick = lambda e: [ln for ln in e.splitlines() if re.match(r'^[^\t]*: \^( -> |$)', ln)]
    assert sorted(pick(bfs)) == sorted(pick(dfs)) and len(pick(bfs)) > 0   # same paths, either order
    # the Hessian's KKT system each step (PrintEq) and its log-det Hessian (PrintH)
    a, c = _files("talk", "talk")
    rc, _, err = _run("-a", a, "-c", c, "-e", "1", "-i", "15", "-s", "-p", "-eval")
    assert rc == 0, err
    o = _oracle("talk", "talk")
    n, k = o.n, o.info["n_constraints"]
    kkt = [ln for ln in _section(err, "H", "1\t") if "|" in ln]
    assert len(kkt) == n + k
    H = _dense([ln.split("|")[0] for ln in kkt], n + k)
    assert (H[:n, n:] > 0).sum(axis=1).tolist() == [1] * n   # exp(x_i) in its constraint's column
    assert (H[n:, :n] == 0).all()                              # the upper triangle only
    hess = err.splitlines()
    j = hess.index("Hessian:")
    assert hess[j + 1].strip() == f"rows: {n}"


def _dumped_weights(path):
    """(state, kind, label) -> weight from a Dump (src/Fsa.cpp:47-71)"""
    lines = open(path, encoding="latin-1").read().split("\n")
    sep = lines[0] if lines[0] else " "
    end = lines[2]
    out = {}
    body = [ln for ln in lines[3:] if ln != ""]
    for em, tr in zip(body[0::2], body[1::2]):
        t = em.split(sep)
        state = t[0]
        for name, w in zip(t[1::2], t[2::2]):
            out[(state, "E", name)] = float(w)
        t = tr.split(sep)
        for name, w in zip(t[1::2], t[2::2]):
            out[(state, "T", name)] = float(w)
    return out, end


@pytest.mark.parametrize("wfsa,corpus", [("talk", "talk"), ("test3", "test")])
def test_dump_after_rewrite_weights(wfsa, corpus, tmp_path):
    a, c = _files(wfsa, corpus)
    out = str(tmp_path / "out.wfsa")
    rc, _, err = _run("-a", a, "-c", c, "-opt", "QuasiNewton", "-e", "4", "-o", out)
    assert rc == 0, err
    o = _oracle(wfsa, corpus)
    o.qn_run(flags=0, epochs=4)
    x = o.x()
    trim = o.trimmed_index()
    want = {}
    for name, t in zip(o.full_param_names(), trim):
        want[name] = x[t] if t >= 0 else (0.0 if t == -1 else -math.inf)
    got, end = _dumped_weights(out)
    assert end == "$"
    assert set(want) <= set(got)
    for key, w in got.items():
        e = want.get(key, 0.0)   # unequivocal edges: log 1
        if math.isinf(e):
            assert w == e, key
        else:
            assert math.isclose(w, e, rel_tol=2e-5, abs_tol=2e-6), (key, w, e)


def test_crlf_automaton_fails_to_parse():
    """data/test.wfsa.win: CRLF line ends.  The tokenizer splits on the first
    line's separator, "\\r" here, so the start line's emission swallows the
    next line and the parse fails -- the reference's outcome."""
    a = os.path.join(DATA, "test.wfsa.win")
    c = os.path.join(DATA, "test.corpus")
    rc, _, err = _run("-a", a, "-c", c, "-s")
    assert rc == 1
    assert 'Invalid FSA format! You should enlist transitions of "a" after emissions of the same state!' in err
