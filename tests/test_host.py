"""CPU tests of the product's host side: the C-ABI library loads and exports
what include/*.h declares, the .wfsa/.corpus readers and parameter numbering
match the reference (via the oracle and Appendix A), the trellis compiler,
sharding, the synthetic generator and the CLI's device-free paths."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import DATA, ROOT

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "appendix_a.json")))
PAIRS = [("test", "test"), ("test.list", "test"), ("test2", "test"), ("test3", "test"), ("test4", "test"),
         ("test.loop", "test"), ("talk", "talk"), ("talk", "test"), ("test5", "test5"), ("test5_2", "test5")]
CLI = os.path.join(ROOT, "w-fsa_amd", "wfsa_amd", "wfsa")


def declared_functions():
    names = []
    for h in ("wfsa_dev.h", "wfsa_host.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(wfsa_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    import ctypes
    import wfsa_amd
    lib = wfsa_amd.load()
    names = declared_functions()
    assert len(names) >= 40
    for n in names:
        assert hasattr(lib, n), n
        assert n in wfsa_amd._lib.EXPORTS, f"{n} not bound in _lib.py"
    nm = subprocess.run(["nm", "-D", "--defined-only", wfsa_amd._lib.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", nm), n
    assert ctypes.sizeof(wfsa_amd._lib.ModelDesc) == 4 * 4 + 8 * 8


def test_device_calls_fail_loudly_without_gpu():
    import wfsa_amd as W
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(W.WfsaError, match="no HIP device|gfx950"):
        W.Device(0)


@pytest.mark.parametrize("a,c", PAIRS)
def test_readers_match_oracle(a, c):
    import wfsa_amd as W
    from oracle import Oracle
    fsa = W.Fsa.read_file(os.path.join(DATA, a + ".wfsa"))
    o = Oracle.from_files(os.path.join(DATA, a + ".wfsa"), os.path.join(DATA, c + ".corpus"))
    cnt = fsa.counts()
    assert cnt["states"] == o.info["n_states"]
    assert cnt["parameters"] == o.info["n_full"]
    assert sorted(fsa.param_names()) == sorted(o.full_param_names())
    corpus = W.Corpus.read_file(os.path.join(DATA, c + ".corpus"))
    strings, w = corpus.strings()
    assert len(strings) == o.info["n_corpus"]


def test_corpus_quirks():
    """tokens are concatenated, the last token is the weight, a trailing
    separator yields an empty extra line (src/Corpus.cpp:21-53)"""
    import wfsa_amd as W
    c = W.Corpus.read_file(os.path.join(DATA, "test.corpus"))
    strings, w = c.strings()
    assert strings == ["a", "aa", "aaa", "ab", "b", "bc", "bd"]
    np.testing.assert_allclose(w, [1, 1, 1, 1, 1, 2, 0.3])
    strings, w = W.Corpus.read_text("::\nta::lk::3\nx::1\n").strings()
    assert strings == ["talk", "x"] and list(w) == [3.0, 1.0]
    with pytest.raises(W.WfsaError, match="duplicate"):
        W.Corpus.read_text("\na 1\na 2\n")
    with pytest.raises(W.WfsaError, match="probability"):
        W.Corpus.read_text("\na 0\n")


def test_fsa_errors_like_reference():
    import wfsa_amd as W
    with pytest.raises(W.WfsaError, match="Start state should emit empty string"):
        W.Fsa.read_text("\n^\n$\n^ a 0\n^ X 0\n")
    with pytest.raises(W.WfsaError, match="connects to start state"):
        W.Fsa.read_text("\n^\n$\n^  0\n^ X 0\nX a 0\nX ^ 0\n")
    with pytest.raises(W.WfsaError, match="appears more than once"):
        W.Fsa.read_text("\n^\n$\n^  0\n^ X 0\nX a 0 a 1\nX $ 0\n")
    with pytest.raises(W.WfsaError, match="Start and end states should be different"):
        W.Fsa.read_text("\n^\n^\n\n")  # (a separator right before EOF is not cut: GetWord quirk)


def test_parameter_numbering_is_the_references():
    """Appendix A lists talk's gradient in the reference's own index order
    (unordered_map iteration under the FNV hash).  Map the oracle's
    name-keyed gradient onto the product's numbering: it must reproduce that
    exact vector."""
    import wfsa_amd as W
    from oracle import Oracle
    case = next(c for c in GOLD["cases"] if c["wfsa"] == "talk" and c["corpus"] == "talk")
    fsa = W.Fsa.read_file(os.path.join(DATA, "talk.wfsa"))
    o = Oracle.from_files(os.path.join(DATA, "talk.wfsa"), os.path.join(DATA, "talk.corpus"))
    o.qn_init(7)
    o.objective_grad()
    by_name = dict(zip(o.param_names(), o.grad()))
    ours = [by_name[n] for n in fsa.param_names()]
    np.testing.assert_allclose(ours, case["grad_index_order"], rtol=1e-12)


def test_trellis_compiler():
    import wfsa_amd as W
    fsa = W.Fsa.read_file(os.path.join(DATA, "talk.wfsa"))
    nodes, edges, ends, plist = W.trellis_stats(fsa)
    # 6 states + chain nodes of "talk" (3) x 2 + "ed" (1) = 13
    assert nodes == 13
    assert ends == 4 and edges > 0 and plist >= 7
    with pytest.raises(W.WfsaError, match="epsilon cycle"):
        W.trellis_stats(W.Fsa.read_text("\n^\n$\n^  0\n^ A 0\nA  0 a 0\nA B 0 $ 0\nB  0\nB A 0\n"))
    # epsilon chains are fine
    W.trellis_stats(W.Fsa.read_text("\n^\n$\n^  0\n^ A 0\nA  0 a 0\nA B 0 $ 0\nB  0\nB $ 0\n"))


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_shard_ranges_partition_and_balance(nranks):
    import wfsa_amd as W
    rng = np.random.default_rng(nranks)
    lens = rng.integers(1, 100, size=5000)
    off = np.concatenate([[0], np.cumsum(lens)])
    prev = 0
    loads = []
    for r in range(nranks):
        b, e = W.shard_range(off, nranks, r)
        assert b == prev and e >= b
        prev = e
        loads.append(off[e] - off[b])
    assert prev == 5000
    assert max(loads) - min(loads) <= 2 * lens.max()


def test_synthetic_generator():
    import wfsa_amd as W
    a = W.Synthetic(n_states=64, degree=4, vocab=16, n_strings=2000, seed=7)
    b = W.Synthetic(n_states=64, degree=4, vocab=16, n_strings=2000, seed=7)
    sa, oa, wa = a.corpus()
    sb, ob, wb = b.corpus()
    assert a.wfsa_text == b.wfsa_text
    assert np.array_equal(sa, sb) and np.array_equal(oa, ob) and np.array_equal(wa, wb)
    strs = {bytes(sa[oa[i]:oa[i + 1]]) for i in range(len(wa))}
    assert len(strs) == 2000
    assert wa.min() >= 1 and wa.max() <= 10
    from oracle import Oracle, TRELLIS
    o = Oracle.from_arrays(a.wfsa_text, sa[:oa[200]], oa[:201], wa[:200], mode=TRELLIS)
    assert o.info["n_strings"] == 200       # every sampled string is in the language


def test_cli_help_and_missing_input():
    """the reference's `testhelp` CTest; a missing file exits 1"""
    if not os.path.exists(CLI):
        pytest.skip("CLI not built")
    assert subprocess.run([CLI, "-h"], capture_output=True).returncode == 0
    r = subprocess.run([CLI, "-a", os.path.join(DATA, "talk.wfsa"), "-c", "/nonexistent.corpus"],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "Unable to open" in r.stderr
    r = subprocess.run([CLI, "-opt", "Hessian", "-a", "x", "-c", "y"], capture_output=True, text=True)
    assert r.returncode == 1


def test_crlf_automaton_fails_like_reference():
    """data/test.wfsa.win (CRLF): the separator line is "\\r", so the start
    line's emission runs into the next line; the parse stops at the reference's
    "transitions after emissions" check (fails to parse)."""
    import wfsa_amd as W
    with pytest.raises(W.WfsaError, match='You should enlist transitions of "a" after emissions of the same state!'):
        W.Fsa.read_file(os.path.join(DATA, "test.wfsa.win"))


def test_bench_never_reports_more_gpus_than_rank_processes():
    """bench.py --gpus N (N > 1) without a launcher starts its own ranks or
    refuses; on a node with fewer GPUs it refuses (exit 2) instead of
    reporting N GPUs from one process"""
    import subprocess
    import sys
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "refusing" in r.stderr and r.stdout.strip() == ""
    # a launcher's WORLD_SIZE that disagrees with --gpus is refused too
    env2 = dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       capture_output=True, text=True, env=env2, timeout=120)
    assert r.returncode == 2 and "refusing" in r.stderr
    # work-skipping experiment knobs are refused
    env3 = dict(env, WFSA_FBS_DBG="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")], capture_output=True, text=True, env=env3,
                       timeout=120)
    assert r.returncode == 2 and "WFSA_FBS_DBG" in r.stderr
