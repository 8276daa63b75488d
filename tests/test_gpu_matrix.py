"""GPU tests of matrix-file mode (Learner::LoadMatrices,
src/Learner.cpp:125-199; main.cpp -m): the reference's path matrices, written
from the oracle's enumeration in the reference's text format
(tests/matrix_io.py), loaded through the C ABI and the CLI; the device's SpMV
chain against the oracle -- objective/gradient at random x, QuasiNewton
epochs including the rmin column with the reference's own path index, and
Appendix A's final KL.  Needs a gfx950 device."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import DATA, ROOT

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "appendix_a.json")))
CASES = [c for c in GOLD["cases"] if not c.get("empty")]
CLI = os.path.join(ROOT, "w-fsa_amd", "wfsa_amd", "wfsa")


def _oracle(case):
    from oracle import Oracle
    return Oracle.from_files(os.path.join(DATA, case["wfsa"] + ".wfsa"), os.path.join(DATA, case["corpus"] + ".corpus"))


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['wfsa']}+{c['corpus']}")
def test_device_paths_objective_matches_oracle(case):
    import wfsa_amd as W
    o = _oracle(case)
    prow, pcol, pdata, mrow = o.paths()
    dev = W.Device(0)
    dev.load_paths(o.n, prow, pcol, pdata, mrow, np.arange(mrow[-1]), o.p())
    rec, pc, used = dev.recognize()
    assert rec.all()
    np.testing.assert_array_equal(pc, np.diff(mrow))
    rng = np.random.default_rng(11)
    for _ in range(3):
        x = rng.normal(-1.0, 0.5, size=o.n)
        o.set_x(x)
        kl, ll = o.objective_grad()
        got_ll, got_g, got_lq = dev.objective_grad(x)
        assert abs(got_ll - ll) <= 1e-13 * abs(ll)
        np.testing.assert_allclose(got_g, o.grad(), rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(got_lq, o.logq(), rtol=1e-13, atol=1e-15)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['wfsa']}+{c['corpus']}")
def test_quasinewton_from_matrix_files(case, tmp_path):
    """QN epochs over loaded matrices == the oracle's QN run; rmin column ==
    min relative path probability before each step with the reference's path
    index; final KL == Appendix A"""
    import wfsa_amd as W
    from matrix_io import write_matrices
    from oracle.hessian import HessianOracle
    o = _oracle(case)
    prefix = str(tmp_path / "m")
    write_matrices(o, prefix)
    h = HessianOracle(o)
    o.qn_init(7)
    want, rmin = [], []
    for _ in range(20):
        h.x = o.x()
        _, rpp = h.modeled()
        if h.unique:
            rmin.append((0.0, 0.0))
        else:
            i = int(np.argmin(rpp))
            rmin.append((rpp[i], float(i)))
        want.append(o.qn_step(1.0))
        if o.qn_halt(1e-6):
            break
    lrn = W.QuasiNewtonLearner(0, optimizer="QuasiNewton")
    lrn.LoadMatrices(prefix)
    lrn.Finalize()
    rows = np.array(lrn.run(flags=7, epochs=20, tol=1e-6))
    want = np.array(want)
    assert rows.shape[0] == want.shape[0] == case["epochs"]
    np.testing.assert_allclose(rows[:, 0], want[:, 0], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(rows[:, 1:5], want[:, 1:5], rtol=1e-7, atol=1e-11)
    np.testing.assert_allclose(rows[:, 5], [r[0] for r in rmin], rtol=1e-9)
    np.testing.assert_array_equal(rows[:, 6], [r[1] for r in rmin])
    assert abs(rows[-1, 0] - case["kl_final"]) <= 1e-9 * max(1.0, abs(case["kl_final"]))
    # the loaded matrices save back unchanged (the reference's text format)
    lrn.SaveMatrices(str(tmp_path / "again"))
    for ext in (".C", ".M", ".P"):
        a = open(prefix + ext).read().split()
        b = open(str(tmp_path / "again") + ext).read().split()
        assert len(a) == len(b) and np.allclose(np.array(a, dtype=float), np.array(b, dtype=float), rtol=1e-14)


def test_cli_matrix_mode_talk(tmp_path):
    """`wfsa -m <prefix -n -eval -e 20 -i 31` (default HessianLearner): the
    Result line of SURVEY Appendix A's talk vector (logdetH: numerically
    singular, see tests/test_gpu_hessian.py), x and lambda on stdout"""
    from matrix_io import write_matrices
    case = [c for c in CASES if c["wfsa"] == "talk"][0]
    o = _oracle(case)
    prefix = str(tmp_path / "talk")
    write_matrices(o, prefix)
    r = subprocess.run([CLI, "-m", "<" + prefix, "-n", "-eval", "-e", "20", "-i", "31"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Loading matrices" in r.stderr and "unique paths: false" in r.stderr
    line = [l for l in r.stderr.splitlines() if l.startswith("Result:")][-1]
    got = np.array([float(v) for v in line.split()[1:]])
    want = np.array(GOLD["talk_hessian_result"]["result"])
    keep = [0, 1, 2, 3, 5, 6, 7]
    np.testing.assert_allclose(got[keep], want[keep], rtol=5e-13, atol=1e-14)
    assert got[4] == np.inf or got[4] < -15.0
    out = r.stdout.split("\n")
    assert len(out[0].split()) == o.n and len(out[1].split()) == o.info["n_constraints"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['wfsa']}+{c['corpus']}")
def test_hessian_from_matrix_files(case, tmp_path):
    """HessianLearner over loaded matrices (H_f from the paths on the device)
    epoch by epoch against the dense restatement -- including test5, whose
    ambiguity region no compiled bubble holds in automaton mode"""
    import wfsa_amd as W
    from matrix_io import write_matrices
    from oracle.hessian import HessianOracle
    o = _oracle(case)
    prefix = str(tmp_path / "m")
    write_matrices(o, prefix)
    h = HessianOracle(o)
    want = np.array(h.run(flags=31, epochs=20, tol=1e-6))
    lrn = W.HessianLearner(0)
    lrn.LoadMatrices(prefix)
    lrn.Finalize()
    got = np.array(lrn.run(flags=31, epochs=20, tol=1e-6))
    assert got.shape == want.shape
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(got[:, 4:6], want[:, 4:6])
    np.testing.assert_allclose(got[:, 7], want[:, 7], rtol=1e-8, atol=1e-300)
    np.testing.assert_array_equal(got[:, 8], want[:, 8])   # the reference's path index


def test_cli_matrix_mode_missing_file(tmp_path):
    r = subprocess.run([CLI, "-m", "<" + str(tmp_path / "nope")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Unable to open" in r.stderr
