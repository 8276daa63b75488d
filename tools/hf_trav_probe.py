"""Which synthetic families put strings on the traversal tiers and still let
the Hessian restatement converge (a candidate list for tests/test_gpu_hessian.py)."""
import sys
import warnings

import numpy as np

sys.path.insert(0, "w-fsa_amd")
sys.path.insert(0, ".")
warnings.simplefilter("ignore")
import wfsa_amd as W  # noqa: E402
from oracle import Oracle  # noqa: E402
from oracle.hessian import HessianOracle  # noqa: E402

FAMS = [dict(n_states=16, degree=2, vocab=4, emissions=2, n_strings=200, max_len=16, seed=4),
        dict(n_states=10, degree=3, vocab=4, emissions=1, n_strings=200, max_len=14, seed=3),
        dict(n_states=16, degree=3, vocab=4, emissions=2, n_strings=100, max_len=12, seed=3),
        dict(n_states=12, degree=3, vocab=3, emissions=2, n_strings=150, max_len=24, seed=3)]
for fam in FAMS:
    syn = W.Synthetic(**fam)
    sym, off, wt = syn.corpus()
    dev = W.Device(0)
    dev.load_model(W.Fsa.read_text(syn.wfsa_text))
    dev.load_corpus(sym, off, wt / wt.sum())
    dev.recognize()
    tiers = dev.string_tiers()
    msg = f"{fam} tiers {np.bincount(tiers + 1).tolist()}"
    try:
        h = HessianOracle(Oracle.from_arrays(syn.wfsa_text, sym, off, wt, max_paths=3_000_000))
        want = np.array(h.run(flags=31, epochs=20, tol=1e-6))
        msg += f" oracle ok {len(want)} epochs"
    except Exception as e:  # noqa: BLE001
        msg += f" oracle {e}"
    lrn = W.HessianLearner(0)
    lrn.BuildFromPacked(W.Fsa.read_text(syn.wfsa_text), sym, off, wt)
    lrn.Finalize()
    try:
        got = np.array(lrn.run(flags=31, epochs=20, tol=1e-6))
        msg += f" ours ok {len(got)} epochs KL {got[-1, 0]:.12g}"
        if "oracle ok" in msg:
            msg += f" maxdiff KL {np.abs(got[:, 0] - want[:len(got), 0]).max():.3g}"
    except Exception as e:  # noqa: BLE001
        msg += f" ours {e}"
    print(msg, flush=True)
