import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "w-fsa_amd"); sys.path.insert(0, ".")
import wfsa_amd as W
from test_gpu_ranks import _recognized
fams = [dict(n_states=20, degree=4, vocab=6, emissions=2, n_strings=300, max_len=12),
        dict(n_states=8, degree=2, vocab=4, emissions=1, n_strings=200, max_len=8),
        dict(n_states=64, degree=4, vocab=16, emissions=1, n_strings=400, max_len=10),
        dict(n_states=16, degree=3, vocab=8, emissions=1, n_strings=2000, max_len=16),
        dict(n_states=32, degree=4, vocab=16, emissions=1, n_strings=3000, max_len=20)]
for f in fams:
    for flags in (31, 15, 7):
        syn = W.Synthetic(seed=3, **f)
        sym, off, p, _ = _recognized(syn)
        fsa = W.Fsa.read_text(syn.wfsa_text)
        l = W.HessianLearner(0)
        l.BuildFromPacked(fsa, sym, off, p); l.Finalize()
        try:
            rows = l.run(flags=flags, epochs=8, tol=1e-9)
            print(f, flags, "OK", len(rows), len(off)-1, rows[-1][:3])
        except Exception as e:
            print(f, flags, "ERR", e)
