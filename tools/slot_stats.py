import os, sys
sys.path.insert(0, "w-fsa_amd")
import wfsa_amd as W
syn = W.Synthetic(n_states=1024, degree=8, vocab=64, emissions=1, n_strings=1000000, max_len=128, seed=1)
sym, off, wt = syn.corpus()
fsa = W.Fsa.read_text(syn.wfsa_text)
lrn = W.QuasiNewtonLearner(0)
lrn.BuildFromPacked(fsa, sym, off, wt)
lrn.Finalize()
lrn.Init(7)
lrn.Run(3, 1.0, -1.0)
st = lrn.stats()
print({k: st[k] for k in ("n_bubbles", "bubble_words", "slot_chunks", "max_group_chunks", "stream_bytes")}, lrn.info()["n_constraints"])
