"""Scratch diagnostic: bundle-scan window counts vs the per-read scan."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "telomere-analyzer_amd"))
import numpy as np, torch
import _oracle as O
from nanotel_amd import NanoTel
os.environ["NT_JIT"] = "1"
def run(seqs, **kw):
    nt = NanoTel(**kw)
    assert nt.tscan
    a = nt.analyze(seqs, want_windows=True, want_hits=True)
    b = nt.analyze(seqs, want_windows=True, want_hits=False)
    nbad = 0
    for i in range(len(seqs)):
        for p in range(nt.n_pass):
            x = np.array(nt.window_counts(a, i, p), np.int64); y = np.array(nt.window_counts(b, i, p), np.int64)
            d = np.nonzero(x != y)[0]
            if len(d):
                nbad += 1
                if nbad < 12:
                    print("read", i, "len", len(seqs[i]), "pass", p, "ndiff", len(d), "of", len(x),
                          "hs with diffs", sorted(set(int(j) // 32 for j in d)), "of", (len(x) + 31) // 32,
                          [(int(j), int(x[j]), int(y[j])) for j in d[:6]])
    print(kw, "reads with diffs", nbad)
    nt.close()
rng = np.random.default_rng(5)
seqs2 = ["".join(rng.choice(list("ACGT"), int(n))) for n in rng.integers(50, 9000, 64)]
seqs2 = [("TTAGGG" * 300)[: len(s) // 3] + s for s in seqs2]
run(seqs2, patterns="TTAGGG TTAGGGTTAGGG TTAGG", subseq_length=50, min_density=0.5)
lens = [len(s) for s in seqs2]
print("bundle order (longest first):", sorted(range(len(lens)), key=lambda r: -lens[r]))
