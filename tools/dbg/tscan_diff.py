"""Debug aid: window counts of the bundle scan vs the per-read scan, per read."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O
from nanotel_amd import NanoTel

names, seqs = O.read_fasta(os.path.join(ROOT, "tests", "golden", "sample.fasta"))
extra = []
rng = np.random.default_rng(3)
for n in (2981, 3000, 6400, 6450, 10000):
    extra.append("".join("ACGT"[i] for i in rng.integers(0, 4, n)))
for label, ss in (("example", seqs), ("random", extra), ("uniform", [extra[2]] * 32)):
    nt = NanoTel(patterns="TTAGGG")
    a = nt.analyze(ss, want_windows=True, want_hits=True)
    b = nt.analyze(ss, want_windows=True, want_hits=False)
    print(label, "tscan", nt.tscan)
    for i in range(len(ss)):
        for p in range(2):
            x = nt.window_counts(a, i, p).astype(int)
            y = nt.window_counts(b, i, p).astype(int)
            d = np.nonzero(x != y)[0]
            if d.size:
                print(f"  read {i} len {len(ss[i])} pass {p}: {d.size} windows differ, first {d[:8].tolist()}"
                      f" legacy {x[d[:8]].tolist()} tscan {y[d[:8]].tolist()}")
        if i > 3:
            break
