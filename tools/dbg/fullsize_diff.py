"""Debug aid: bundle scan vs per-read scan on a large c4-shaped batch; prints the reads that differ."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from nanotel_amd import synth_params  # noqa: E402
import test_gpu_parity as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
var = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
if len(sys.argv) > 3:  # first the c50k program at 1 M reads in the same process (as the test order)
    G.test_full_size_bundle_scan_equals_per_read_scan(("TTAGGG", None, int(sys.argv[3]), 50_000, 0.0))
    print("warm-up done")
cfg = os.environ.get("CFG", "c4")
nt = G._nt(patterns="TTAGGG TCAGGG", tvr_patterns="TGAGGG TTGGGG") if cfg == "c4" else G._nt(patterns="TTAGGG")
sp = synth_params(read_len=50_000, first_read=31, variant_rate=var)
t = G._device_batch(nt, sp, n, 50_000)
args = lambda: (t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(), t["win_off"].data_ptr(),
                n, n * t["rows"], 50_000, t["start"].data_ptr(), t["end"].data_ptr(), t["dens"].data_ptr(),
                t["flags"].data_ptr(), t["wc"].data_ptr())
nt.scan_call_device(*args())
nt.synchronize()
ref = {k: t[k].clone() for k in ("start", "end", "dens", "flags", "wc")}
for k in ref:
    t[k].zero_()
if os.environ.get("POISON_TP"):  # garbage in the T-layout buffer before the transposer
    _orig = torch.empty
    torch.empty = lambda *a, **k: _orig(*a, **k).fill_(-1) if k.get("device") == "cuda" else _orig(*a, **k)
b, keep = G._device_bundles(nt, t, n, 50_000)
if os.environ.get("POISON_TP"):
    torch.empty = _orig
nt.scan_call_device(*args(), bundles=b)
nt.synchronize()
np_ = nt.n_pass
bad = torch.zeros(n, dtype=torch.bool, device="cuda")
for k in ("start", "end", "dens"):
    bad |= (t[k] != ref[k]).reshape(n, 3).any(1)
bad |= t["flags"] != ref["flags"]
wcb = (G._valid_counts(t, n, np_) != G._valid_counts(t, n, np_, ref["wc"])).reshape(n, -1).any(1)
print("n_pass", np_, "reads differing in calls", int(bad.sum()), "in counts", int(wcb.sum()))
idx = torch.nonzero(bad | wcb).flatten().cpu().numpy()
for i in idx[:12]:
    i = int(i)
    print(i, "bundle", i // 32, "slot", i % 32,
          "start", t["start"][3 * i:3 * i + 3].tolist(), ref["start"][3 * i:3 * i + 3].tolist(),
          "end", t["end"][3 * i:3 * i + 3].tolist(), ref["end"][3 * i:3 * i + 3].tolist(),
          "flags", int(t["flags"][i]), int(ref["flags"][i]), "wcdiff", bool(wcb[i]))
    if wcb[i]:
        a = G._valid_counts(t, n, np_)[i].cpu().numpy().astype(int)
        r = G._valid_counts(t, n, np_, ref["wc"])[i].cpu().numpy().astype(int)
        for p in range(np_):
            d = np.nonzero(a[p] != r[p])[0]
            if len(d):
                print("   pass", p, "windows", d[:10].tolist(), "bundle", a[p][d[:5]].tolist(), "perread", r[p][d[:5]].tolist())
np.save("gpurun_out/fsdiff_idx.npy", idx)
