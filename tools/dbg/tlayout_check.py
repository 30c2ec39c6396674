"""Debug aid: check every word of the device T-layout (nt_bundle_layout)
against the reads (zeros past them): python tools/dbg/tlayout_check.py [read_len]."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))
from nanotel_amd import NanoTel, read_blocks, synth_params, synth_read_ascii, window_count, window_rows  # noqa: E402
from nanotel_amd.api import DeviceBundles  # noqa: E402

rl = int(sys.argv[1]) if len(sys.argv) > 1 else 13001
n, L = 80, 100
nt = NanoTel(patterns="TTAGGG")
sp = synth_params(read_len=rl, first_read=5)
nblk = read_blocks(rl)
rows = window_rows(window_count(rl, L))
planes = torch.zeros(n * nblk * 2, dtype=torch.int32, device="cuda")
blk = torch.empty(n, dtype=torch.int64, device="cuda")
lens = torch.empty(n, dtype=torch.int32, device="cuda")
woff = torch.empty(n, dtype=torch.int64, device="cuda")
nt.synth_device(sp, n, planes.data_ptr())
nt.uniform_layout_device(n, rl, blk.data_ptr(), lens.data_ptr(), woff.data_ptr())
plan = nt.bundle_plan(np.full(n, rl, np.uint32))
br = torch.from_numpy(plan.bnd_read.view(np.int32)).cuda()
bs = torch.from_numpy(plan.bnd_stripe.view(np.int64)).cuda()
tp = torch.full((plan.tplane_bytes // 4,), -1, dtype=torch.int32, device="cuda")  # poison: every word must be written
b = DeviceBundles(tp.data_ptr(), br.data_ptr(), bs.data_ptr(), plan.n_bundles, 0, 0, plan.tplane_bytes)
nt.bundle_layout_device(planes.data_ptr(), blk.data_ptr(), lens.data_ptr(), woff.data_ptr(), n, n * rows, b)
nt.synchronize()
T = (L + 1) // 2
w = tp.cpu().numpy().view(np.uint32).reshape(-1, T, 64, 4)  # [stripe][t][block][lo0, hi0, lo1, hi1]
codes = np.zeros((n, 0), np.uint8)
npos = (plan.bnd_stripe[1] - plan.bnd_stripe[0]) * 64 * L
codes = np.zeros((n, int(npos)), np.uint8)
lut = np.zeros(256, np.uint8)
for i, c in enumerate(b"ACGT"):
    lut[c] = i
for i in range(n):
    codes[i, :rl] = lut[np.frombuffer(synth_read_ascii(sp, i).encode(), np.uint8)]
bad = 0
for bi in range(plan.n_bundles):
    g0, g1 = int(plan.bnd_stripe[bi]), int(plan.bnd_stripe[bi + 1])
    slots = [int(x) for x in plan.bnd_read[bi * 32:(bi + 1) * 32]]
    for g in range(g0, g1):
        for par in (0, 1):
            q = ((g - g0) * 64 + np.arange(64)[None, :]) * L + 2 * np.arange(T)[:, None] + par  # [t][block]
            ok = (2 * np.arange(T)[:, None] + par) < L
            lo = np.zeros((T, 64), np.uint64)
            hi = np.zeros((T, 64), np.uint64)
            for s, r in enumerate(slots):
                if r == 0xFFFFFFFF:
                    continue
                c = np.where(ok & (q < codes.shape[1]), codes[r][np.minimum(q, codes.shape[1] - 1)], 0)
                lo |= (c & 1).astype(np.uint64) << np.uint64(s)
                hi |= (c >> 1).astype(np.uint64) << np.uint64(s)
            got_lo, got_hi = w[g, :, :, 2 * par], w[g, :, :, 2 * par + 1]
            m = ok
            d = (m & (got_lo != lo)) | (m & (got_hi != hi))
            bad += int(d.sum())
            if d.any() and bad < 20:
                t, k = np.argwhere(d)[0]
                print("bundle", bi, "stripe", g, "t", t, "block", k, "par", par, hex(int(lo[t, k])), hex(int(got_lo[t, k])))
print("bundles", plan.n_bundles, "stripes", int(plan.bnd_stripe[-1]), "bad", bad)
