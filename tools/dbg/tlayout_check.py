"""Debug aid: check the device T-layout (nt_bundle_layout) against the reads."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))
from nanotel_amd import NanoTel, read_blocks, synth_params, synth_read_ascii, window_count
from nanotel_amd.api import DeviceBundles

n, rl, L = 64, 3001, 100
nt = NanoTel(patterns="TTAGGG")
sp = synth_params(read_len=rl, first_read=5)
nblk = read_blocks(rl)
nw = window_count(rl, L)
planes = torch.zeros(n * nblk * 2, dtype=torch.int32, device="cuda")
blk = torch.empty(n, dtype=torch.int64, device="cuda")
lens = torch.empty(n, dtype=torch.int32, device="cuda")
woff = torch.empty(n, dtype=torch.int64, device="cuda")
nt.synth_device(sp, n, planes.data_ptr())
nt.uniform_layout_device(n, rl, blk.data_ptr(), lens.data_ptr(), woff.data_ptr())
plan = nt.bundle_plan(np.full(n, rl, np.uint32))
br = torch.from_numpy(plan.bnd_read.view(np.int32)).cuda()
bs = torch.from_numpy(plan.bnd_stripe.view(np.int64)).cuda()
tp = torch.empty(plan.tplane_bytes // 4, dtype=torch.int32, device="cuda")
b = DeviceBundles(tp.data_ptr(), br.data_ptr(), bs.data_ptr(), plan.n_bundles, 0, 0, plan.tplane_bytes)
nt.bundle_layout_device(planes.data_ptr(), blk.data_ptr(), lens.data_ptr(), woff.data_ptr(), n, n * nw, b)
nt.synchronize()
T = (L + 1) // 2
w = tp.cpu().numpy().view(np.uint32).reshape(-1, 4)
print("bundles", plan.n_bundles, "stripes", plan.bnd_stripe.tolist(), "read table", plan.bnd_read[:8].tolist())
reads = [synth_read_ascii(sp, i) for i in range(n)]
bad = 0
for bi in range(plan.n_bundles):
    g0 = int(plan.bnd_stripe[bi])
    for q in list(range(0, 300)) + list(range(rl - 50, rl + 20)):
        k, o = divmod(q, L)
        word = (g0 + k // 64) * T * 64 + (o // 2) * 64 + (k % 64)
        lo, hi = w[word][2 * (o & 1)], w[word][2 * (o & 1) + 1]
        for s in range(32):
            r = int(plan.bnd_read[bi * 32 + s])
            c = "ACGT".index(reads[r][q]) if q < rl else 0
            got = ((int(lo) >> s) & 1) | (((int(hi) >> s) & 1) << 1)
            if got != c:
                bad += 1
                if bad < 10:
                    print("bundle", bi, "q", q, "slot", s, "read", r, "want", c, "got", got)
print("bad", bad)
