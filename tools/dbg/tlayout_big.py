"""Timing aid: the bench's bundle layout of 1M x 50 kb (one nt_bundle_layout launch)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))
from nanotel_amd import NanoTel, read_blocks, synth_params, window_count, window_rows  # noqa: E402
from nanotel_amd.api import DeviceBundles  # noqa: E402
n, rl, L = int(os.environ.get("NREADS", "1000000")), 50000, 100
nt = NanoTel(patterns="TTAGGG")
planes = torch.zeros(n * read_blocks(rl) * 2, dtype=torch.int32, device="cuda")
blk = torch.empty(n, dtype=torch.int64, device="cuda")
lens = torch.empty(n, dtype=torch.int32, device="cuda")
woff = torch.empty(n, dtype=torch.int64, device="cuda")
nt.synth_device(synth_params(read_len=rl), n, planes.data_ptr())
nt.uniform_layout_device(n, rl, blk.data_ptr(), lens.data_ptr(), woff.data_ptr())
plan = nt.bundle_plan(np.full(n, rl, np.uint32))
br = torch.from_numpy(plan.bnd_read.view(np.int32)).cuda()
bs = torch.from_numpy(plan.bnd_stripe.view(np.int64)).cuda()
tp = torch.empty(plan.tplane_bytes // 4, dtype=torch.int32, device="cuda")
b = DeviceBundles(tp.data_ptr(), br.data_ptr(), bs.data_ptr(), plan.n_bundles, 0, 0, plan.tplane_bytes)
for _ in range(2):
    nt.bundle_layout_device(planes.data_ptr(), blk.data_ptr(), lens.data_ptr(), woff.data_ptr(), n,
                            n * window_rows(window_count(rl, L)), b)
nt.synchronize()
print("ok")
