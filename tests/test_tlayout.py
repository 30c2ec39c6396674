"""The host T-layout builder (nt_bundle_layout_host: the bundle scan's copy of
the reads, built at ingest) against a numpy restatement of the layout's
definition in nt_common.h.  CPU only (the GPU test compares it with the device
builder, tests/test_gpu_parity.py::test_host_tlayout_matches_device)."""
import ctypes

import numpy as np
import pytest

from nanotel_amd import _lib
from nanotel_amd.api import BundlePlan, bundle_layout_host


def pack(seqs, L=100):
    """nt_pack_reads of ASCII reads -> (planes, blk_off, len)."""
    lib = _lib.lib()
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(s) for s in seqs], np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    assert lib.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, L, ctypes.byref(tb),
                             ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml), ctypes.byref(bad)) == 0
    planes = np.full(2 * tb.value + 2, 0xA5A5A5A5, np.uint32)  # garbage past the reads: must be masked
    blk = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    wo = np.zeros(n, np.uint64)
    assert lib.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 0, L, planes.ctypes.data,
                             blk.ctypes.data, ln.ctypes.data, wo.ctypes.data, None, None, None) == 0
    # bits past each read's end inside its last block: garbage too
    for r in range(n):
        m = int(ln[r])
        if m % 32:
            w = 2 * (int(blk[r]) + m // 32)
            planes[w] |= np.uint32(0xFFFFFFFF << (m % 32) & 0xFFFFFFFF)
            planes[w + 1] |= np.uint32(0xFFFFFFFF << (m % 32) & 0xFFFFFFFF)
    return planes, blk, ln


def plan_of(lengths, L):
    """nt_bundle_plan's grouping (restated): longest first, ties in input
    order, 32 to a bundle; a bundle spans ceil(ceil(n_max / L) / 64) stripes."""
    order = sorted(range(len(lengths)), key=lambda r: -int(lengths[r]))
    nb = (len(order) + 31) // 32
    bread = np.full(nb * 32, 0xFFFFFFFF, np.uint32)
    bread[:len(order)] = order
    bstripe = np.zeros(nb + 1, np.uint64)
    g = 0
    for b in range(nb):
        bstripe[b] = g
        nmax = int(lengths[order[32 * b]])
        g += ((nmax + L - 1) // L + 63) // 64
    bstripe[nb] = g
    return BundlePlan(bread, bstripe, np.zeros(0, np.uint32), g * ((L + 1) // 2) * 64 * 16)


def tlayout_numpy(planes, blk, ln, plan, L):
    T = (L + 1) // 2
    out = np.zeros(plan.tplane_bytes // 4, np.uint32)
    for b in range(plan.n_bundles):
        for s in range(32):
            r = int(plan.bnd_read[32 * b + s])
            if r == 0xFFFFFFFF:
                continue
            m = int(ln[r])
            p = np.arange(m, dtype=np.int64)
            w = planes[2 * (int(blk[r]) + p // 32)]
            x = planes[2 * (int(blk[r]) + p // 32) + 1]
            lo = (w >> (p % 32).astype(np.uint32)) & 1
            hi = (x >> (p % 32).astype(np.uint32)) & 1
            k, o = p // L, p % L
            idx = ((int(plan.bnd_stripe[b]) + k // 64) * T + o // 2) * 64 + k % 64
            d = 4 * idx + 2 * (o % 2)
            np.bitwise_or.at(out, d, (lo << s).astype(np.uint32))
            np.bitwise_or.at(out, d + 1, (hi << s).astype(np.uint32))
    return out


@pytest.mark.parametrize("L", [100, 37, 50, 170])
def test_host_tlayout_matches_definition(L):
    rng = np.random.default_rng(L)
    alpha = np.frombuffer(b"ACGT", np.uint8)
    lens = [int(rng.integers(1, 9000)) for _ in range(70)] + [6400 * 2, 64 * L, 64 * L + 1, 31, 32, 33]
    seqs = [alpha[rng.integers(0, 4, n)].tobytes() for n in lens]
    planes, blk, ln = pack(seqs, L)
    plan = plan_of(ln, L)
    got = bundle_layout_host(planes, blk, ln, plan, L)
    want = tlayout_numpy(planes, blk, ln, plan, L)
    assert got.shape == want.shape
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])


def test_host_tlayout_argument_checks():
    planes, blk, ln = pack([b"ACGT" * 100], 100)
    plan = plan_of(ln, 100)
    small = BundlePlan(plan.bnd_read, plan.bnd_stripe, plan.list, plan.tplane_bytes - 16)
    with pytest.raises(Exception):
        bundle_layout_host(planes, blk, ln, small, 100)
    with pytest.raises(Exception):
        bundle_layout_host(planes, blk, ln, plan, 171)
