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
    order, 32 to a bundle; a bundle spans ceil(ceil(n_max / L) / 64) stripes,
    its first block column = 64 x its first stripe."""
    order = sorted(range(len(lengths)), key=lambda r: -int(lengths[r]))
    nb = (len(order) + 31) // 32
    bread = np.full(nb * 32, 0xFFFFFFFF, np.uint32)
    bread[:len(order)] = order
    bblock = np.zeros(nb + 1, np.uint64)
    col = 0
    for b in range(nb):
        bblock[b] = col
        col += -(-((int(lengths[order[32 * b]]) + L - 1) // L) // 64) * 64
    bblock[nb] = col
    return BundlePlan(bread, bblock, np.zeros(0, np.uint32), col // 64 * ((L + 1) // 2) * 64 * 16)


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
            c = int(plan.bnd_block[b]) + k  # the block's column
            idx = ((c // 64) * T + o // 2) * 64 + c % 64
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
    check_layout(planes, blk, ln, plan, L)


def check_layout(planes, blk, ln, plan, L):
    got = bundle_layout_host(planes, blk, ln, plan, L)
    want = tlayout_numpy(planes, blk, ln, plan, L)
    assert got.shape == want.shape
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:8], got[bad[:8]], want[bad[:8]])


def test_host_tlayout_argument_checks():
    planes, blk, ln = pack([b"ACGT" * 100], 100)
    plan = plan_of(ln, 100)
    small = BundlePlan(plan.bnd_read, plan.bnd_block, plan.list, plan.tplane_bytes - 16)
    with pytest.raises(Exception):
        bundle_layout_host(planes, blk, ln, small, 100)
    with pytest.raises(Exception):
        bundle_layout_host(planes, blk, ln, plan, 171)
    off = BundlePlan(plan.bnd_read, plan.bnd_block + np.uint64(16), plan.list, plan.tplane_bytes * 2)
    with pytest.raises(Exception):  # a bundle that does not start on a stripe
        bundle_layout_host(planes, blk, ln, off, 100)
