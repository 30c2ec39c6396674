"""CPU-side checks of the C-ABI library: it loads, exports every symbol that
include/nanotel.h declares, and its host-only entry points (no GPU needed)
behave like the reference (window split, serial assignment, packing)."""
import math
import os
import re
import subprocess

import numpy as np
import pytest

import _oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nanotel.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nt_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from nanotel_amd import _lib
    L = _lib.lib()
    decl = declared_functions()
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(L, name), name
    assert set(decl) == set(_lib.SIGNATURES), set(decl) ^ set(_lib.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in decl:
        assert re.search(rf"\bT {name}\b", out), name


def test_library_has_gfx950_code_object():
    from nanotel_amd import _lib
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_window_count_matches_oracle():
    from nanotel_amd import window_count
    for n in list(range(1, 400)) + [2981, 20410, 59430, 15880, 10 ** 6]:
        for L in (1, 2, 7, 37, 100, 150):
            assert window_count(n, L) == O.window_count(n, L), (n, L)


def test_window_rows_padding():
    # count rows padded to whole 128-byte lines (64 windows), C and numpy agree
    from nanotel_amd import window_rows
    nws = np.array([0, 1, 2, 63, 64, 65, 127, 128, 500, 501, 10 ** 6], np.int64)
    got = window_rows(nws)
    assert list(got) == [0, 64, 64, 64, 64, 128, 128, 128, 512, 512, 1000000]
    assert all(window_rows(int(x)) == int(y) for x, y in zip(nws, got))


def test_pack_reads_window_offsets_are_padded_rows():
    import ctypes
    from nanotel_amd import _lib, window_count, window_rows
    L = _lib.lib()
    seqs = [b"A" * 6450, b"C" * 99, b"G" * 150, b"T" * 12800]
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(s) for s in seqs], np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    assert L.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 100, ctypes.byref(tb),
                           ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml), ctypes.byref(bad)) == 0
    rows = [window_rows(window_count(len(x), 100)) for x in seqs]
    assert tw.value == sum(rows)
    planes = np.zeros(2 * tb.value, np.uint32)
    blk, wo = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    assert L.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 0, 100, planes.ctypes.data,
                           blk.ctypes.data, ln.ctypes.data, wo.ctypes.data, None, None, None) == 0
    assert list(wo) == [0, rows[0], rows[0] + rows[1], rows[0] + rows[1] + rows[2]]
    assert all(int(w) % 64 == 0 for w in wo)


@pytest.mark.parametrize("seed", range(6))
def test_assign_serials_matches_oracle(seed):
    from nanotel_amd import assign_serials
    rng = np.random.default_rng(seed)
    ss_c, mx_c = 1.0, -math.inf
    ss_o, mx_o = 1.0, -math.inf
    for chunk in range(5):
        n = int(rng.choice([0, 3, 7, 8, 9, 57, 1000]))
        p = [0.0, 0.3, 1.0][int(rng.integers(0, 3))] if chunk else 0.0 if seed % 2 else 0.5
        t = (rng.random(n) < p).astype(np.uint8)
        s_c, o_c, ss_c, mx_c = assign_serials(t, ss_c, mx_c)
        s_o, o_o, ss_o, mx_o = O.assign_serials(list(t), ss_o, mx_o)
        assert list(o_c) == o_o
        assert [x for x in s_c if not math.isnan(x)] == [x for x in s_o if not math.isnan(x)]
        assert (ss_c == ss_o) or (math.isinf(ss_c) and math.isinf(ss_o))
        assert (mx_c == mx_o) or (math.isinf(mx_c) and math.isinf(mx_o))


def test_serials_reference_semantics():
    from nanotel_amd import assign_serials
    # < 8 reads: sequential; non-telomeric reads consume no serial
    s, o, ss, mx = assign_serials([1, 0, 1])
    assert list(o) == [0, 2] and s[0] == 1 and s[2] == 2 and ss == 3
    # >= 8 reads: round-robin groups, group g starts at serial_start + |groups < g|
    s, o, ss, mx = assign_serials([1] * 10)
    assert list(o) == [0, 8, 1, 9, 2, 3, 4, 5, 6, 7]
    assert [s[i] for i in o] == [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]
    s, o, ss, mx = assign_serials([0, 1, 0, 0, 0, 0, 0, 0, 0, 1])
    assert list(o) == [1, 9] and s[1] == 3 and s[9] == 4 and ss == 5
    # no row in the first chunk: max(numeric(0)) + 1 = -Inf forever
    s, o, ss, mx = assign_serials([0] * 9)
    assert ss == -math.inf
    s, o, ss, mx = assign_serials([1, 1], ss, mx)
    assert s[0] == -math.inf and ss == -math.inf


def test_pack_reads_layout_and_rc():
    import ctypes
    from nanotel_amd import _lib
    L = _lib.lib()
    seqs = [b"ACGTN" * 13, b"ttaggg", b"RYACGTACGTACGTACGTACGTACGTACGTACGTA"]
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(s) for s in seqs], np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    rc = L.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 100,
                         ctypes.byref(tb), ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml),
                         ctypes.byref(bad))
    assert rc == 0 and tb.value == 4 + 2 + 2 and te.value == 13 + 2 and ml.value == 65
    for rcflag in (0, 1):
        planes = np.zeros(2 * tb.value, np.uint32)
        blk = np.zeros(n, np.uint64)
        ln = np.zeros(n, np.uint32)
        wo = np.zeros(n, np.uint64)
        eo = np.zeros(n + 1, np.uint32)
        ep = np.zeros(te.value, np.uint32)
        ec = np.zeros(te.value, np.uint8)
        rc = L.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, rcflag, 100,
                             planes.ctypes.data, blk.ctypes.data, ln.ctypes.data, wo.ctypes.data,
                             eo.ctypes.data, ep.ctypes.data, ec.ctypes.data)
        assert rc == 0
        codes = {1: "A", 2: "C", 4: "G", 8: "T", 15: "N", 5: "R", 10: "Y"}
        for r, s in enumerate(seqs):
            ref = s.decode().upper()
            if rcflag:
                ref = O.reverse_complement(ref)
            b0 = int(blk[r])
            assert b0 % 2 == 0
            out = []
            exc = {int(ep[i]): int(ec[i]) for i in range(eo[r], eo[r + 1])}
            for pos in range(len(s)):
                w = planes[2 * (b0 + pos // 32):2 * (b0 + pos // 32) + 2]
                c = int((w[0] >> (pos % 32)) & 1) | (int((w[1] >> (pos % 32)) & 1) << 1)
                out.append(codes[exc[pos]] if pos in exc else "ACGT"[c])
            assert "".join(out) == ref, (r, rcflag)


@pytest.mark.parametrize("rcflag", [0, 1])
def test_pack_reads_whole_blocks_random(rcflag):
    """The 32-bases-at-a-time packer (whole blocks of plain bases) against a
    numpy decode: mixed case, ragged lengths, a few IUPAC letters so that
    some blocks take the per-base path next to fast ones."""
    import ctypes
    from nanotel_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(7 + rcflag)
    alpha = np.frombuffer(b"ACGTacgt", np.uint8)
    seqs = []
    for r in range(40):
        n = int(rng.integers(1, 3000))
        s = alpha[rng.integers(0, 8, n)].copy()
        if r % 3 == 0:
            k = int(rng.integers(1, 4))
            s[rng.integers(0, n, k)] = np.frombuffer(b"N", np.uint8)[0]
        seqs.append(s.tobytes())
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(s) for s in seqs], np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    assert L.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 100,
                           ctypes.byref(tb), ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml),
                           ctypes.byref(bad)) == 0
    assert te.value == sum(s.upper().count(b"N") for s in seqs)
    planes = np.full(2 * tb.value, 0xDEADBEEF, np.uint32)
    blk = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint32)
    wo = np.zeros(n, np.uint64)
    eo = np.zeros(n + 1, np.uint32)
    ep = np.zeros(max(1, te.value), np.uint32)
    ec = np.zeros(max(1, te.value), np.uint8)
    assert L.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, rcflag, 100,
                           planes.ctypes.data, blk.ctypes.data, ln.ctypes.data, wo.ctypes.data,
                           eo.ctypes.data, ep.ctypes.data, ec.ctypes.data) == 0
    lut = np.full(256, 255, np.uint8)
    for i, ch in enumerate(b"ACGT"):
        lut[ch] = i
        lut[ch + 32] = i
    for r, s in enumerate(seqs):
        a = np.frombuffer(s, np.uint8)
        code = lut[a]
        if rcflag:
            code = code[::-1]
            code = np.where(code == 255, 255, 3 - code)
        m = len(s)
        nblk = (m + 31) // 32
        w = planes[2 * int(blk[r]):2 * (int(blk[r]) + nblk)].reshape(nblk, 2)
        bits = np.arange(32, dtype=np.uint32)
        lo = ((w[:, 0:1] >> bits) & 1).reshape(-1)[:m]
        hi = ((w[:, 1:2] >> bits) & 1).reshape(-1)[:m]
        got = (lo | (hi << 1)).astype(np.uint8)
        exc = code == 255
        assert np.array_equal(got[~exc], code[~exc]), r
        assert np.all(got[exc] == 0), r  # planes hold A at exception positions
        pos = ep[eo[r]:eo[r + 1]]
        assert np.array_equal(np.sort(pos), np.flatnonzero(exc)), r
        if nblk < 2 * ((m + 63) // 64):  # pad block of the 64-base segment is zeroed
            assert planes[2 * (int(blk[r]) + nblk)] == 0 and planes[2 * (int(blk[r]) + nblk) + 1] == 0
