"""nt_rows_columns (include/nanotel.h): analyze_read's rows of a chunk as the
columns of the reference's data.frame (NanoTel.R:1820-1837, 1926-1974), in the
group-major row order of nt_assign_serials (NanoTel.R:2234-2258).  CPU only:
the per-read outputs come from the oracle (test stand-in for the kernels), the
rows from the C-ABI helper, formatted by the driver's summary writer."""
import csv
import math
import os
import random
import struct

import numpy as np
import pytest

import _oracle as O
from nanotel_amd import assign_serials
from nanotel_amd.api import NA_INT32, NA_REAL_BITS, rows_columns
from nanotel_amd.driver import chunk_rows, format_row

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _oracle_chunk(seqs, patterns, tvr=None, legacy=False):
    P = O.Patterns(patterns, tvr)
    n = len(seqs)
    res = {"start": np.full((n, 3), -1, np.int32), "end": np.full((n, 3), -1, np.int32),
           "density": np.zeros((n, 3)), "telomeric": np.zeros(n, bool)}
    for i, s in enumerate(seqs):
        r = O.analyze_read(s, P, legacy_no_ext=legacy)
        k = r["n_pass"]
        res["start"][i, :k] = r["start"]
        res["end"][i, :k] = r["end"]
        res["density"][i, :k] = r["density"]
        res["telomeric"][i] = r["telomeric"]
    return res


def _python_rows(res, names, lengths, serials, order, n_pass):
    """Restatement of analyze_read's add_row (NanoTel.R:1926-1974), the checker."""
    rows = []
    for j in order:
        j = int(j)
        row = [float(serials[j]), names[j], int(lengths[j])]
        for p in range(n_pass):
            s, e = int(res["start"][j, p]), int(res["end"][j, p])
            row += [None] * 4 if s == -1 else [float(res["density"][j, p]), s, e, e - s + 1]
        rows.append(row)
    return rows


def test_example_summary_csv_byte_for_byte():
    """Example/sample.fasta (legacy code version of Example_output): the rows built
    by the helper and formatted by the driver equal summary.csv's lines."""
    names, seqs = O.read_fasta(os.path.join(GOLD, "sample.fasta"))
    res = _oracle_chunk(seqs, "TTAGGG", legacy=True)
    lens = np.array([len(s) for s in seqs], np.uint64)
    ser, order, nxt, _ = assign_serials(res["telomeric"], 1.0)
    rows = chunk_rows(res, names, lens, ser, order, 2)
    lines = [format_row(r) for r in rows]
    with open(os.path.join(GOLD, "example_summary.csv"), newline="") as f:
        gold = f.read().splitlines()[1:]
    assert lines == gold
    assert nxt == 5.0


def _tvr_chunk(n, seed):
    rnd = random.Random(seed)
    seqs = []
    for i in range(n):
        bg = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(800, 4000)))
        kind = i % 4
        if kind == 0:
            s = "TTAGGG" * rnd.randint(20, 300) + bg          # P1/P2 tract
        elif kind == 1:
            s = "TGAGGG" * rnd.randint(40, 300) + bg          # TVR-only: P1/P2 NA, P3 row
        elif kind == 2:
            s = bg                                             # no row
        else:
            s = "TTAGGG" * 30 + "TTGGGG" * rnd.randint(20, 200) + bg
        seqs.append(s)
    return [f"read_{i} extra header words" for i in range(n)], seqs


@pytest.mark.parametrize("n,seed", [(5, 1), (43, 2)])
def test_tvr_chunk_rows_match_restatement(n, seed):
    """3 passes, < 8 reads (sequential) and >= 8 reads (8-way group order)."""
    names, seqs = _tvr_chunk(n, seed)
    res = _oracle_chunk(seqs, "TTAGGG", "TGAGGG TTGGGG")
    lens = np.array([len(s) for s in seqs], np.uint64)
    ser, order, _, _ = assign_serials(res["telomeric"], 17.0)
    got = [format_row(r) for r in chunk_rows(res, names, lens, ser, order, 3)]
    want = [format_row(r) for r in _python_rows(res, names, lens, ser, order, 3)]
    assert got == want
    assert len(got) > 0


def test_na_values_are_r_na():
    names, seqs = _tvr_chunk(12, 3)
    res = _oracle_chunk(seqs, "TTAGGG", "TGAGGG TTGGGG")
    lens = np.array([len(s) for s in seqs], np.uint64)
    ser, order, _, _ = assign_serials(res["telomeric"], 1.0)
    c = rows_columns(res, lens, ser, order, 3)
    assert c["na"].any(), "expected a TVR-only row (P1/P2 NA)"
    for p in range(3):
        for i in range(order.size):
            j = int(order[i])
            if res["start"][j, p] == -1:
                assert c["start"][p, i] == NA_INT32 and c["end"][p, i] == NA_INT32
                assert c["width"][p, i] == NA_INT32
                bits = struct.unpack("<Q", struct.pack("<d", c["density"][p, i]))[0]
                assert bits == NA_REAL_BITS and math.isnan(c["density"][p, i])
            else:
                assert c["width"][p, i] == res["end"][j, p] - res["start"][j, p] + 1
        assert np.array_equal(c["serial"], ser[order])
        assert np.array_equal(c["length"], lens[order].astype(np.int32))


def test_rows_columns_errors():
    res = {"start": np.full((2, 3), -1, np.int32), "end": np.full((2, 3), -1, np.int32),
           "density": np.zeros((2, 3))}
    from nanotel_amd import NanoTelError
    with pytest.raises(NanoTelError):
        rows_columns(res, np.array([10, 10], np.uint64), np.zeros(2), np.array([2], np.int64), 2)
    with pytest.raises(NanoTelError):
        rows_columns(res, np.array([1 << 31, 10], np.uint64), np.zeros(2), np.array([0], np.int64), 2)
    c = rows_columns(res, np.array([10, 10], np.uint64), np.zeros(2), np.zeros(0, np.int64), 2)
    assert c["serial"].size == 0


def _python_csv(c, names, n_pass, sci):
    from nanotel_amd.io import csv_field, format_double, format_int
    lines = []
    for i in range(c["serial"].size):
        f = [format_double(float(c["serial"][i]), sci), csv_field(names[i]), format_int(int(c["length"][i]))]
        for p in range(n_pass):
            if c["na"][p, i]:
                f += ["NA"] * 4
            else:
                f += [format_double(float(c["density"][p, i])), format_int(int(c["start"][p, i])),
                      format_int(int(c["end"][p, i])), format_int(int(c["width"][p, i]))]
        lines.append(",".join(f) + "\n")
    return "".join(lines).encode()


@pytest.mark.parametrize("sci", [None, 100000.0])
def test_rows_csv_matches_python_writer(sci):
    """nt_rows_csv (the C++ summary.csv writer) against the Python rules
    (io.format_double / csv_field) on edge values: NA passes, -Inf serials,
    large integral serials, tiny and integral densities, quoted names."""
    import ctypes
    from nanotel_amd.api import rows_csv
    rng = np.random.default_rng(3)
    n = 400
    dens = rng.random((n, 3))
    dens[::7] = np.round(dens[::7], 2)
    dens[::11] = 1.0
    dens[::13] = rng.random((len(dens[::13]), 3)) * 1e-5
    start = rng.integers(1, 50000, (n, 3)).astype(np.int32)
    start[::5, 1] = -1
    end = (start + rng.integers(0, 9000, (n, 3))).astype(np.int32)
    res = {"start": start, "end": end, "density": dens}
    lens = rng.integers(1, 2_000_000, n).astype(np.uint64)
    ser = rng.integers(1, 10 ** 7, n).astype(np.float64)
    ser[::9] = 1_000_000.0
    ser[::17] = float("-inf")
    order = rng.permutation(n)[:300].astype(np.int64)
    c = rows_columns(res, lens, ser, order, 3)
    names = [f"read_{j}" + (',"x"' if j % 4 == 0 else " runid=7") for j in order]
    bufs = [ctypes.create_string_buffer(s.encode(), len(s)) for s in names]
    ptrs = np.array([ctypes.addressof(b) for b in bufs], np.uint64)
    nls = np.array([len(s) for s in names], np.uint64)
    csv, ids = rows_csv(c, ptrs, nls, 3, sci)
    assert csv == _python_csv(c, names, 3, sci)
    assert ids == "".join(s + "\n" for s in names).encode()
    for x in (1e-05, 0.0001, 12345.678, 1e16 + 2, 0.5, 2.0 / 3):
        c1 = {k: v[..., :1].copy() for k, v in c.items()}
        c1["density"][0, 0] = x
        assert rows_csv(c1, ptrs[:1], nls[:1], 3, sci)[0] == _python_csv(c1, names[:1], 3, sci), x
