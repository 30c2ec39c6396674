"""Parity of the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact on every output: called start/end per pass, fp64 densities,
telomeric flag, per-window covered counts, per-pattern hit counts.
"""
import os
import zlib

import numpy as np
import pytest

import _oracle as O
from _parity import compare, oracle_rows

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(autouse=True)
def _torch_stream():
    """The tests' torch work on a stream of their own (not the null stream,
    which a context stream created non-blocking does not wait for); _nt()
    puts each context on it, so fills, copies and clears are ordered with
    the kernels."""
    import torch
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        yield
    s.synchronize()


def _nt(jit=True, **kw):
    """NanoTel context; jit=False forces the ahead-of-time scan kernels."""
    from nanotel_amd import NanoTel
    old = os.environ.get("NT_JIT")
    os.environ["NT_JIT"] = "1" if jit else "0"
    try:
        nt = NanoTel(**kw)
    finally:
        if old is None:
            del os.environ["NT_JIT"]
        else:
            os.environ["NT_JIT"] = old
    assert nt.jit == jit, "hiprtc specialisation unavailable"
    # the context works on the tests' torch stream (_torch_stream): torch
    # fills, copies and clears of device buffers are ordered with its kernels
    # (on a stream of its own, a zeros() still in flight could land on the
    # scan's counts)
    import torch
    h = torch.cuda.current_stream().cuda_stream
    assert h, "the null stream: the context would keep its own"
    nt.set_stream(h)
    return nt


def _check_both(nt, seqs, orow, **kw):
    """The per-read scan (hit counters asked for: a parity output only it
    produces) and, for a program the bundle scan covers, the bundle scan (no
    hit counters: the reads transposed 32 to a bundle), both against the oracle."""
    res = nt.analyze(seqs, want_windows=True, want_hits=True)
    compare(nt, res, orow, **kw)
    res2 = nt.analyze(seqs, want_windows=True, want_hits=False)
    compare(nt, res2, orow, check_hits=False, **kw)
    return res, res2


def _example():
    return O.read_fasta(os.path.join(GOLD, "sample.fasta"))


def _telo_read(rng, n, motif="TTAGGG", where="left", tract=(200, 3000), sub=0.03, exc=0.0,
               exc_letters="NRYKMSWBDHV", lower=0.0):
    bases = np.array(list("ACGT"))
    s = list(bases[rng.integers(0, 4, n)])
    tl = int(rng.integers(tract[0], tract[1] + 1)) if n > 0 else 0
    tl = min(tl, n)
    if where == "left":
        a = 0
    elif where == "right":
        a = n - tl
    else:
        a = int(rng.integers(0, max(1, n - tl)))
    for i in range(tl):
        s[a + i] = motif[i % len(motif)]
        if rng.random() < sub:
            s[a + i] = bases[rng.integers(0, 4)]
    if exc > 0:
        for i in range(n):
            if rng.random() < exc:
                s[i] = exc_letters[rng.integers(0, len(exc_letters))]
    if lower > 0:
        for i in range(n):
            if rng.random() < lower:
                s[i] = s[i].lower()
    return "".join(s)


def test_example_golden_through_hip():
    names, seqs = _example()
    for legacy in (True, False):
        nt = _nt(patterns="TTAGGG", min_density=0.6, legacy_no_ext=legacy)
        assert nt.tscan
        _check_both(nt, seqs, oracle_rows(seqs, "TTAGGG", legacy=legacy))
        nt.close()
    # the committed golden itself (legacy) through the HIP path
    import csv
    rows = list(csv.DictReader(open(os.path.join(GOLD, "example_summary.csv"))))
    nt = _nt(patterns="TTAGGG", legacy_no_ext=True)
    res = nt.analyze(seqs)
    for i, g in enumerate(rows):
        assert int(res["start"][i][0]) == int(g["Telomere_start"])
        assert int(res["end"][i][1]) == int(g["Telomere_end_mismatch"])
        assert repr(float(res["density"][i][0])) == g["telo_density"]
        assert repr(float(res["density"][i][1])) == g["telo_density_mismatch"]


def test_synthetic_generator_reads():
    from nanotel_amd import synth_params, synth_read_ascii
    for read_len, rc_layout, var in ((10000, False, 0.0), (50000, True, 0.05)):
        sp = synth_params(read_len=read_len, rc_layout=rc_layout, variant_rate=var)
        seqs = [synth_read_ascii(sp, i) for i in range(24)]
        nt = _nt(patterns="TTAGGG", rc=rc_layout)
        res, _ = _check_both(nt, seqs, oracle_rows(seqs, "TTAGGG", rc=rc_layout))
        assert res["telomeric"].sum() > 0


@pytest.mark.parametrize("cfg", [
    dict(read_len=10000, patterns="TTAGGG", tvr=None, rc=False, variant=0.0),  # BASELINE configs[1]
    dict(read_len=50000, patterns="YYAGGG", tvr=None, rc=True, variant=0.05),  # configs[2] (--rc)
    dict(read_len=50000, patterns="TTAGGG TCAGGG", tvr="TGAGGG TTGGGG", rc=False, variant=0.05),  # configs[3]
], ids=["c10k", "c3", "c4"])
def test_baseline_config_reads(cfg):
    # the bench's synthetic reads of each BASELINE configuration (a sample of
    # 64), through the host path and the hiprtc scan, against the oracle
    from nanotel_amd import synth_params, synth_read_ascii
    sp = synth_params(read_len=cfg["read_len"], rc_layout=cfg["rc"], variant_rate=cfg["variant"], first_read=4242)
    seqs = [synth_read_ascii(sp, i) for i in range(64)]
    nt = _nt(patterns=cfg["patterns"], tvr_patterns=cfg["tvr"], rc=cfg["rc"])
    assert nt.tscan
    res, _ = _check_both(nt, seqs, oracle_rows(seqs, cfg["patterns"], tvr=cfg["tvr"], rc=cfg["rc"]))
    assert 0 < res["telomeric"].sum() < 64


@pytest.mark.parametrize("cfg", [
    dict(patterns="TTAGGG"),
    dict(patterns="YYAGGG"),
    dict(patterns="TTAGGG TCAGGG"),
    dict(patterns="TTAGGG TTAGGG"),
    dict(patterns="CCCTAA", check_right_edge=True),
    dict(patterns="TTAGGG TCAGGG", tvr_patterns="TGAGGG TTGGGG"),
    dict(patterns="TTAGGG", tvr_patterns="TTGGGG"),
    dict(patterns="TTAGGG", subseq_length=50, min_density=0.5),
    dict(patterns="TTAGGG", subseq_length=37, min_density=0.3),
    dict(patterns="TTAGGG", rc=True),
    dict(patterns="ttaggg"),
    dict(patterns="TTAGGN"),
    dict(patterns="TTRGGG CCCTAA", tvr_patterns="TYAGGG"),
    dict(patterns="TAGGGTTAGGGTTAGGGT"),
])
@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_random_reads(cfg, jit):
    _random_reads(cfg, jit)


# the calling kernel specialised for the patterns (nt_call.h through hiprtc,
# ~8-25 s to build per pattern set, so a representative subset): forced with
# NT_CALL_JIT=1 for these small batches (by default it serves batches of
# >= 65,536 reads, where the full-size tests and the bench exercise it)
@pytest.mark.parametrize("cfg", [
    dict(patterns="TTAGGG"),
    dict(patterns="YYAGGG"),
    dict(patterns="CCCTAA", check_right_edge=True),
    dict(patterns="TTAGGG TCAGGG", tvr_patterns="TGAGGG TTGGGG"),
    dict(patterns="TTAGGG", subseq_length=37, min_density=0.3),
    dict(patterns="TTAGGN"),
    dict(patterns="TTRGGG CCCTAA", tvr_patterns="TYAGGG"),
    dict(patterns="TAGGGTTAGGGTTAGGGT"),
])
def test_random_reads_specialised_call(cfg, monkeypatch):
    monkeypatch.setenv("NT_CALL_JIT", "1")
    nt = _random_reads(cfg, True)
    assert nt.call_jit(), "the specialised calling kernel did not run"


# more than 8 patterns per list (the reference takes any number: NanoTel.R:2322-2334)
MANY = [
    dict(patterns="TTAGGG TCAGGG TGAGGG TTGGGG CTAGGG TTAGGC GGGTTA TTTAGG TTAGGA", tvr_patterns="TTCGGG"),
    dict(patterns="TTAGGG TCAGGG YYAGGG TTAGG TTAGGGTTAGGG CCCTAA CCCTRA TTAGGN GGGTTAG TTGGG AAAAAAAAAA TAGGG",
         tvr_patterns="TTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTT TGAGGG"),
]


@pytest.mark.parametrize("cfg", MANY, ids=["9_equal_len", "12_mixed_32_letter_tvr"])
@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_many_patterns(cfg, jit):
    nt = _random_reads(cfg, jit, check_tscan=False)
    if jit:
        assert nt.tscan == (cfg is MANY[0])  # equal-length lists take the bundle scan


# mixed-length lists through the bundle scan (one walk group per distinct
# length, nt_tscan.h TPipeMixed)
MIXED = [
    dict(patterns="TTAGGG TTAGG"),
    dict(patterns="TTAGGG TTAGG CCCTAAA", tvr_patterns="TGAGGG TTGGG"),
    dict(patterns="TTAGGG TTAGGGTTAGGG TTAGG", subseq_length=50, min_density=0.5),
    dict(patterns="TTAGGG TTRGG", tvr_patterns="TTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTT TGAGG"),
]


@pytest.mark.parametrize("cfg", MIXED, ids=["6_5", "6_5_7_tvr_6_5", "6_12_5_L50", "6_5_tvr_32_5"])
def test_mixed_length_lists_bundle_scan(cfg):
    nt = _random_reads(cfg, True, check_tscan=False)
    assert nt.tscan, "mixed-length list not on the bundle scan"


# Pattern lists whose patterns differ in one letter: the bundle scan walks them
# merged (TTAGGG + TCAGGG -> TYAGGG, nt_jit.cpp merged_types; the union of the
# <= 1-mismatch matches is the merged pattern's); the per-read scan keeps them
# apart (its hit counters); both against the oracle on the unmerged list.
MERGED = [
    dict(patterns="TTAGGG TCAGGG TAAGGG"),                      # three merge into one
    dict(patterns="TTAGGG TTAGGC TCAGGG", tvr_patterns="TGAGGG TTAGGA"),  # chains and a TVR pair
    dict(patterns="TTAGGG TTRGGG"),                             # an IUPAC letter in the union
]


@pytest.mark.parametrize("cfg", MERGED, ids=["three", "chain_tvr", "iupac"])
def test_merged_pattern_lists_bundle_scan(cfg):
    nt = _random_reads(cfg, True, check_tscan=False)
    assert nt.tscan


# Reads with a few non-ACGT letters through the bundle scan (VERDICT r3 item
# 6): the planes hold A at the letters; the calling kernel recounts every
# window within (longest pattern - 1) of one (call_fix_windows, nt_call.h).
EXC_WINDOWS = 16  # NT_EXC_WINDOWS (nt_common.h)


def _exc_windows(pos, n, L, mm):
    """exc_windows (nt_common.h) restated: the windows before the last that
    hold a position within mm - 1 of an exception."""
    from nanotel_amd import window_count
    nw = window_count(n, L)
    out = set()
    for p in pos:
        a, b = max(p - (mm - 1), 0), min(p + mm - 1, n - 1)
        out.update(w for w in range(a // L, min(b // L, nw - 2) + 1))
    return sorted(out)


def _sparse_exception_reads(seed, L=100):
    rng = np.random.default_rng(seed)
    letters = "NNNNRY-"
    seqs = []
    for i in range(640):
        n = int(rng.choice([int(rng.integers(150, 1200)), int(rng.integers(1200, 9000)),
                            int(rng.integers(9000, 30000))]))
        s = list(_telo_read(rng, n, where=["left", "right", "mid"][i % 3], tract=(100, min(n, 4000))))
        kind = i % 8
        if kind == 1:  # one letter anywhere
            pos = [int(rng.integers(0, n))]
        elif kind == 2:  # at the read's ends and around window boundaries
            k = int(rng.integers(1, max(2, n // L)))
            pos = [0, n - 1, min(n - 1, k * L - 1), min(n - 1, k * L), min(n - 1, k * L + 5)]
        elif kind == 3:  # a run inside the tract area
            a = int(rng.integers(0, max(1, min(n, 4000) - 40)))
            pos = list(range(a, min(n, a + int(rng.integers(5, 40)))))
        elif kind == 4:  # a few scattered letters
            pos = sorted(int(x) for x in rng.integers(0, n, int(rng.integers(2, 6))))
        elif kind == 5:  # spread over more than NT_EXC_WINDOWS windows: the per-read scan
            pos = list(range(int(rng.integers(0, 50)), n, 2 * L + 7))
        elif kind == 6:  # inside the last window only
            pos = [n - 1 - int(rng.integers(0, min(n, 60)))]
        else:
            pos = []
        for p in pos:
            s[p] = letters[int(rng.integers(0, len(letters)))]
        seqs.append("".join(s))
    return seqs


@pytest.mark.parametrize("cfg", [
    dict(patterns="TTAGGG"),
    dict(patterns="YYAGGG"),
    dict(patterns="TTAGGN"),
    dict(patterns="TTAGGG TCAGGG", tvr_patterns="TGAGGG TTGGGG"),
    dict(patterns="TTAGGG TTAGG", tvr_patterns="TTAGGGTTAGGGTTAGGG"),
    dict(patterns="TTAGGG", subseq_length=37, min_density=0.3),
], ids=["fixed", "iupac", "pattern_n", "p3", "mixed_18_tvr", "L37"])
def test_sparse_exceptions_take_the_bundle_scan(cfg):
    L = cfg.get("subseq_length", 100)
    seqs = _sparse_exception_reads(zlib.crc32(str(sorted(cfg.items())).encode()), L)
    nt = _nt(**cfg)
    assert nt.tscan
    # which reads the bundles take: nt_exc_marks against the restated rule
    mm = max(len(p) for p in (cfg["patterns"] + " " + cfg.get("tvr_patterns", "")).split())
    exc_off, exc_pos = [0], []
    for s in seqs:
        exc_pos += [i for i, ch in enumerate(s) if ch not in "ACGTacgt"]
        exc_off.append(len(exc_pos))
    lens = np.array([len(s) for s in seqs], np.uint32)
    marks = nt.exc_marks(lens, np.array(exc_off, np.uint32), np.array(exc_pos, np.uint32))
    want = [len(_exc_windows(exc_pos[exc_off[r]:exc_off[r + 1]], len(seqs[r]), L, mm)) > EXC_WINDOWS
            for r in range(len(seqs))]
    assert marks.tolist() == [int(x) for x in want]
    with_exc = sum(1 for r in range(len(seqs)) if exc_off[r + 1] > exc_off[r])
    assert 0 < int(marks.sum()) < with_exc // 2  # most reads with letters are bundled
    res = nt.analyze(seqs, want_windows=True, want_hits=False)
    compare(nt, res, oracle_rows(seqs, cfg["patterns"], tvr=cfg.get("tvr_patterns"), L=L,
                                 min_density=cfg.get("min_density", 0.6)), check_hits=False)
    assert res["telomeric"].sum() > 20


def test_sparse_exceptions_specialised_call(monkeypatch):
    # the same recounts in the calling kernel specialised for the patterns
    monkeypatch.setenv("NT_CALL_JIT", "1")
    seqs = _sparse_exception_reads(77)
    for pats, tvr in (("TTAGGG", None), ("TTAGGG TCAGGG", "TGAGGG TTGGGG")):
        nt = _nt(patterns=pats, tvr_patterns=tvr)
        res = nt.analyze(seqs, want_windows=True, want_hits=False)
        assert nt.call_jit(), "the specialised calling kernel did not run"
        compare(nt, res, oracle_rows(seqs, pats, tvr=tvr), check_hits=False)
        nt.close()


def _n_mers(k, n, seed):
    rng = np.random.default_rng(seed)
    out = ["TTAGGG"]
    while len(out) < n:
        m = "".join(rng.choice(list("ACGT"), k))
        if m not in out:
            out.append(m)
    return " ".join(out)


def test_many_patterns_aot_lds_overflow():
    """33 patterns + 2 TVRs (68 hit counters): the ahead-of-time per-read scan
    keeps 64 hit counters per wave and counter in LDS, more than a workgroup
    may take even for a read without windows -- every read goes to the
    global-scratch instantiation instead of a failing LDS launch."""
    cfg = dict(patterns=_n_mers(6, 33, 5), tvr_patterns="TGAGGG TTGGGG")
    _random_reads(cfg, False, check_tscan=False)


def test_many_patterns_specialised_call(monkeypatch):
    monkeypatch.setenv("NT_CALL_JIT", "1")
    nt = _random_reads(MANY[0], True, check_tscan=False)
    assert nt.call_jit(), "the specialised calling kernel did not run"


# TVRs of 33..64 letters (the reference takes TVRs of any length: NanoTel.R:
# 360-393; the scan carries a second overflow word, the calling kernel wider
# neighbourhoods).  The TVR motif ACCCTG is >= 2 letters from every pattern, so
# P3 differs from P2 exactly where the long TVR matches.
LONG_TVR = [
    dict(patterns="TTAGGG TCAGGG CTAGGG TTAGGC GGGTTA TTTAGG TTAGGA TTCGGG TAAGGG",
         tvr_patterns=("ACCCTG" * 7)[:40]),
    dict(patterns="TTAGGG", tvr_patterns=("ACCCTG" * 6)[:33] + " TGAGGG"),
    dict(patterns="TTAGGG TCAGGG", tvr_patterns=("ACCCTG" * 11)[:64] + " " + ("ACCCTGACCNTG" * 4)[:45]),
]


def _long_tvr_reads(seed, n_reads=150):
    """Reads with a TTAGGG tract next to an ACCCTG tract (either order, at
    either end or inside), TVR-only and plain reads; 1 % substitutions, IUPAC
    exception letters in every 5th read, lower case in every 7th."""
    rng = np.random.default_rng(seed)
    bases = np.array(list("ACGT"))
    seqs = []
    for i in range(n_reads):
        n = int(rng.choice([rng.integers(1, 400), rng.integers(400, 6000), rng.integers(6000, 30000)]))
        s = list(bases[rng.integers(0, 4, n)])
        a, b = int(rng.integers(0, 2500)), int(rng.integers(0, 2500))
        kind = i % 4
        tract = (("TTAGGG" * (a // 6 + 1))[:a] + ("ACCCTG" * (b // 6 + 1))[:b] if kind == 0 else
                 ("ACCCTG" * (b // 6 + 1))[:b] + ("TTAGGG" * (a // 6 + 1))[:a] if kind == 1 else
                 ("ACCCTG" * (b // 6 + 1))[:b] if kind == 2 else "")
        tract = tract[:n]
        at = 0 if i % 3 == 0 else (n - len(tract) if i % 3 == 1 else int(rng.integers(0, max(1, n - len(tract)))))
        for k, ch in enumerate(tract):
            s[at + k] = ch if rng.random() >= 0.01 else bases[rng.integers(0, 4)]
        if i % 5 == 0:
            for k in np.nonzero(rng.random(n) < 0.002)[0]:
                s[k] = "NRYKMSWBDHV"[rng.integers(0, 11)]
        if i % 7 == 0:
            for k in np.nonzero(rng.random(n) < 0.01)[0]:
                s[k] = s[k].lower()
        seqs.append("".join(s))
    return seqs


@pytest.mark.parametrize("cfg", LONG_TVR, ids=["9_pat_40_letter_tvr", "33_letter_tvr", "64_letter_iupac_tvr"])
@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_long_tvr(cfg, jit):
    seqs = _long_tvr_reads(zlib.crc32(str(sorted(cfg.items())).encode()))
    nt = _nt(jit=jit, **cfg)
    assert not nt.tscan  # the bundle scan takes patterns / TVRs of <= 32 letters
    res, _ = _check_both(nt, seqs, oracle_rows(seqs, cfg["patterns"], tvr=cfg["tvr_patterns"]))
    p3 = res["start"][:, 2] != -1
    differs = (res["start"][:, 2] != res["start"][:, 1]) | (res["end"][:, 2] != res["end"][:, 1])
    assert p3.sum() > 10 and differs.sum() > 5, "the long TVR did not change P3"


def test_long_tvr_specialised_call(monkeypatch):
    monkeypatch.setenv("NT_CALL_JIT", "1")
    cfg = LONG_TVR[1]  # (a hiprtc build of seconds; LONG_TVR[0]'s takes minutes uncached)
    seqs = _long_tvr_reads(7)
    nt = _nt(jit=True, **cfg)
    _check_both(nt, seqs, oracle_rows(seqs, cfg["patterns"], tvr=cfg["tvr_patterns"]))
    assert nt.call_jit(), "the specialised calling kernel did not run"


def test_tvr_length_limit():
    from nanotel_amd import NanoTelError
    _nt(patterns="TTAGGG", tvr_patterns="A" * 64)
    with pytest.raises(NanoTelError) as e:
        _nt(patterns="TTAGGG", tvr_patterns="A" * 65)
    assert e.value.name == "NT_E_LIMIT"


# Short and ragged reads on the bundle path: 10 kb reads (100 windows, a
# bundle's second stripe part-filled), reads whose windows fill every block of
# their bundle (3,200 and 3,160 bases: the checkpoint at window nw is the
# read's total), ragged lengths, 700-base reads.
def _short_ragged_reads(seed):
    rng = np.random.default_rng(seed)
    lens = ([10000] * 128 + [3200] * 64 + [3160] * 64 + [int(x) for x in rng.integers(1500, 4000, 96)] +
            [700] * 32 + [int(x) for x in rng.integers(5000, 12000, 40)])
    seqs = []
    for i, n in enumerate(lens):
        where = ["left", "right", "mid"][i % 3]
        seqs.append(_telo_read(rng, n, where=where, tract=(100, min(n, 2500)), sub=0.02 if i % 2 else 0.05,
                               lower=0.01 if i % 7 == 0 else 0.0))
    return seqs


@pytest.mark.parametrize("cfg", [dict(patterns="TTAGGG"), dict(patterns="TTAGGG TCAGGG", tvr_patterns="TGAGGG TTGGGG")],
                         ids=["p2", "p3"])
def test_short_ragged_bundles(cfg):
    seqs = _short_ragged_reads(11)
    nt = _nt(**cfg)
    assert nt.tscan
    res = nt.analyze(seqs, want_windows=True, want_hits=False)
    compare(nt, res, oracle_rows(seqs, cfg["patterns"], tvr=cfg.get("tvr_patterns")), check_hits=False)


def _random_reads(cfg, jit, check_tscan=True):
    rng = np.random.default_rng(zlib.crc32(str(sorted(cfg.items())).encode()))
    seqs = []
    right = cfg.get("check_right_edge", False)
    motif = "CCCTAA" if right else "TTAGGG"
    for i in range(120):
        n = int(rng.choice([rng.integers(51 if right else 1, 400), rng.integers(400, 5000),
                            rng.integers(5000, 30000)]))
        where = ["left", "right", "mid"][i % 3]
        seqs.append(_telo_read(rng, n, motif=motif, where=where,
                               exc=0.002 if i % 5 == 0 else 0.0, lower=0.01 if i % 7 == 0 else 0.0))
    nt = _nt(jit=jit, **cfg)
    if check_tscan:
        assert nt.tscan == jit
    orow = oracle_rows(seqs, cfg["patterns"], tvr=cfg.get("tvr_patterns"), L=cfg.get("subseq_length", 100),
                       min_density=cfg.get("min_density", 0.6), right_edge=right, rc=cfg.get("rc", False))
    _check_both(nt, seqs, orow)
    return nt


@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_iupac_subject_letters_and_tiny_reads(jit):
    rng = np.random.default_rng(7)
    seqs = ["A", "T", "N", "TTAGGG", "TTAGG", "NNNNNNNNNN", "TTAGGGTTAGGGTTAGGGNNNN"]
    for n in range(1, 140, 3):
        seqs.append(_telo_read(rng, n, tract=(0, n), exc=0.05))
    for pats in ("TTAGGG", "YYAGGG", "TTAGGG TCAGGG", "NNNNNN"):
        nt = _nt(jit=jit, patterns=pats, tvr_patterns="TGAGGG")
        _check_both(nt, seqs, oracle_rows(seqs, pats, tvr="TGAGGG"))


@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_long_reads_global_scratch_path(jit):
    # reads beyond the LDS budget go through the global-scratch kernel
    rng = np.random.default_rng(11)
    seqs = [_telo_read(rng, 230000, tract=(5000, 20000)), _telo_read(rng, 1200, where="left"),
            _telo_read(rng, 181000, where="right", tract=(5000, 9000))]
    for pats, tvr in (("TTAGGG", "TTGGGG"), ("TTAGGG", None)):
        nt = _nt(jit=jit, patterns=pats, tvr_patterns=tvr)
        _check_both(nt, seqs, oracle_rows(seqs, pats, tvr=tvr))


@pytest.mark.parametrize("right", [False, True], ids=["left_edge", "right_edge"])
def test_reads_with_9_to_16_bitmask_words(right):
    # the calling kernel copies a pass's telomeric-window bitmask to LDS when
    # it has <= 16 words (<= 1,024 windows): reads of 513-1,024 windows, around
    # the 512 / 1,024 boundaries, tracts at the left, right and inside
    rng = np.random.default_rng(21 + int(right))
    motif = "CCCTAA" if right else "TTAGGG"
    seqs = []
    for i, n in enumerate([51249, 51250, 51300, 64001, 77777, 90000, 102399, 102400, 102449, 102450,
                           60000, 99000]):
        seqs.append(_telo_read(rng, n, motif=motif, where=["left", "right", "mid"][i % 3], tract=(2000, 15000)))
    for tvr in (None, "TTGGGG"):
        nt = _nt(patterns=motif, tvr_patterns=tvr, check_right_edge=right)
        res, _ = _check_both(nt, seqs, oracle_rows(seqs, motif, tvr=tvr, right_edge=right))
        assert res["telomeric"].sum() > 0


def test_error_behaviour():
    from nanotel_amd import NanoTelError
    nt = _nt(patterns="CCCTAA", check_right_edge=True)
    with pytest.raises(NanoTelError) as e:
        nt.analyze(["ACGT" * 10])  # n <= 50: find_right_telo on a 0-row table
    assert e.value.name == "NT_E_RIGHT_EMPTY"
    nt = _nt(patterns="TTAGGG")
    with pytest.raises(NanoTelError) as e:
        nt.analyze(["ACGTX"])
    assert e.value.name == "NT_E_LETTER"
    with pytest.raises(NanoTelError) as e:
        nt.analyze(["ACGT", ""])
    assert e.value.name == "NT_E_EMPTY_READ"
    with pytest.raises(NanoTelError) as e:
        _nt(patterns=" TTAGGG")
    assert e.value.name == "NT_E_PATTERN"


@pytest.mark.parametrize("tvr", [None, "TTGGGG"], ids=["p2", "p3_split"])
def test_error_rows_agree_across_calling_forms(tvr, monkeypatch):
    """Rows of reads the reference errors on (find_right_telo on a 0-row table,
    --check_right_edge, reads of <= 50 bases): the ahead-of-time calling kernel
    and the specialised one (a kernel per pass for 3-pass programs, its errors
    carried through end = -2 / -3 to the combine kernel) write the same rows
    -- start = end = -1, density 0 for the failing pass, the error flag --
    beside normal rows, and nt_analyze_host returns NT_E_RIGHT_EMPTY."""
    import ctypes
    from nanotel_amd._lib import lib
    rng = np.random.default_rng(44)
    seqs = [_telo_read(rng, int(rng.integers(300, 6000)), motif="CCCTAA", where="right") for _ in range(40)]
    seqs[7] = "ACGT" * 10
    seqs[23] = "CCCTAA" * 8
    bseqs = [x.encode() for x in seqs]
    ptrs = (ctypes.c_char_p * len(bseqs))(*bseqs)
    lens = np.array([len(b) for b in bseqs], np.uint64)
    got = []
    for jit in ("0", "1"):
        monkeypatch.setenv("NT_CALL_JIT", jit)
        nt = _nt(patterns="CCCTAA", tvr_patterns=tvr, check_right_edge=True)
        o = dict(start=np.zeros((40, 3), np.int32), end=np.zeros((40, 3), np.int32),
                 density=np.zeros((40, 3)), flags=np.zeros(40, np.uint8))
        rc = lib().nt_analyze_host(nt.handle, ctypes.addressof(ptrs), lens.ctypes.data, 40,
                                   o["start"].ctypes.data, o["end"].ctypes.data, o["density"].ctypes.data,
                                   o["flags"].ctypes.data, None, None)
        assert rc == -5  # NT_E_RIGHT_EMPTY
        assert nt.call_jit() == (jit == "1")
        got.append(o)
        nt.close()
    for k in ("start", "end", "density", "flags"):
        assert np.array_equal(got[0][k], got[1][k]), k
    assert got[0]["flags"][7] & 0x20 and got[0]["flags"][23] & 0x20
    assert (got[0]["start"][7, :2] == -1).all() and (got[0]["end"][7, :2] == -1).all()
    assert (got[0]["flags"] & 1).sum() > 5


def test_device_synth_matches_host_generator():
    import torch
    from nanotel_amd import NanoTel, read_blocks, synth_params, synth_read_ascii
    sp = synth_params(read_len=5000, first_read=123)
    nt = _nt(patterns="TTAGGG")
    n = 16
    nblk = read_blocks(5000)
    assert nblk == 2 * 79
    planes = torch.zeros(n * nblk * 2, dtype=torch.int32, device="cuda")
    nt.synth_device(sp, n, planes.data_ptr())
    nt.synchronize()
    p = planes.cpu().numpy().view(np.uint32).reshape(n, nblk, 2)
    for r in range(n):
        host = synth_read_ascii(sp, r)
        lo = np.unpackbits(np.ascontiguousarray(p[r, :, 0]).view(np.uint8), bitorder="little")[:5000]
        hi = np.unpackbits(np.ascontiguousarray(p[r, :, 1]).view(np.uint8), bitorder="little")[:5000]
        dev = "".join("ACGT"[c] for c in (lo + 2 * hi))
        assert dev == host


def _device_batch(nt, sp, n, read_len, L=100, hits=True):
    """Synthetic reads generated on the device + the uniform layout (bench path)."""
    import torch
    from nanotel_amd import read_blocks, window_count, window_rows
    nblk = read_blocks(read_len)
    nw = window_count(read_len, L)
    rows = window_rows(nw)  # padded count rows (nt_common.h)
    t = dict(
        planes=torch.zeros(n * nblk * 2, dtype=torch.int32, device="cuda"),
        blk_off=torch.empty(n, dtype=torch.int64, device="cuda"),
        lens=torch.empty(n, dtype=torch.int32, device="cuda"),
        win_off=torch.empty(n, dtype=torch.int64, device="cuda"),
        wc=torch.zeros(n * rows * nt.n_pass, dtype=torch.uint8 if nt.count_bytes == 1 else torch.int16,
                       device="cuda"),
        start=torch.empty(n * 3, dtype=torch.int32, device="cuda"),
        end=torch.empty(n * 3, dtype=torch.int32, device="cuda"),
        dens=torch.empty(n * 3, dtype=torch.float64, device="cuda"),
        flags=torch.zeros(n, dtype=torch.uint8, device="cuda"),
        hits=torch.zeros(n * nt.n_hits if hits else 1, dtype=torch.int32, device="cuda"),
    )
    nt.synth_device(sp, n, t["planes"].data_ptr())
    nt.uniform_layout_device(n, read_len, t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                             t["win_off"].data_ptr())
    t["nw"], t["rows"] = nw, rows
    return t


def _valid_counts(t, n, n_pass, wc=None):
    """The window counts of a uniform batch without the row padding: (n, n_pass, nw)."""
    wc = t["wc"] if wc is None else wc
    return wc.reshape(n, n_pass, t["rows"])[:, :, :t["nw"]]


def _run_device(nt, t, n, read_len):
    nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                        t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                        t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(),
                        t["wc"].data_ptr(), hits=t["hits"].data_ptr())
    nt.synchronize()


@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_device_resident_path_matches_host_path(jit):
    # the bench's device-resident batch (device generator + uniform layout)
    # against the host-packed path and, on a sample, the oracle
    from nanotel_amd import synth_params, synth_read_ascii
    n, read_len = 96, 50000
    sp = synth_params(read_len=read_len, first_read=5000)
    nt = _nt(jit=jit, patterns="TTAGGG")
    t = _device_batch(nt, sp, n, read_len)
    _run_device(nt, t, n, read_len)
    seqs = [synth_read_ascii(sp, i) for i in range(n)]
    res = nt.analyze(seqs, want_windows=True, want_hits=True)
    assert np.array_equal(t["start"].cpu().numpy().reshape(n, 3), res["start"])
    assert np.array_equal(t["end"].cpu().numpy().reshape(n, 3), res["end"])
    assert np.array_equal(t["dens"].cpu().numpy().reshape(n, 3).view(np.uint64),
                          res["density"].view(np.uint64))
    assert np.array_equal(t["flags"].cpu().numpy(), res["flags"])
    assert np.array_equal(_valid_counts(t, n, nt.n_pass).cpu().numpy().view(nt.count_dtype),
                          res["win_counts"].reshape(n, nt.n_pass, -1)[:, :, :t["nw"]])
    assert np.array_equal(t["hits"].cpu().numpy().view(np.uint32).reshape(n, -1), res["hits"])
    compare(nt, res, oracle_rows(seqs[:6], "TTAGGG"))


def _device_bundles(nt, t, n, read_len, has_exc=None):
    """The bench's bundles of a device batch (host plan from the lengths and
    block offsets); has_exc: reads left to the per-read scan (their list goes
    with the bundles)."""
    import torch
    from nanotel_amd.api import DeviceBundles
    plan = nt.bundle_plan(np.full(n, read_len, np.uint32), has_exc, blk_off=t["blk_off"].cpu().numpy().view(np.uint64))
    d = dict(bnd_read=torch.from_numpy(plan.bnd_read.view(np.int32)).cuda())
    nl = len(plan.list)
    if nl:
        d["list"] = torch.from_numpy(plan.list.view(np.int32)).cuda()
    b = DeviceBundles(d["bnd_read"].data_ptr(), plan.n_bundles, d["list"].data_ptr() if nl else 0, nl)
    nt.synchronize()
    return b, d


@pytest.mark.parametrize("read_len", [50000, 10000, 6450, 3001])
def test_device_bundle_scan_matches_per_read_scan(read_len):
    # the bench's path: device-generated reads, bundle layout on the device,
    # bundle scan; against the per-read scan of the same batch (hit counters
    # asked for) on every output, and the oracle on a sample
    from nanotel_amd import synth_params, synth_read_ascii
    n = 160  # 5 bundles
    sp = synth_params(read_len=read_len, first_read=900)
    nt = _nt(patterns="TTAGGG")
    assert nt.tscan
    t = _device_batch(nt, sp, n, read_len)
    _run_device(nt, t, n, read_len)
    ref = {k: t[k].clone() for k in ("start", "end", "dens", "flags", "wc")}
    for k in ref:
        t[k].zero_()
    b, keep = _device_bundles(nt, t, n, read_len)
    nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                        t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                        t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr(),
                        bundles=b)
    nt.synchronize()
    import torch
    for k in ref:
        if k == "wc":  # the padding windows are unspecified
            assert torch.equal(_valid_counts(t, n, nt.n_pass), _valid_counts(t, n, nt.n_pass, ref[k])), k
        else:
            assert torch.equal(t[k], ref[k]), k
    seqs = [synth_read_ascii(sp, i) for i in range(0, n, 23)]
    res = {"start": t["start"].cpu().numpy().reshape(n, 3)[::23], "end": t["end"].cpu().numpy().reshape(n, 3)[::23],
           "density": t["dens"].cpu().numpy().reshape(n, 3)[::23], "flags": t["flags"].cpu().numpy()[::23]}
    res["telomeric"] = (res["flags"] & 1) != 0
    compare(nt, res, oracle_rows(seqs, "TTAGGG"), check_windows=False, check_hits=False)


@pytest.mark.parametrize("tvr", [None, "TGAGGG TTGGGG"], ids=["p2", "p3"])
def test_device_bundles_with_sparse_exceptions(tvr):
    # bench.py --n-frac: device-generated reads, one N in every 4th read as an
    # exception list entry only (the planes keep the
    # generator's base there), all of them in the bundles; against the oracle
    # on the reads with that letter written in, window counts included
    import torch
    import bench
    from nanotel_amd import synth_params, synth_read_ascii
    n, read_len = 320, 12000
    pats = "TTAGGG TCAGGG" if tvr else "TTAGGG"
    nt = _nt(patterns=pats, tvr_patterns=tvr)
    sp = synth_params(read_len=read_len, first_read=77, variant_rate=0.05 if tvr else 0.0)
    t = _device_batch(nt, sp, n, read_len, hits=False)
    off, pos, code = bench.exc_synth(n, read_len, 0.25, 0)
    assert len(pos) == n // 4
    ex = [torch.from_numpy(off.view(np.int32)).cuda(), torch.from_numpy(pos.view(np.int32)).cuda(),
          torch.from_numpy(code).cuda()]
    marks = nt.exc_marks(np.full(n, read_len, np.uint32), off, pos)
    assert int(marks.sum()) == 0  # one letter each: every read in a bundle
    b, keep = _device_bundles(nt, t, n, read_len, marks)
    assert b.n_list == 0
    nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                        t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                        t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr(),
                        exc_off=ex[0].data_ptr(), exc_pos=ex[1].data_ptr(), exc_code=ex[2].data_ptr(), bundles=b)
    nt.synchronize()
    idx = list(range(0, 96, 4)) + [1, 2, 3, 5, 6]
    seqs = []
    for i in idx:
        s = list(synth_read_ascii(sp, i))
        for e in range(int(off[i]), int(off[i + 1])):
            s[int(pos[e])] = "N"
        seqs.append("".join(s))
    res = {"start": t["start"].cpu().numpy().reshape(n, 3)[idx], "end": t["end"].cpu().numpy().reshape(n, 3)[idx],
           "density": t["dens"].cpu().numpy().reshape(n, 3)[idx], "flags": t["flags"].cpu().numpy()[idx]}
    res["telomeric"] = (res["flags"] & 1) != 0
    orows = oracle_rows(seqs, pats, tvr=tvr, want_hits=False)
    compare(nt, res, orows, check_windows=False, check_hits=False)
    wc = _valid_counts(t, n, nt.n_pass).cpu().numpy().view(nt.count_dtype)
    for k, i in enumerate(idx):
        for p in range(nt.n_pass):
            assert wc[i, p].tolist() == orows[k]["win_counts"][p], (i, p)
    assert res["telomeric"].sum() > 3


def test_pipelined_batches_match_serial():
    """nt_set_pipelined: each call's last bundle range's calling runs beside the
    next call's scan (the bench's stream of batches).  Four calls over three
    different device batches, each with its own outputs, equal the serial
    calls' outputs bit for bit (the library's aux buffers alternate; a shared
    one would be overwritten under the running calling)."""
    import torch
    from nanotel_amd import synth_params
    n, read_len = 8192, 10000  # 256 bundles: two bundle ranges
    nt = _nt(patterns="TTAGGG")
    assert nt.tscan
    batches = []
    for first in (0, 70000, 140000):
        t = _device_batch(nt, synth_params(read_len=read_len, first_read=first), n, read_len, hits=False)
        b, keep = _device_bundles(nt, t, n, read_len)
        batches.append((t, b, keep))
    keys = ("start", "end", "dens", "flags", "wc")

    def run(t, b, o):
        nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                            t["win_off"].data_ptr(), n, n * t["rows"], read_len, o["start"].data_ptr(),
                            o["end"].data_ptr(), o["dens"].data_ptr(), o["flags"].data_ptr(), o["wc"].data_ptr(),
                            bundles=b)

    refs = []
    for t, b, _ in batches:
        o = {k: torch.full_like(t[k], 0x55) for k in keys}
        run(t, b, o)
        nt.synchronize()
        refs.append(o)
    order = [0, 1, 2, 0]
    outs = [{k: torch.full_like(batches[i][0][k], 0x55) for k in keys} for i in order]
    nt.set_pipelined(True)
    for i, o in zip(order, outs):
        run(batches[i][0], batches[i][1], o)
    nt.join()
    nt.synchronize()
    nt.set_pipelined(False)
    for i, o in zip(order, outs):
        t, r = batches[i][0], refs[i]
        for k in keys:
            if k == "wc":
                assert torch.equal(_valid_counts(t, n, nt.n_pass, o[k]), _valid_counts(t, n, nt.n_pass, r[k])), (i, k)
            else:
                assert torch.equal(o[k], r[k]), (i, k)
    assert int((refs[0]["flags"] & 1).sum()) > 1000  # telomeric reads: the calling did work
    nt.close()


@pytest.mark.parametrize("back", [0, 1], ids=["one_input_set", "two_input_sets"])
def test_pipelined_calls_with_rewritten_inputs(back):
    """Pipelined calls whose INPUTS are rewritten between calls: a
    caller with one input set waits for the previous call's calling
    (nt_wait_call(ctx, 0)) before refilling it on the context stream; one with
    two alternating sets waits for the call before that (back = 1), keeping the
    overlap.  Every call's outputs equal the serial calls' bit for bit."""
    import torch
    from nanotel_amd import synth_params
    from nanotel_amd.api import DeviceBundles
    n, read_len = 8192, 10000
    nt = _nt(patterns="TTAGGG")
    st = torch.cuda.Stream()
    nt.set_stream(st.cuda_stream)
    batches = []
    with torch.cuda.stream(st):
        for first in (0, 70000, 140000):
            t = _device_batch(nt, synth_params(read_len=read_len, first_read=first), n, read_len, hits=False)
            b, keep = _device_bundles(nt, t, n, read_len)
            batches.append((t, b, keep))
        keys = ("start", "end", "dens", "flags", "wc")

        def run(t, b, o):
            nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                                t["win_off"].data_ptr(), n, n * t["rows"], read_len, o["start"].data_ptr(),
                                o["end"].data_ptr(), o["dens"].data_ptr(), o["flags"].data_ptr(),
                                o["wc"].data_ptr(), bundles=b)

        refs = []
        for t, b, _ in batches:
            o = {k: torch.full_like(t[k], 0x55) for k in keys}
            run(t, b, o)
            nt.synchronize()
            refs.append(o)
        # the input sets the caller rewrites: the planes (the uniform layout and
        # the bundle lists are the same for every batch here)
        sets = []
        for _ in range(back + 1):
            t0, b0, _ = batches[0]
            x = dict(t0)
            x["planes"] = torch.empty_like(t0["planes"])
            sets.append((x, b0))
        order = [0, 1, 2, 0, 2, 1]
        outs = [{k: torch.full_like(batches[i][0][k], 0x55) for k in keys} for i in order]
        nt.set_pipelined(True)
        for c, (i, o) in enumerate(zip(order, outs)):
            x, xb = sets[c % len(sets)]
            if c >= len(sets):
                nt.wait_call(back)  # the calling that still reads this set
            x["planes"].copy_(batches[i][0]["planes"])
            run(x, xb, o)
        nt.join()
        nt.synchronize()
        nt.set_pipelined(False)
    for i, o in zip(order, outs):
        t, r = batches[i][0], refs[i]
        for k in keys:
            if k == "wc":
                assert torch.equal(_valid_counts(t, n, nt.n_pass, o[k]), _valid_counts(t, n, nt.n_pass, r[k])), (i, k)
            else:
                assert torch.equal(o[k], r[k]), (i, k)
    nt.close()


@pytest.mark.parametrize("tvr", [None, "TGAGGG TTGGGG"], ids=["p2", "p3"])
def test_bundle_ranges_with_mixed_lengths_and_exceptions(tvr):
    # enough bundles for the two bundle-scan ranges (calling beside the scan),
    # reads of many lengths (bundles sorted by length, ragged ends, reads of one
    # window) and ~4 % of reads with N / IUPAC letters (the short ones in the
    # bundles, their windows near the letters recounted; the long ones, whose
    # letters reach more than NT_EXC_WINDOWS windows, on the per-read scan)
    rng = np.random.default_rng(20261016)
    seqs = []
    for i in range(4500):
        n = int(rng.choice([int(rng.integers(1, 400)), int(rng.integers(400, 3000)), int(rng.integers(3000, 9000))]))
        seqs.append(_telo_read(rng, n, where=["left", "right", "mid"][i % 3], tract=(50, 2500),
                               exc=0.002 if i % 25 == 0 else 0.0))
    pats = "TTAGGG TCAGGG" if tvr else "TTAGGG"
    nt = _nt(patterns=pats, tvr_patterns=tvr)
    assert nt.tscan
    _check_both(nt, seqs, oracle_rows(seqs, pats, tvr=tvr))
    nt.close()


@pytest.mark.parametrize("cfg", [("TTAGGG", None, 1_000_000, 50_000, 0.0),
                                 ("TTAGGG TCAGGG", "TGAGGG TTGGGG", 400_000, 50_000, 0.05)],
                         ids=["c50k_full", "c4_shape"])
def test_full_size_bundle_scan_equals_per_read_scan(cfg):
    # BASELINE's headline batch (1 M x 50 kb, 50 Gbases) and the c4 program:
    # the bundle scan (as bench.py runs it) and the per-read scan agree on every
    # output of every read -- a size-independent check of the path at full size
    # (the oracle covers the same code on samples above)
    import torch
    from nanotel_amd import synth_params
    pats, tvr, n, read_len, var = cfg
    nt = _nt(patterns=pats, tvr_patterns=tvr)
    assert nt.tscan
    sp = synth_params(read_len=read_len, first_read=31, variant_rate=var)
    t = _device_batch(nt, sp, n, read_len)
    nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                        t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                        t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr())
    nt.synchronize()
    ref = {k: t[k].clone() for k in ("start", "end", "dens", "flags", "wc")}
    for k in ref:
        t[k].zero_()
    b, keep = _device_bundles(nt, t, n, read_len)
    nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                        t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                        t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr(),
                        bundles=b)
    nt.synchronize()
    for k in ("start", "end", "dens", "flags"):
        assert torch.equal(t[k], ref[k]), k
    assert torch.equal(_valid_counts(t, n, nt.n_pass), _valid_counts(t, n, nt.n_pass, ref["wc"]))
    assert int(((t["flags"] & 1) != 0).sum()) > n // 4  # telomeric reads present
    del t, ref, keep
    torch.cuda.empty_cache()


@pytest.mark.parametrize("L", [37, 100, 50, 127, 170])
def test_bundle_scan_ragged_packed_batch(L):
    # ragged bundles from the host packer (lengths sorted within a bundle, read
    # ends inside plane words, bundles whose reads lie anywhere in the batch),
    # odd L (the second half window one position short), L = 127 and 170
    # (rows of more than 64 units: two loads a slot; 3 ranges a walk): the bundle scan
    # against the per-read scan of the same device batch on every output
    rng = np.random.default_rng(5 + L)
    seqs = []
    for i in range(150):
        n_i = int(rng.integers(1, 12000))
        s_i = bytearray(rng.choice(list(b"ACGT"), n_i).tolist())
        if i % 3 == 0 and n_i > 3000:  # a telomeric tract somewhere
            a0 = int(rng.integers(0, n_i - 2000))
            s_i[a0:a0 + 1800] = (b"TTAGGG" * 300)[:1800]
        seqs.append(bytes(s_i))
    _bundle_scan_vs_per_read(seqs, L, 5, min_telomeric=6)


def _bundle_scan_vs_per_read(seqs, L, n_bundles, min_telomeric=0):
    # host-packed reads: the bundle scan against the per-read scan of the same
    # device batch on every output (every window count of every read and pass)
    import ctypes
    import torch
    from nanotel_amd import _lib
    from nanotel_amd.api import DeviceBundles
    lib = _lib.lib()
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(x) for x in seqs], np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    assert lib.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, L, ctypes.byref(tb),
                             ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml), ctypes.byref(bad)) == 0
    planes = np.zeros(2 * tb.value + 2, np.uint32)
    blk, ln, wo = np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint64)
    assert lib.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 0, L, planes.ctypes.data,
                             blk.ctypes.data, ln.ctypes.data, wo.ctypes.data, None, None, None) == 0
    nt = _nt(patterns="TTAGGG", subseq_length=L)
    assert nt.tscan
    plan = nt.bundle_plan(ln, blk_off=blk)
    assert plan.n_bundles == n_bundles and len(plan.list) == 0
    dev = {k: torch.from_numpy(v).cuda() for k, v in (("planes", planes.view(np.int32)), ("blk", blk.view(np.int64)),
                                                    ("ln", ln.view(np.int32)), ("wo", wo.view(np.int64)))}
    br = torch.from_numpy(plan.bnd_read.view(np.int32)).cuda()
    bb = DeviceBundles(br.data_ptr(), plan.n_bundles, 0, 0)
    nwc = int(tw.value) * nt.n_pass
    outs = []
    for bundles in (None, bb):
        o = dict(start=torch.full((n * 3,), 7, dtype=torch.int32, device="cuda"),
                 end=torch.full((n * 3,), 7, dtype=torch.int32, device="cuda"),
                 dens=torch.full((n * 3,), 7.0, dtype=torch.float64, device="cuda"),
                 flags=torch.zeros(n, dtype=torch.uint8, device="cuda"),
                 wc=torch.full((nwc,), 0x55, dtype=torch.uint8, device="cuda"))
        nt.scan_call_device(dev["planes"].data_ptr(), dev["blk"].data_ptr(), dev["ln"].data_ptr(),
                            dev["wo"].data_ptr(), n, int(tw.value), int(ml.value), o["start"].data_ptr(),
                            o["end"].data_ptr(), o["dens"].data_ptr(), o["flags"].data_ptr(), o["wc"].data_ptr(),
                            bundles=bundles)
        nt.synchronize()
        outs.append({k: v.cpu().numpy() for k, v in o.items()})
    ref, got = outs
    for k in ("start", "end", "flags"):
        assert np.array_equal(got[k], ref[k]), (k, np.flatnonzero(got[k] != ref[k])[:8])
    assert np.array_equal(got["dens"].view(np.uint64), ref["dens"].view(np.uint64))
    # every window count of every read and pass (padding windows excluded)
    for r in range(n):
        nw = int(lib.nt_window_count(int(ln[r]), L))
        rows = int(lib.nt_window_rows(nw))
        for p in range(nt.n_pass):
            o = int(wo[r]) * nt.n_pass + p * rows
            assert np.array_equal(got["wc"][o:o + nw], ref["wc"][o:o + nw]), (r, p)
    assert int(((ref["flags"] & 1) != 0).sum()) >= min_telomeric


@pytest.mark.parametrize("L", [100, 37, 127, 170])
def test_bundle_scan_short_last_half_stripe(L):
    # bundles whose longest read ends 1..9 windows into its last half stripe
    # (most of the walk's lanes past every read: DESIGN 4.4 tried a tail walk
    # for them) and around them, ragged inside each bundle, a telomeric tract
    # reaching the longest read's end in every other bundle
    rng = np.random.default_rng(40 + L)
    tops = [100, 73, 72, 41, 40, 37, 36, 34, 33, 9, 8, 5, 4, 2, 1]  # windows of each bundle's longest read
    seqs = []
    for i, t in enumerate(tops):
        lo = tops[i + 1] * L + 1 if i + 1 < len(tops) else 1
        hi = t * L
        lens = [hi] + [int(x) for x in rng.integers(lo, hi + 1, 31)]
        for j, n_i in enumerate(lens):
            s_i = bytearray(rng.choice(list(b"ACGT"), n_i).tolist())
            if j == 0 and i % 2 == 0:
                k = min(n_i, 40 * L) // 6 * 6
                s_i[n_i - k:] = (b"TTAGGG" * (k // 6 + 1))[:k]
            seqs.append(bytes(s_i))
    _bundle_scan_vs_per_read(seqs, L, len(tops), min_telomeric=4)


@pytest.mark.parametrize("L", [100, 170])
def test_bundle_scan_short_last_read_at_allocation_end(L):
    # The batch's last read is short and shares a bundle with 31 long reads,
    # and the planes end exactly at the end of their device allocation: every
    # half stripe of the long slots loads a row for the short slot too, up to
    # ~13 KB past its last plane word.  Those loads must stay inside the
    # bundle's buffer range (they load zeros past it; the whole offset is in
    # voffset, which the range check covers).  Bundle scan against the per-read
    # scan of the same device batch on every output.
    import ctypes
    import torch
    from nanotel_amd import _lib
    from nanotel_amd.api import DeviceBundles
    rng = np.random.default_rng(400 + L)
    seqs = []
    for i in range(63):
        n_i = int(rng.integers(30000, 40000))
        s_i = bytearray(rng.choice(list(b"ACGT"), n_i).tolist())
        if i % 2 == 0:
            s_i[:4000] = (b"TTAGGG" * 700)[:4000]
        seqs.append(bytes(s_i))
    seqs.append(b"TTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTT")  # 44 bases: no window
    lib = _lib.lib()
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(x) for x in seqs], np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    assert lib.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, L, ctypes.byref(tb),
                             ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml), ctypes.byref(bad)) == 0
    planes = np.zeros(2 * tb.value, np.uint32)
    blk, ln, wo = np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint64)
    assert lib.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 0, L, planes.ctypes.data,
                             blk.ctypes.data, ln.ctypes.data, wo.ctypes.data, None, None, None) == 0
    assert int(blk[-1]) + 2 == tb.value  # the short read's one block pair ends the planes
    nt = _nt(patterns="TTAGGG", subseq_length=L)
    assert nt.tscan
    plan = nt.bundle_plan(ln, blk_off=blk)
    assert plan.n_bundles == 2 and len(plan.list) == 0
    assert n - 1 in set(plan.bnd_read[32:64].tolist())  # with 31 long reads
    # the planes at the very end of an allocation of whole 2 MiB pages
    pb = planes.nbytes
    alloc = (pb + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    buf = torch.zeros(alloc // 4, dtype=torch.int32, device="cuda")
    off = (alloc - pb) // 4
    assert off % 4 == 0  # 16-byte aligned base
    buf[off:].copy_(torch.from_numpy(planes.view(np.int32)))
    pl_ptr = buf.data_ptr() + 4 * off
    dev = {k: torch.from_numpy(v).cuda() for k, v in (("blk", blk.view(np.int64)), ("ln", ln.view(np.int32)),
                                                    ("wo", wo.view(np.int64)))}
    br = torch.from_numpy(plan.bnd_read.view(np.int32)).cuda()
    bb = DeviceBundles(br.data_ptr(), plan.n_bundles, 0, 0)
    nwc = int(tw.value) * nt.n_pass
    outs = []
    for bundles in (None, bb):
        o = dict(start=torch.full((n * 3,), 7, dtype=torch.int32, device="cuda"),
                 end=torch.full((n * 3,), 7, dtype=torch.int32, device="cuda"),
                 dens=torch.full((n * 3,), 7.0, dtype=torch.float64, device="cuda"),
                 flags=torch.zeros(n, dtype=torch.uint8, device="cuda"),
                 wc=torch.full((nwc,), 0x55, dtype=torch.uint8, device="cuda"))
        nt.scan_call_device(pl_ptr, dev["blk"].data_ptr(), dev["ln"].data_ptr(),
                            dev["wo"].data_ptr(), n, int(tw.value), int(ml.value), o["start"].data_ptr(),
                            o["end"].data_ptr(), o["dens"].data_ptr(), o["flags"].data_ptr(), o["wc"].data_ptr(),
                            bundles=bundles)
        nt.synchronize()
        outs.append({k: v.cpu().numpy() for k, v in o.items()})
    ref, got = outs
    for k in ("start", "end", "flags"):
        assert np.array_equal(got[k], ref[k]), (k, np.flatnonzero(got[k] != ref[k])[:8])
    assert np.array_equal(got["dens"].view(np.uint64), ref["dens"].view(np.uint64))
    for r in range(n):
        nw = int(lib.nt_window_count(int(ln[r]), L))
        rows = int(lib.nt_window_rows(nw))
        for p in range(nt.n_pass):
            o = int(wo[r]) * nt.n_pass + p * rows
            assert np.array_equal(got["wc"][o:o + nw], ref["wc"][o:o + nw]), (r, p)
    assert int(((ref["flags"] & 1) != 0).sum()) >= 20
    nt.close()


def test_rc_device_matches_host_packer():
    # nt_rc_device (the --rc transform of a device-resident batch) against the
    # host packer's fused reverse complement (nt_pack_reads rc = 1) on every
    # plane word of ragged reads: lengths around word and block boundaries,
    # the padding words of each read's blocks zero
    import ctypes
    import torch
    from nanotel_amd import _lib
    rng = np.random.default_rng(77)
    lens_l = [1, 2, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 1000, 4095, 4096, 4097, 50000]
    lens_l += [int(x) for x in rng.integers(1, 20000, 45)]
    seqs = [bytes(rng.choice(list(b"ACGT"), n).tolist()) for n in lens_l]
    lib = _lib.lib()
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array(lens_l, np.uint64)
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    assert lib.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 100, ctypes.byref(tb),
                             ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml), ctypes.byref(bad)) == 0
    packed = []
    for rc in (0, 1):
        planes = np.full(2 * tb.value + 2, 0x5A5A5A5A, np.uint32)
        blk, ln, wo = np.zeros(n, np.uint64), np.zeros(n, np.uint32), np.zeros(n, np.uint64)
        assert lib.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, rc, 100,
                                 planes.ctypes.data, blk.ctypes.data, ln.ctypes.data, wo.ctypes.data,
                                 None, None, None) == 0
        packed.append((planes, blk, ln))
    (fwd, blk, ln), (want, blk1, _) = packed
    assert np.array_equal(blk, blk1)
    nt = _nt(patterns="TTAGGG")
    d_in = torch.from_numpy(fwd.view(np.int32)).cuda()
    d_out = torch.full_like(d_in, 0x3C3C3C3C)
    d_blk = torch.from_numpy(blk.view(np.int64)).cuda()
    d_len = torch.from_numpy(ln.view(np.int32)).cuda()
    nt.rc_device(d_in.data_ptr(), d_out.data_ptr(), d_blk.data_ptr(), d_len.data_ptr(), n)
    nt.synchronize()
    got = d_out.cpu().numpy().view(np.uint32)
    for r in range(n):
        w0 = 2 * int(blk[r])
        nwd = 2 * 2 * ((int(ln[r]) + 63) // 64)  # uint32 words of the read's blocks (lo, hi pairs)
        assert np.array_equal(got[w0:w0 + nwd], want[w0:w0 + nwd]), (r, int(ln[r]))
    nt.close()


def test_bundle_plan_keeps_bundles_compact():
    # nt_bundle_plan with blk_off: a bundle whose reads' planes lie more than
    # 2 GiB apart goes to the per-read scan whole; the others stay bundles
    nt = _nt(patterns="TTAGGG")
    n = 96
    ln = np.full(n, 50000, np.uint32)
    blk = np.arange(n, dtype=np.uint64) * 1564
    blk[40] = np.uint64(1) << 29  # 4 GiB: read 40's bundle (reads 32-63) spans too far
    plan = nt.bundle_plan(ln, blk_off=blk)
    assert plan.n_bundles == 2
    assert np.array_equal(plan.list, np.arange(32, 64, dtype=np.uint32))
    assert set(plan.bnd_read.tolist()) == set(range(32)) | set(range(64, 96))
    plan = nt.bundle_plan(ln)  # no blk_off: the caller vouches
    assert plan.n_bundles == 3 and len(plan.list) == 0


@pytest.mark.parametrize("cfg", [("TTAGGG", None, {}), ("TTAGGG", None, {"NT_CALL_JIT": "1"}),
                                 ("TTAGGG TCAGGG", "TGAGGG TTGGGG", {}),
                                 ("TTAGGG TCAGGG", "TGAGGG TTGGGG", {"NT_CALL_JIT": "1", "NT_CALL_SPLIT": "1"})],
                         ids=["fused_aot", "fused_jit", "p3_aot", "p3_split"])
def test_bundle_spanning_more_than_2gib_is_reported(cfg, monkeypatch):
    # A device batch planned without its blk_off (the caller vouches) whose
    # bundle's planes lie more than 2 GiB apart: the bundle scan cannot address
    # them with one buffer descriptor, so it skips the bundle and marks its
    # reads' first checkpoint (kTsSpanError); every calling form (the fused
    # kernel ahead of time / specialised, the per-pass split and its combine
    # kernel) reports exactly those reads as ROW_DONE | ROW_ERR_ALIGN, and every
    # other read equals the per-read scan of the same batch.
    import torch
    from nanotel_amd import read_blocks, synth_params
    from nanotel_amd._lib import ROW_DONE, ROW_ERR_ALIGN
    from nanotel_amd.api import DeviceBundles
    pats, tvr, env = cfg
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n, read_len, far = 96, 5000, 40
    nt = _nt(patterns=pats, tvr_patterns=tvr)
    assert nt.tscan
    t = _device_batch(nt, synth_params(read_len=read_len, first_read=300), n, read_len, hits=False)
    wpr = 2 * read_blocks(read_len)  # int32 plane words a read
    far_blk = (1 << 28) + 8192       # blocks of 8 bytes: 2 GiB + 64 KB into the buffer (> 2 GiB from the bundle base)
    big = torch.zeros(2 * far_blk + wpr + 64, dtype=torch.int32, device="cuda")
    big[:n * wpr].copy_(t["planes"])
    big[2 * far_blk:2 * far_blk + wpr].copy_(t["planes"][far * wpr:(far + 1) * wpr])
    t["planes"] = big
    t["blk_off"][far] = far_blk
    torch.cuda.synchronize()

    def run(bundles):
        for k in ("start", "end"):
            t[k].fill_(7)
        t["dens"].fill_(7.0)
        t["flags"].zero_()
        t["wc"].fill_(0x55)
        torch.cuda.synchronize()
        nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                            t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                            t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr(),
                            bundles=bundles)
        nt.synchronize()
        return {k: t[k].cpu().numpy().copy() for k in ("start", "end", "dens", "flags", "wc")}

    ref = run(None)  # the per-read scan: one 64-bit address a read
    assert not (ref["flags"] & ROW_ERR_ALIGN).any()
    plan = nt.bundle_plan(np.full(n, read_len, np.uint32))  # no blk_off: the bundle stays
    assert plan.n_bundles == 3 and len(plan.list) == 0
    br = torch.from_numpy(plan.bnd_read.view(np.int32)).cuda()
    got = run(DeviceBundles(br.data_ptr(), plan.n_bundles, 0, 0))
    bad_b = int(np.flatnonzero(plan.bnd_read == far)[0]) // 32
    bad = set(int(r) for r in plan.bnd_read[32 * bad_b:32 * bad_b + 32] if r != 0xFFFFFFFF)
    assert far in bad and len(bad) == 32
    ok = np.array([r not in bad for r in range(n)])
    assert all(int(got["flags"][r]) == (ROW_DONE | ROW_ERR_ALIGN) for r in bad), got["flags"][sorted(bad)]
    assert np.array_equal(got["flags"][ok], ref["flags"][ok])
    assert int(((ref["flags"][ok] & 1) != 0).sum()) > 8  # telomeric reads among the others
    for k in ("start", "end"):
        assert np.array_equal(got[k].reshape(n, 3)[ok], ref[k].reshape(n, 3)[ok]), k
    assert np.array_equal(got["dens"].reshape(n, 3)[ok].view(np.uint64), ref["dens"].reshape(n, 3)[ok].view(np.uint64))
    wc_g = got["wc"].reshape(n, nt.n_pass, t["rows"])[:, :, :t["nw"]]
    wc_r = ref["wc"].reshape(n, nt.n_pass, t["rows"])[:, :, :t["nw"]]
    assert np.array_equal(wc_g[ok], wc_r[ok])
    nt.close()
    del big, t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("tvr", [None, "TGAGGG TTGGGG"], ids=["p2", "p3"])
def test_reads_without_windows_in_bundles_on_a_poisoned_aux_buffer(tvr, monkeypatch):
    # Reads of <= L/2 bases have no window (split_telo, NanoTel.R:216-223) but
    # sit in bundles; the calling kernel's span check reads their first
    # checkpoint, which the bundle scan must write although no flush covers
    # it.  The context first runs a telomeric batch (bitmask words of all
    # ones in the reused aux buffer), then, with the aux buffer filled with
    # 0xFF bytes before every call (NT_DBG_POISON_AUX: every word read must
    # be written), bundles that mix windowless and windowed reads.
    monkeypatch.setenv("NT_DBG_POISON_AUX", "255")
    rng = np.random.default_rng(93)
    nt = _nt(patterns="TTAGGG", tvr_patterns=tvr)
    assert nt.tscan
    telo = [_telo_read(rng, 12000, tract=(6000, 11000), sub=0.0) for _ in range(64)]
    nt.analyze(telo, want_windows=True)
    seqs = [_telo_read(rng, int(k), tract=(0, int(k))) for k in rng.integers(1, 51, 80)]
    seqs += [_telo_read(rng, int(k), tract=(0, int(k))) for k in rng.integers(51, 400, 30)]
    seqs += ["TTAGGG" * 8, "T" * 50, "TTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTT"]
    rng.shuffle(seqs)
    res = nt.analyze(seqs, want_windows=True)
    compare(nt, res, oracle_rows(seqs, "TTAGGG", tvr=tvr), check_hits=False)
    nt.close()


# BASELINE.json configs[2], [3] (10M x 50 kb) and one GPU's shard of
# configs[4] (12.5M x 50 kb, 156 GB of planes resident), bundle scan, and the
# shard on the per-read scan: the bench's full-size batches, sampled against
# the oracle on reads regenerated on the host (nt_synth_ascii) -- the first
# and last reads (the last bundles: block offsets past 2^31) and reads spread
# over the whole batch; every row field and every window count of every pass
# (NanoTel.R:717-766, 1080-1155).
#
# c3 is --rc: the reads are generated as they arrive (rc_layout: the telomere
# is the reverse complement, at the far end) and turned into scan orientation
# by the device reverse complement (nt_rc_device, chunks of 1M reads through a
# scratch buffer) before the scan; the oracle reverse-complements its copy of
# every sampled read (NanoTel.R:2219-2221).
FULL_CONFIGS = {  # patterns, TVRs, reads, variant rate, bundle path, read length, --rc
    "c3": ("YYAGGG", None, 10_000_000, 0.05, True, 50_000, True),
    "c4": ("TTAGGG TCAGGG", "TGAGGG TTGGGG", 10_000_000, 0.05, True, 50_000, False),
    "c5": ("TTAGGG", None, 12_500_000, 0.0, True, 50_000, False),
    "c5_per_read": ("TTAGGG", None, 12_500_000, 0.0, False, 50_000, False),
    "c10k": ("TTAGGG", None, 1_000_000, 0.0, True, 10_000, False),
}


def _rc_device_batch(nt, t, n, read_len, chunk=1_000_000):
    """Reverse-complement every read of a uniform device batch in place, in
    chunks through a scratch buffer (nt_rc_device is out of place)."""
    import torch
    from nanotel_amd import read_blocks
    wpr = read_blocks(read_len) * 2  # int32 plane words a read
    tmp = torch.empty(min(n, chunk) * wpr, dtype=torch.int32, device="cuda")
    for r0 in range(0, n, chunk):
        m = min(chunk, n - r0)
        # the kernel writes read r at planes_out + blk_off[r] words: shift the
        # scratch base back by the chunk's first read
        nt.rc_device(t["planes"].data_ptr(), tmp.data_ptr() - r0 * wpr * 4, t["blk_off"].data_ptr() + 8 * r0,
                     t["lens"].data_ptr() + 4 * r0, m)
        nt.synchronize()
        t["planes"][r0 * wpr:(r0 + m) * wpr].copy_(tmp[:m * wpr])
    torch.cuda.synchronize()
    del tmp


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", list(FULL_CONFIGS))
def test_full_size_config_sampled_vs_oracle(name):
    import torch
    from nanotel_amd import synth_params, synth_read_ascii
    pats, tvr, n, var, bundle, read_len, rc = FULL_CONFIGS[name]
    nt = _nt(patterns=pats, tvr_patterns=tvr, rc=rc)
    sp = synth_params(read_len=read_len, first_read=0, variant_rate=var, rc_layout=rc)
    t = _device_batch(nt, sp, n, read_len, hits=False)
    if rc:
        _rc_device_batch(nt, t, n, read_len)
    b = keep = None
    extra = np.zeros(0, np.int64)
    if bundle:
        b, keep = _device_bundles(nt, t, n, read_len)
    nt.scan_call_device(t["planes"].data_ptr(), t["blk_off"].data_ptr(), t["lens"].data_ptr(),
                        t["win_off"].data_ptr(), n, n * t["rows"], read_len, t["start"].data_ptr(),
                        t["end"].data_ptr(), t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr(),
                        bundles=b)
    nt.synchronize()
    flags = t["flags"]
    assert int((flags & 0x80).eq(0).sum()) == 0, "a read was not processed"
    n_telo = int(((flags & 1) != 0).sum())
    # the sample: 256 first, 384 last (12 bundles), 1400 spread over the batch
    idx = np.unique(np.concatenate([np.arange(256), np.arange(n - 384, n),
                                    np.linspace(256, n - 385, 1400).astype(np.int64), extra]))
    it = torch.from_numpy(idx).cuda()
    res = {"start": t["start"].view(n, 3)[it].cpu().numpy(), "end": t["end"].view(n, 3)[it].cpu().numpy(),
           "density": t["dens"].view(n, 3)[it].cpu().numpy(), "flags": flags[it].cpu().numpy()}
    res["telomeric"] = (res["flags"] & 1) != 0
    rows = t["rows"]
    res["win_counts"] = t["wc"].view(n, nt.n_pass * rows)[it].cpu().numpy().view(nt.count_dtype).reshape(-1)
    res["win_off"] = np.arange(idx.size, dtype=np.int64) * rows
    res["n_windows"] = np.full(idx.size, t["nw"], np.int64)
    del t, keep, it
    torch.cuda.empty_cache()
    seqs = [synth_read_ascii(sp, int(i)) for i in idx]
    compare(nt, res, oracle_rows(seqs, pats, tvr=tvr, rc=rc, want_hits=False), check_hits=False)
    assert res["telomeric"].sum() > idx.size // 4 and n_telo > n // 4
    nt.close()


def test_odd_block_offset_is_reported():
    from nanotel_amd import synth_params
    from nanotel_amd._lib import ROW_DONE, ROW_ERR_ALIGN
    n, read_len = 8, 3000
    nt = _nt(patterns="TTAGGG")
    t = _device_batch(nt, synth_params(read_len=read_len), n, read_len)
    t["blk_off"][3] += 1
    _run_device(nt, t, n, read_len)
    f = t["flags"].cpu().numpy()
    assert f[3] == (ROW_DONE | ROW_ERR_ALIGN)
    assert all((f[i] & ROW_ERR_ALIGN) == 0 for i in range(n) if i != 3)


@pytest.mark.parametrize("path", ["jit", "aot", "bundle"])
def test_offsets_beyond_32_bits(path):
    # Batches of 10M x 50 kb reads have block offsets >= 2^31 and window
    # offsets >= 2^32 (a sign-extended 32-bit block offset once faulted there).
    # Reproduced without allocating them: the planes / window-count base
    # pointers are shifted down by exactly the offsets added to blk_off /
    # win_off.  Bundle path: the bundle scan's descriptor base is its lowest
    # read's planes, 2^34 bytes past the shifted base.
    import torch
    from nanotel_amd import synth_params
    n, read_len = 64 if path != "bundle" else 96, 50000
    nt = _nt(jit=path != "aot", patterns="TTAGGG")
    t = _device_batch(nt, synth_params(read_len=read_len, first_read=77), n, read_len)
    _run_device(nt, t, n, read_len)
    keys = ("start", "end", "dens", "flags", "wc")
    ref = {k: t[k].clone() for k in keys}
    for k in keys:
        t[k].zero_()
    boff, woff = 1 << 31, 1 << 32  # blocks of 8 bytes, windows
    blk, win = t["blk_off"] + boff, t["win_off"] + woff
    bundles, keep = None, None
    if path == "bundle":
        bundles, keep = _device_bundles(nt, t, n, read_len)
    nt.scan_call_device(t["planes"].data_ptr() - boff * 8, blk.data_ptr(), t["lens"].data_ptr(), win.data_ptr(),
                        n, woff + n * t["rows"], read_len, t["start"].data_ptr(), t["end"].data_ptr(),
                        t["dens"].data_ptr(), t["flags"].data_ptr(), t["wc"].data_ptr() - woff * nt.n_pass * nt.count_bytes,
                        bundles=bundles)
    nt.synchronize()
    for k in keys:
        if k == "wc":
            assert torch.equal(_valid_counts(t, n, nt.n_pass), _valid_counts(t, n, nt.n_pass, ref[k])), k
        else:
            assert torch.equal(t[k], ref[k]), k
    del keep


@pytest.mark.parametrize("jit", [True, False], ids=["jit", "aot"])
def test_subbatched_overlap_matches_serial(jit):
    # NT_SUBBATCH > 1: the calling kernel of sub-batch k runs on a second
    # stream beside the scan of sub-batch k+1; outputs must not change
    from nanotel_amd import synth_params
    n, read_len = 1100, 7000
    sp = synth_params(read_len=read_len, first_read=77)
    nt = _nt(jit=jit, patterns="TTAGGG", tvr_patterns="TTGGGG")
    outs = []
    for sub in ("1", "3"):
        os.environ["NT_SUBBATCH"] = sub
        try:
            t = _device_batch(nt, sp, n, read_len)
            _run_device(nt, t, n, read_len)
        finally:
            del os.environ["NT_SUBBATCH"]
        outs.append({k: t[k].cpu().numpy() for k in ("start", "end", "dens", "flags", "wc", "hits")})
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k
    assert (outs[0]["flags"] & 1).sum() > 100


@pytest.mark.parametrize("plan", [("1.0", "3"), ("0.5", "1"), ("0.0", "7"), ("0.9", "64")])
def test_read_distribution_plans(plan):
    # static runs + 8 per-XCD queues (scan_reads): every read scanned exactly
    # once whatever the split between the static part and the claims
    frac, claim = plan
    rng = np.random.default_rng(11)
    lens = rng.integers(1, 3000, 20000)
    lens[::97] = rng.integers(3000, 40000, lens[::97].size)
    alpha = np.frombuffer(b"ACGTTAGGG", dtype=np.uint8)
    seqs = [alpha[rng.integers(0, alpha.size, int(n))].tobytes().decode() for n in lens]
    for i in range(0, len(seqs), 13):
        seqs[i] = "TTAGGG" * (len(seqs[i]) // 6) + seqs[i][: len(seqs[i]) % 6]
    nt = _nt(patterns="TTAGGG")
    ref = nt.analyze(seqs, want_windows=True, want_hits=True)
    os.environ["NT_STATIC_FRAC"], os.environ["NT_CLAIM"] = frac, claim
    try:
        res = nt.analyze(seqs, want_windows=True, want_hits=True)
    finally:
        del os.environ["NT_STATIC_FRAC"], os.environ["NT_CLAIM"]
    for k in ("start", "end", "flags", "win_counts", "hits"):
        assert np.array_equal(ref[k], res[k]), k
    assert np.array_equal(ref["density"].view(np.uint64), res["density"].view(np.uint64))
    assert (res["flags"] & 1).sum() > 1000
    idx = list(range(0, len(seqs), 997))
    compare(nt, {k: v[idx] if isinstance(v, np.ndarray) and v.shape[:1] == (len(seqs),) else v
                 for k, v in res.items()}, oracle_rows([seqs[i] for i in idx], "TTAGGG"), check_windows=False)


@pytest.mark.parametrize("cfg", [
    dict(patterns="TTAGGG"),
    dict(patterns="TTAGGG", check_right_edge=True),
    dict(patterns="TTAGGG CCCTAA", min_density=0.5),
    dict(patterns="YYAGGG", rc=True),
    dict(patterns="ttaggn", min_density=0.7),
    dict(patterns="TTAGGG", min_density=0.61),
])
def test_use_filter_matches_oracle(cfg):
    # --use_filter (filter_reads/filter_density, NanoTel.R:2083-2163) on the GPU
    rng = np.random.default_rng(zlib.crc32(str(sorted(cfg.items())).encode()))
    right = cfg.get("check_right_edge", False)
    motif = {"ttaggn": "TTAGGA"}.get(cfg["patterns"], "TTAGGG")
    seqs = []  # scan orientation (the input is their reverse complement under rc)
    for i in range(400):
        n = int(rng.choice([rng.integers(1, 999), rng.integers(999, 1002), rng.integers(1002, 6000)]))
        s = list(np.array(list("ACGT"))[rng.integers(0, 4, n)])
        if n >= 300 and i % 2 == 0:  # an edge tract of varying length around the threshold
            t = int(rng.integers(40, 200))
            a = n - 270 + int(rng.integers(-20, 20)) if right else 70 + int(rng.integers(-20, 20))
            a = max(0, min(a, n - t))
            for j in range(t):
                s[a + j] = motif[j % 6] if rng.random() > 0.03 else "ACGT"[rng.integers(0, 4)]
        if i % 5 == 0:  # subject ambiguity letters / lowercase
            for j in rng.integers(0, n, max(1, n // 100)):
                s[j] = "NRYKMSWBDHVnacgt"[rng.integers(0, 16)]
        seqs.append("".join(s))
    nt = _nt(**cfg)
    keep = nt.filter([O.reverse_complement(s) for s in seqs] if cfg.get("rc") else seqs)
    P = O.Patterns(cfg["patterns"])
    want = [O.filter_read(s, P, cfg.get("min_density", 0.6), right) for s in seqs]
    bad = [i for i in range(len(seqs)) if bool(keep[i]) != want[i]]
    assert not bad, (len(bad), bad[:5])
    assert 20 < sum(want) < 380


# ---- random programs (seeded fuzz): pattern sets of 1-3 patterns of one
# length (3-12 letters, some IUPAC), optional exact TVRs, subseq_length,
# min_density, --rc and --check_right_edge drawn at random; reads with tracts
# of the first pattern (its IUPAC letters resolved to a base of their set).
# The ahead-of-time kernels for most seeds, the hiprtc bundle scan for a few
# (each of those builds its own kernel).
_IUPAC = {"R": "AG", "Y": "CT", "K": "GT", "M": "AC", "S": "CG", "W": "AT", "B": "CGT", "D": "AGT",
          "H": "ACT", "V": "ACG", "N": "ACGT"}


def _rand_pattern(rng, m, iupac):
    return "".join(rng.choice(list(_IUPAC)) if rng.random() < iupac else "ACGT"[rng.integers(0, 4)]
                   for _ in range(m))


def _fuzz_cfg(seed):
    rng = np.random.default_rng(1000 + seed)
    m = int(rng.integers(3, 13))
    pats = [_rand_pattern(rng, m, 0.15) for _ in range(int(rng.integers(1, 4)))]
    cfg = dict(patterns=" ".join(pats), subseq_length=int(rng.choice([37, 50, 64, 100, 127, 150])),
               min_density=float(rng.choice([0.3, 0.5, 0.6, 0.8])))
    if rng.random() < 0.4:
        m2 = int(rng.integers(3, 13))
        cfg["tvr_patterns"] = " ".join(_rand_pattern(rng, m2, 0.0) for _ in range(int(rng.integers(1, 3))))
    if rng.random() < 0.25:
        cfg["rc"] = True
    if rng.random() < 0.2:
        cfg["check_right_edge"] = True
    motif = "".join(c if c in "ACGT" else _IUPAC[c][rng.integers(0, len(_IUPAC[c]))] for c in pats[0])
    if cfg.get("rc"):  # (the reads are scanned reverse-complemented)
        motif = motif[::-1].translate(str.maketrans("ACGT", "TGCA"))
    return cfg, motif, rng


@pytest.mark.parametrize("seed", range(64))
def test_fuzz_random_programs(seed):
    cfg, motif, rng = _fuzz_cfg(seed)
    jit = seed % 7 == 3  # 9 of the 64 through the hiprtc bundle scan
    right = cfg.get("check_right_edge", False)
    seqs = []
    for i in range(60):
        # (--check_right_edge: reads of at least one window, the reference's
        # find_right_telo stops on an empty window table, NanoTel.R:861)
        n = int(rng.choice([rng.integers(cfg["subseq_length"] // 2 + 1 if right else 1, 600),
                            rng.integers(600, 8000), rng.integers(8000, 20000)]))
        seqs.append(_telo_read(rng, n, motif=motif, where=["left", "right", "mid"][i % 3],
                               tract=(min(n, 3 * len(motif)), max(min(n, 3 * len(motif)), min(n, 4000))),
                               exc=0.002 if i % 6 == 0 else 0.0))
    nt = _nt(jit=jit, **cfg)
    orow = oracle_rows(seqs, cfg["patterns"], tvr=cfg.get("tvr_patterns"), L=cfg["subseq_length"],
                       min_density=cfg["min_density"], right_edge=right, rc=cfg.get("rc", False))
    _check_both(nt, seqs, orow)
