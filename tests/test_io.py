"""Host ingest and output writers, CPU only.

* the C++ reader (nt_reader_*) against a plain Python parse, over FASTA,
  FASTQ, gzip, a nested directory stream and chunks that span files;
* the summary.csv writer: the oracle's rows for Example/sample.fasta
  (legacy mode) are written byte-identical to the committed
  Example_output/summary.csv;
* reads/<serial>.fasta.gz: the written reads equal Example_output/reads/*.fasta;
* R's as.character() of doubles for the file names.
"""
import gzip
import os

import numpy as np
import pytest

import _oracle as O
from _parity import oracle_rows
from nanotel_amd import assign_serials
from nanotel_amd.driver import chunk_rows, reverse_complement, write_summary_csv
from nanotel_amd.io import Reader, format_double, r_as_character, write_fasta_gz

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _chunks(path, fmt, nrec):
    out = []
    with Reader(path, fmt) as r:
        while True:
            ch = r.next_chunk(nrec)
            if ch is None:
                break
            out.append([(ch.name(i), ch.seq(i).decode()) for i in range(ch.n)])
    return out


def test_reader_fasta_matches_python_parse():
    names, seqs = O.read_fasta(os.path.join(GOLD, "sample.fasta"))
    got = _chunks(os.path.join(GOLD, "sample.fasta"), "fasta", 10000)
    assert len(got) == 1 and got[0] == list(zip(names, seqs))
    got3 = _chunks(os.path.join(GOLD, "sample.fasta"), "fasta", 3)
    assert [len(c) for c in got3] == [3, 1]
    assert sum(got3, []) == list(zip(names, seqs))


def _write_fastq(path, recs, gz=False, crlf=False):
    nl = "\r\n" if crlf else "\n"
    txt = "".join(f"@{n}{nl}{s}{nl}+{nl}{'I' * len(s)}{nl}" for n, s in recs)
    if gz:
        with gzip.open(path, "wt", newline="") as f:
            f.write(txt)
    else:
        with open(path, "w", newline="") as f:
            f.write(txt)


def test_reader_fastq_gz_directory_stream(tmp_path):
    rng = np.random.default_rng(3)

    def rec(i):
        return (f"read_{i} runid=abc ch={i}", "".join(rng.choice(list("ACGTN"), int(rng.integers(1, 300)))))

    recs = [rec(i) for i in range(17)]
    d = tmp_path / "in"
    (d / "sub").mkdir(parents=True)
    # sorted full paths: in/a.fastq, in/b.fastq.gz, in/sub/c.fastq
    _write_fastq(d / "a.fastq", recs[:5])
    _write_fastq(d / "b.fastq.gz", recs[5:12], gz=True, crlf=True)
    _write_fastq(d / "sub" / "c.fastq", recs[12:])
    with Reader(str(d), "fastq") as r:
        assert [os.path.relpath(p, d) for p in r.files()] == ["a.fastq", "b.fastq.gz", "sub/c.fastq"]
    for nrec in (1, 4, 7, 100):
        got = _chunks(str(d), "fastq", nrec)
        assert [len(c) for c in got] == [min(nrec, 17 - i) for i in range(0, 17, nrec)]
        assert sum(got, []) == recs


@pytest.mark.parametrize("threads", ["0", "1", "3", None])
def test_reader_run_directory_inflated_ahead(tmp_path, monkeypatch, threads):
    """A run directory of many fastq.gz parts (the multi-file input is inflated
    ahead on worker threads, NT_READER_THREADS; 0 = streamed): the same record
    stream for every thread count, chunks spanning parts, an empty part, a
    FASTA directory, and a broken part reported as an error."""
    if threads is None:
        monkeypatch.delenv("NT_READER_THREADS", raising=False)
    else:
        monkeypatch.setenv("NT_READER_THREADS", threads)
    rng = np.random.default_rng(5)
    recs = [(f"r{i} ch={i}", "".join(rng.choice(list("ACGT"), int(rng.integers(1, 2000))))) for i in range(60)]
    d = tmp_path / "run"
    d.mkdir()
    cuts = [0, 7, 7, 20, 33, 34, 50, 60]  # part 1 is empty
    for k in range(len(cuts) - 1):
        _write_fastq(d / f"part_{k:02d}.fastq.gz", recs[cuts[k]:cuts[k + 1]], gz=True)
    for nrec in (1, 6, 13, 1000):
        got = _chunks(str(d), "fastq", nrec)
        assert [len(c) for c in got] == [min(nrec, 60 - i) for i in range(0, 60, nrec)]
        assert sum(got, []) == recs
    fa = tmp_path / "fa"
    fa.mkdir()
    for k in range(3):
        with gzip.open(fa / f"p{k}.fa.gz", "wt") as f:
            for n, s in recs[20 * k:20 * k + 20]:
                f.write(f">{n}\n" + "\n".join(s[i:i + 80] for i in range(0, len(s), 80)) + "\n")
    assert sum(_chunks(str(fa), "fasta", 9), []) == recs
    (d / "part_99.fastq.gz").write_bytes(b"\x1f\x8b\x08\x00garbage")
    from nanotel_amd import NanoTelError
    with pytest.raises(NanoTelError):
        _chunks(str(d), "fastq", 1000)


def test_reader_parts_outgrow_the_isize_hint(tmp_path, monkeypatch):
    """Parts inflated whole start at the size their gzip trailer (ISIZE) gives:
    a multi-member part (bgzip-style, the trailer holds the LAST member's size)
    and a part of 40 MB must grow past it; the mappings go back to the reader's
    pool and serve the next reader in the process (read twice, same records)."""
    monkeypatch.setenv("NT_READER_THREADS", "2")
    rng = np.random.default_rng(9)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    recs = [(f"m{i}", acgt[rng.integers(0, 4, int(rng.integers(50, 5000)))].tobytes().decode()) for i in range(400)]
    d = tmp_path / "run"
    d.mkdir()
    with open(d / "part_00.fastq.gz", "wb") as f:  # 40 members, the last one tiny
        for k in range(40):
            sub = recs[10 * k:10 * k + 10] if k < 39 else recs[390:391]
            f.write(gzip.compress("".join(f"@{n}\n{s}\n+\n{'I' * len(s)}\n" for n, s in sub).encode()))
    big = [(f"b{i}", acgt[rng.integers(0, 4, 20000)].tobytes().decode()) for i in range(1000)]
    _write_fastq(d / "part_01.fastq.gz", big, gz=True)
    want = recs[:391] + big
    for _ in range(2):
        assert sum(_chunks(str(d), "fastq", 97), []) == want


def test_reader_skips_dot_files(tmp_path):
    """dir(recursive = TRUE) leaves out names starting with '.' (all.files =
    FALSE, NanoTel.R:2176): AppleDouble '._*' parts, .DS_Store and hidden
    directories are not part of the record stream or the file list."""
    rng = np.random.default_rng(11)
    recs = [(f"r{i}", "".join(rng.choice(list("ACGT"), int(rng.integers(5, 400))))) for i in range(9)]
    d = tmp_path / "run"
    (d / ".hidden").mkdir(parents=True)
    _write_fastq(d / "a.fastq.gz", recs[:4], gz=True)
    _write_fastq(d / "b.fastq", recs[4:])
    (d / "._a.fastq.gz").write_bytes(b"\x00\x05\x16\x07AppleDouble")
    (d / ".DS_Store").write_bytes(b"\x00\x00\x00\x01Bud1")
    _write_fastq(d / ".hidden" / "c.fastq", recs[:2])
    with Reader(str(d), "fastq") as r:
        assert [os.path.basename(p) for p in r.files()] == ["a.fastq.gz", "b.fastq"]
    assert sum(_chunks(str(d), "fastq", 4), []) == recs


@pytest.mark.parametrize("fmt", ["fasta", "fastq"])
def test_reader_skip_path_matches_next(tmp_path, fmt):
    """nt_reader_skip (ranks passing over other ranks' chunks) keeps the same
    record boundaries and lengths as nt_reader_next, interleaved with it,
    across wrapped FASTA lines, blank and ';' lines, CRLF, gzip and files."""
    rng = np.random.default_rng(12)
    recs = [(f"r{i} x", "".join(rng.choice(list("ACGTN"), int(rng.integers(0 if fmt == "fasta" else 1, 500)))))
            for i in range(40)]
    d = tmp_path / "in"
    (d / "sub").mkdir(parents=True)
    if fmt == "fastq":
        _write_fastq(d / "a.fastq", recs[:15], crlf=True)
        _write_fastq(d / "sub" / "b.fastq.gz", recs[15:], gz=True)
    else:
        with open(d / "a.fa", "w", newline="") as f:
            for n, s in recs[:15]:
                f.write(f">{n}\r\n" + "".join(s[i:i + 60] + "\r\n" for i in range(0, len(s), 60)) + "\n;c\n")
        with gzip.open(d / "sub" / "b.fa.gz", "wt") as f:
            for n, s in recs[15:]:
                f.write(f">{n}\n{s}\n")
    for nrec in (1, 3, 7, 100):
        with Reader(str(d), fmt) as r:
            k, seen = 0, []
            while True:
                ch = r.skip_chunk(nrec) if k % 2 else r.next_chunk(nrec)
                if ch is None:
                    break
                if k % 2 == 0:
                    assert [(ch.name(i), ch.seq(i).decode()) for i in range(ch.n)] == recs[len(seen):len(seen) + ch.n]
                seen += [int(x) for x in ch.lengths]
                k += 1
        assert seen == [len(s) for _, s in recs]


def test_reader_fasta_wrapped_blank_lines(tmp_path):
    p = tmp_path / "x.fa.gz"
    with gzip.open(p, "wt") as f:
        f.write(">r1 desc words\nACGT\nTTAG\n\nGG\n>r2\n\nNNNN\n>r3\n")
    assert _chunks(str(p), "fasta", 10) == [[("r1 desc words", "ACGTTTAGGG"), ("r2", "NNNN"), ("r3", "")]]


def test_reader_errors(tmp_path):
    from nanotel_amd import NanoTelError
    with pytest.raises(NanoTelError):
        Reader(str(tmp_path / "missing.fq"), "fastq")
    p = tmp_path / "bad.fq"
    p.write_text("not a fastq\n")
    with pytest.raises(NanoTelError):
        _chunks(str(p), "fastq", 10)


def test_r_as_character():
    cases = {1.0: "1", 2.0: "2", 100.0: "100", 1e5: "1e+05", 2e5: "2e+05", 123456.0: "123456",
             110000.0: "110000", 1e15: "1e+15", 0.1: "0.1", 1 / 3: "0.333333333333333",
             1234567.0: "1234567", 0.00001: "1e-05", 123.5: "123.5"}
    for x, s in cases.items():
        assert r_as_character(x) == s, (x, r_as_character(x), s)


def test_format_double():
    assert format_double(1.0) == "1"
    assert format_double(0.9919354838709677) == "0.9919354838709677"
    assert format_double(float("nan")) == "NA"
    assert format_double(100000.0) == "100000"
    assert format_double(100000.0, sci_threshold=1e5) == "1e5"


def test_summary_csv_from_oracle_rows_is_byte_identical():
    # the legacy (2023) code produced Example_output/summary.csv
    names, seqs = O.read_fasta(os.path.join(GOLD, "sample.fasta"))
    orows = oracle_rows(seqs, "TTAGGG", legacy=True, want_windows=False, want_hits=False)
    n = len(seqs)
    res = {"start": np.array([r["start"] + [-1] for r in orows]),
           "end": np.array([r["end"] + [-1] for r in orows]),
           "density": np.array([r["density"] + [0.0] for r in orows])}
    telo = np.array([r["telomeric"] for r in orows], np.uint8)
    ser, order, _, _ = assign_serials(telo)
    rows = chunk_rows(res, names, [len(s) for s in seqs], ser, order, 2)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"nt_summary_{os.getpid()}.csv")
    write_summary_csv(out, rows, tvr=False)
    assert open(out, "rb").read() == open(os.path.join(GOLD, "example_summary.csv"), "rb").read()
    os.remove(out)
    assert n == 4


def test_written_reads_match_reference(tmp_path):
    names, seqs = O.read_fasta(os.path.join(GOLD, "sample.fasta"))
    for i, (nm, s) in enumerate(zip(names, seqs), start=1):
        p = tmp_path / f"{r_as_character(float(i))}.fasta.gz"
        write_fasta_gz(str(p), nm, s.encode())
        assert gzip.open(p, "rb").read() == open(os.path.join(GOLD, "reads", f"{i}.fasta"), "rb").read()


def test_reverse_complement_matches_oracle():
    s = "ACGTNRYKMSWBDHVacgtn"
    assert reverse_complement(s.encode()).decode().upper() == O.reverse_complement(s).upper()


def _all_records(path, fmt):
    return sum(_chunks(path, fmt, 1000), [])


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_shard_ranges_find_every_record_start(tmp_path, fmt):
    """nt_reader_shard_range over N byte ranges of the concatenated plain files
    (a directory of three files, one empty): the ranks' record starts are the
    records of the unsharded reader, each exactly once, the chain check
    first(r) == next(r - 1) holds, and a seek to any start reads that record.
    FASTQ quality lines start with '@' and '+' (the resynchronisation must not
    take them for headers), CRLF line ends, blank lines between records, empty
    sequences; FASTA wraps at 60 with blank and ';' lines."""
    rng = np.random.default_rng(17)
    recs = [(f"r{i} x", "".join(rng.choice(list("ACGTN"), int(rng.integers(0 if i % 9 else 1, 400)))))
            for i in range(90)]
    d = tmp_path / "in"
    d.mkdir()
    if fmt == "fastq":
        recs = [(n, s or "A") for n, s in recs]

        def w(p, rs):
            with open(p, "w", newline="") as f:
                for i, (n, s) in enumerate(rs):
                    q = "".join(rng.choice(list("@+I#"), len(s)))
                    f.write(f"@{n}\r\n{s}\r\n+\r\n{q}\r\n" + ("\r\n" if i % 4 == 3 else ""))
    else:
        def w(p, rs):
            with open(p, "w") as f:
                for n, s in rs:
                    f.write(f">{n}\n" + "".join(s[i:i + 60] + "\n" for i in range(0, len(s), 60)) + "\n;c\n")
    w(d / "a", recs[:40])
    (d / "b").write_bytes(b"")
    w(d / "c", recs[40:])
    want = _all_records(str(d), fmt)
    assert want == recs
    for world in (1, 2, 3, 7, 40, 300):
        with Reader(str(d), fmt) as r:
            plain, S = r.layout()
            assert plain and S == sum(os.path.getsize(d / x) for x in "abc")
            pos, prev_next = [], None
            for k in range(world):
                p, first, nxt = r.shard_range(S * k // world, S * (k + 1) // world)
                if k:
                    assert first == prev_next, (world, k)
                assert all(S * k // world <= x < S * (k + 1) // world for x in p)
                prev_next = nxt
                pos += [int(x) for x in p]
            assert prev_next == S
            assert len(pos) == len(recs) and pos == sorted(pos)
        for i in (0, 39, 40, 41, 89):
            with Reader(str(d), fmt) as r:
                r.layout()
                r.seek_byte(pos[i])
                ch = r.next_chunk(3)
                assert [(ch.name(j), ch.seq(j).decode()) for j in range(ch.n)] == recs[i:i + 3]
    with Reader(str(d), fmt) as r:
        r.layout()
        r.seek_byte(S)
        assert r.next_chunk(5) is None


def test_count_files_plan_and_record_seek(tmp_path):
    """The run-directory form: per-file record counts (whole gzip parts on host
    threads), a plan that names only some parts, seeks to (part, record) --
    forward within the open part and into a later one -- and reads that
    continue across the planned parts."""
    rng = np.random.default_rng(23)
    recs = [(f"q{i}", "".join(rng.choice(list("ACGT"), int(rng.integers(1, 300))))) for i in range(50)]
    d = tmp_path / "run"
    d.mkdir()
    cuts = [0, 9, 9, 20, 31, 44, 50]
    for k in range(len(cuts) - 1):
        _write_fastq(d / f"p{k}.fastq.gz", recs[cuts[k]:cuts[k + 1]], gz=True)
    with Reader(str(d), "fastq") as r:
        assert r.layout()[0] is False
        assert list(r.count_files([0, 1, 2, 3, 4, 5])) == [9, 0, 11, 11, 13, 6]
        assert list(r.count_files([4])) == [13]
    with Reader(str(d), "fastq") as r:
        r.plan([0, 1, 2, 4, 5])
        r.seek_record(0, 3)
        ch = r.next_chunk(4)
        assert [ch.name(j) for j in range(ch.n)] == [n for n, _ in recs[3:7]]
        r.seek_record(0, 8)  # forward in the open part, then on across the empty part 1
        ch = r.next_chunk(3)
        assert [ch.name(j) for j in range(ch.n)] == [n for n, _ in recs[8:11]]
        r.seek_record(4, 12)  # part 3 is not in the plan: skipped
        ch = r.next_chunk(5)
        assert [ch.name(j) for j in range(ch.n)] == [n for n, _ in recs[43:48]]
        from nanotel_amd import NanoTelError
        with pytest.raises(NanoTelError):
            r.seek_record(3, 0)  # outside the plan
    with Reader(str(d), "fastq") as r:
        r.next_chunk(1)
        from nanotel_amd import NanoTelError
        with pytest.raises(NanoTelError):
            r.plan([0])  # only before the first read


def test_fastq_fast_path_matches_line_parser(tmp_path, monkeypatch):
    """The FASTQ fast path (mapped plain files: records indexed in parallel
    slices, single quality lines skipped unread) gives the line parser's
    records, chunks and errors: CRLF, blank lines between records, empty
    sequences, quality lines starting with '@' / '+', a wrapped quality, a
    quality longer than its sequence, a last record without a newline, a
    truncated quality at the end, and a malformed record after good ones."""
    rng = np.random.default_rng(29)
    recs = [(f"r{i} d", "".join(rng.choice(list("ACGTN"), int(rng.integers(0 if i % 7 else 1, 3000)))))
            for i in range(300)]

    def body(i, n, s, crlf):
        nl = "\r\n" if crlf else "\n"
        q = "".join(rng.choice(list("@+I#"), len(s)))
        if i % 50 == 7 and len(s) > 10:  # wrapped quality
            q = q[:5] + nl + q[5:]
        if i % 50 == 9:  # longer quality (accepted as the line parser does)
            q = q + "II"
        return f"@{n}{nl}{s}{nl}+{nl}{q}{nl}" + (nl if i % 11 == 3 else "")

    cases = {}
    cases["mixed"] = "".join(body(i, n, s, i % 3 == 0) for i, (n, s) in enumerate(recs))
    cases["no_final_newline"] = cases["mixed"].rstrip("\r\n")
    cases["truncated_quality"] = cases["mixed"] + "@tail\nACGTACGT\n+\nIII"
    cases["malformed"] = cases["mixed"] + "@bad\nACGT\nIIII\n"
    # a wrapped quality whose lines and newline add up to the sequence's
    # length (a line end at qe, another inside [c, qe)), and a CRLF quality one
    # letter short (its '\r' at qe - 1): the fast path must not take either as
    # one quality line; the line parser walks on into the next record
    tail = "@next\nACGTACGTAC\n+\nIIIIIIIIII\n"
    cases["wrapped_to_length"] = cases["mixed"] + "@w\nACGTACGTAC\n+\nIIII\nIIIII\n" + tail
    cases["crlf_short"] = cases["mixed"] + "@c\nACGTACGTAC\n+\nIIIIIIIII\r\n" + tail
    big = "".join(body(i, f"b{i}", "ACGT" * 2500, False) for i in range(4000))  # 40 MB: several threads
    cases["big"] = big
    cases["big_wrapped_to_length"] = big + "@w\nACGTACGTAC\n+\nIIII\nIIIII\n" + big[:200000]

    def read_all(path, nrec):
        out, err = [], None
        try:
            with Reader(str(path), "fastq") as r:
                while True:
                    ch = r.next_chunk(nrec)
                    if ch is None:
                        break
                    out.append([(ch.name(i), ch.seq(i)) for i in range(ch.n)])
        except Exception as ex:  # noqa: BLE001
            err = str(ex)
        return out, err

    for key, txt in cases.items():
        p = tmp_path / f"{key}.fastq"
        p.write_bytes(txt.encode())
        for nrec in (7, 1000):
            monkeypatch.setenv("NT_READER_FQ_FAST", "0")
            slow = read_all(p, nrec)
            monkeypatch.setenv("NT_READER_FQ_FAST", "1")
            fast = read_all(p, nrec)
            assert fast == slow, (key, nrec)
        rejected = ("malformed", "wrapped_to_length", "crlf_short", "big_wrapped_to_length")
        assert (slow[1] is not None) == (key in rejected), (key, slow[1])


def test_write_fasta_gz_batch_matches_python_writer(tmp_path):
    """nt_write_fasta_gz (reads/<serial>.fasta.gz in C++, NanoTel.R:1869-1873)
    against the Python writer: the same FASTA text (80-column lines, the
    reverse complement under --rc with Biostrings' IUPAC pairs), gzip with R's
    gzfile header (mtime 0, OS 3) at level 6; an unwritable path raises."""
    import ctypes
    import gzip as _gz
    import zlib
    from nanotel_amd.io import write_fasta_gz, write_fasta_gz_batch
    from nanotel_amd.driver import reverse_complement
    rng = np.random.default_rng(8)
    alpha = list(b"ACGTACGTACGTNRYKMSWBDHVacgtn-")
    seqs = [bytes(rng.choice(alpha, int(n)).tolist()) for n in
            [0, 1, 79, 80, 81, 159, 160, 161, 1000, 50000] + list(rng.integers(1, 5000, 20))]
    names = [f"read_{i} runid=abc ch={i}".encode() for i in range(len(seqs))]
    keep = [ctypes.create_string_buffer(x, len(x) or 1) for x in seqs + names]
    sp = np.array([ctypes.addressof(b) for b in keep[:len(seqs)]], np.uint64)
    npp = np.array([ctypes.addressof(b) for b in keep[len(seqs):]], np.uint64)
    sl = np.array([len(x) for x in seqs], np.uint64)
    nl = np.array([len(x) for x in names], np.uint64)
    for rc in (False, True):
        paths = [str(tmp_path / f"c{int(rc)}_{i}.fasta.gz") for i in range(len(seqs))]
        write_fasta_gz_batch(paths, npp, nl, sp, sl, rc=rc, threads=3)
        for i, p in enumerate(paths):
            ref = tmp_path / "ref.fasta.gz"
            write_fasta_gz(str(ref), names[i].decode(), reverse_complement(seqs[i]) if rc else seqs[i])
            got = open(p, "rb").read()
            assert _gz.decompress(got) == _gz.decompress(ref.read_bytes()), (rc, i)
            assert got[:10] == bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, 0, 3])
            text = _gz.decompress(got)
            co = zlib.compressobj(6, zlib.DEFLATED, -15)  # the raw stream: zlib's level 6, memLevel 8
            assert got[10:-8] == co.compress(text) + co.flush(), (rc, i)
    with pytest.raises(OSError):
        write_fasta_gz_batch([str(tmp_path / "no" / "dir" / "x.fasta.gz")], npp[:1], nl[:1], sp[:1], sl[:1])
