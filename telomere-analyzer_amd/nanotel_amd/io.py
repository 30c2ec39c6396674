"""Host ingest and outputs of the NanoTel driver.

* `Reader`: FASTA/FASTQ(.gz) records in `nrec` chunks through the library's
  C++ reader (nt_reader_*; open_input_files + readDNAStringSet(nrec),
  NanoTel.R:2171-2216).  A chunk hands the read pointers straight to
  nt_analyze_host (no Python copies of the sequences).
* `format_double` / `write_summary_csv`: the summary.csv writer (write_csv,
  NanoTel.R:2430-2432).  readr 2.1.4's number formatting is not available
  offline: doubles are written as the shortest round-trip decimal, integral
  values without a fraction ("1", not "1.0"), NA as "NA" -- which reproduces
  Example_output/summary.csv byte for byte; the scientific switch for large
  integral doubles (readr may write 1e5 as "1e5") is `sci_threshold`.
* `r_as_character`: R's as.character()/toString() of a double (15
  significant digits, fixed unless the scientific form is narrower), used for
  the reads/<serial>.fasta.gz file names (NanoTel.R:1871).
* `write_fasta_gz`: writeXStringSet(..., compress = TRUE): 80-column FASTA.
"""
import ctypes
import gzip
import math
import os

import numpy as np

from ._lib import NanoTelError, lib


class Chunk:
    """One nt_reader_next() chunk; valid through the next next_chunk() call
    (or the next keep()-1 calls), not after."""

    def __init__(self, n, names_p, name_lens_p, seqs_p, seq_lens_p):
        self.n = int(n)
        self._names_p = names_p
        self._name_lens = np.ctypeslib.as_array(ctypes.cast(name_lens_p, ctypes.POINTER(ctypes.c_uint64)),
                                                shape=(self.n,)) if self.n else np.zeros(0, np.uint64)
        self.seq_ptrs = seqs_p.value or 0  # address of const char*[n]
        self.seq_lens_addr = seq_lens_p.value or 0
        self.lengths = np.ctypeslib.as_array(ctypes.cast(seq_lens_p, ctypes.POINTER(ctypes.c_uint64)),
                                             shape=(self.n,)) if self.n else np.zeros(0, np.uint64)
        self._np = ctypes.cast(names_p, ctypes.POINTER(ctypes.c_void_p))
        self._sp = ctypes.cast(seqs_p, ctypes.POINTER(ctypes.c_void_p))

    def name(self, i):
        return ctypes.string_at(self._np[i], int(self._name_lens[i])).decode("utf-8", "replace")

    def names(self):
        return [self.name(i) for i in range(self.n)]

    def seq(self, i):
        return ctypes.string_at(self._sp[i], int(self.lengths[i]))

    def name_pointers(self):
        """The names' host addresses and lengths (uint64 arrays)."""
        if not self.n:
            return np.zeros(0, np.uint64), np.zeros(0, np.uint64)
        return (np.ctypeslib.as_array((ctypes.c_uint64 * self.n).from_address(self._names_p.value)),
                self._name_lens)

    def pointers(self):
        """The sequences' host addresses (uint64 array, a view of the reader's)."""
        if not self.n:
            return np.zeros(0, np.uint64)
        return np.ctypeslib.as_array((ctypes.c_uint64 * self.n).from_address(self.seq_ptrs))


class SkippedChunk:
    """A chunk passed over with nt_reader_skip: the read lengths only (a rank
    of a multi-GPU run steps over the chunks other ranks scan)."""

    def __init__(self, n, seq_lens_p):
        self.n = int(n)
        self.lengths = np.ctypeslib.as_array(ctypes.cast(seq_lens_p, ctypes.POINTER(ctypes.c_uint64)),
                                             shape=(self.n,)) if self.n else np.zeros(0, np.uint64)


class Reader:
    def __init__(self, path, fmt="fastq"):
        if fmt not in ("fasta", "fastq"):
            raise ValueError("Format should be a string fastq or fasta")
        h = ctypes.c_void_p()
        rc = lib().nt_reader_open(os.fsencode(path), 0 if fmt == "fasta" else 1, ctypes.byref(h))
        if rc != 0:
            raise NanoTelError(rc, f"cannot open input {path!r}")
        self._h = h

    def files(self):
        L = lib()
        return [L.nt_reader_file(self._h, i).decode() for i in range(L.nt_reader_file_count(self._h))]

    def next_chunk(self, nrec):
        a, b, c, d = (ctypes.c_void_p() for _ in range(4))
        n = lib().nt_reader_next(self._h, int(nrec), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                 ctypes.byref(d))
        if n < 0:
            raise NanoTelError(int(n), lib().nt_reader_error(self._h).decode())
        if n == 0:
            return None
        return Chunk(n, a, b, c, d)

    def keep(self, chunks):
        """nt_reader_keep: the last `chunks` chunks stay valid (default 2)."""
        rc = lib().nt_reader_keep(self._h, int(chunks))
        if rc != 0:
            raise NanoTelError(int(rc), "nt_reader_keep")

    def skip_chunk(self, nrec):
        """The next nrec records without copying names or sequences
        (nt_reader_skip); None at the end."""
        d = ctypes.c_void_p()
        n = lib().nt_reader_skip(self._h, int(nrec), ctypes.byref(d))
        if n < 0:
            raise NanoTelError(int(n), lib().nt_reader_error(self._h).decode())
        if n == 0:
            return None
        return SkippedChunk(n, d)

    # ---- sharded ingest (nt_reader_layout / shard_range / count_files / plan / seek)

    def _check(self, rc, what):
        if rc < 0:
            raise NanoTelError(int(rc), f"{what}: {lib().nt_reader_error(self._h).decode()}")
        return rc

    def layout(self):
        """(all files plain, total bytes of the concatenated files)."""
        plain, tot = ctypes.c_int(), ctypes.c_uint64()
        self._check(lib().nt_reader_layout(self._h, ctypes.byref(plain), ctypes.byref(tot)), "layout")
        return bool(plain.value), int(tot.value)

    def shard_range(self, a, b):
        """Records starting in bytes [a, b) of the concatenated plain files:
        (their global byte offsets (uint64 array), first record start >= a,
        first record start >= b)."""
        first, nxt = ctypes.c_uint64(), ctypes.c_uint64()
        n = self._check(lib().nt_reader_shard_range(self._h, int(a), int(b), ctypes.byref(first),
                                                    ctypes.byref(nxt)), "shard_range")
        p = ctypes.c_void_p()
        lib().nt_reader_shard_positions(self._h, ctypes.byref(p))
        pos = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint64)), shape=(n,)).copy() \
            if n else np.zeros(0, np.uint64)
        return pos, int(first.value), int(nxt.value)

    def count_files(self, files):
        """Record counts of whole files (indices into files())."""
        f = np.ascontiguousarray(files, np.uint64)
        out = np.zeros(f.size, np.uint64)
        self._check(lib().nt_reader_count_files(self._h, f.ctypes.data, f.size, out.ctypes.data), "count_files")
        return out

    def plan(self, files):
        f = np.ascontiguousarray(files, np.uint64)
        self._check(lib().nt_reader_plan(self._h, f.ctypes.data, f.size), "plan")

    def seek_byte(self, pos):
        self._check(lib().nt_reader_seek(self._h, 0, int(pos), 0), "seek")

    def seek_record(self, file, skip):
        self._check(lib().nt_reader_seek(self._h, 1, int(file), int(skip)), "seek")

    def stats(self):
        """(bytes parsed, bytes inflated) by this reader so far."""
        out = (ctypes.c_uint64 * 2)()
        lib().nt_reader_stats(self._h, out)
        return int(out[0]), int(out[1])

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().nt_reader_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---------------------------------------------------------------- formatting

def format_double(x, sci_threshold=None):
    """write_csv formatting of a double: shortest round-trip digits; integral
    values without '.0'; NA/NaN -> "NA".  sci_threshold: integral values with
    |x| >= threshold and trailing zeros are written as "<digits>e<exp>"
    (readr/grisu style, parity unpinned); None keeps them fixed."""
    if x is None or (isinstance(x, float) and math.isnan(x)):
        return "NA"
    if math.isinf(x):
        return "Inf" if x > 0 else "-Inf"
    if x == int(x) and abs(x) < 1e15:
        i = int(x)
        if sci_threshold is not None and abs(i) >= sci_threshold and i % 10 == 0:
            s = str(abs(i)).rstrip("0")
            e = len(str(abs(i))) - len(s)
            return ("-" if i < 0 else "") + f"{s}e{e}"
        return str(i)
    r = repr(float(x))
    if "e" in r:
        m, e = r.split("e")
        r = f"{m}e{int(e)}"
    return r


def format_int(x):
    return "NA" if x is None else str(int(x))


def csv_field(s):
    """readr quoting: quote when the field holds the delimiter, a quote or a
    line break (quotes doubled)."""
    if any(c in s for c in ',"\n\r'):
        return '"' + s.replace('"', '""') + '"'
    return s


def r_as_character(x):
    """as.character(<double>) in R: up to 15 significant digits, fixed
    notation unless the scientific one is strictly narrower (scipen = 0)."""
    if math.isnan(x):
        return "NA"
    if math.isinf(x):
        return "Inf" if x > 0 else "-Inf"
    if x == 0:
        return "0"
    # minimal significant digits (<= 15) that reproduce x at 15 digits
    ref = float(f"{x:.15g}")
    for d in range(1, 16):
        if float(f"{x:.{d}g}") == ref:
            break
    sci = f"{x:.{d - 1}e}"
    mant, exp = sci.split("e")
    e = int(exp)
    sci_s = f"{mant}e{'-' if e < 0 else '+'}{abs(e):02d}"
    # fixed: digits after the point needed for d significant digits
    nd = max(0, d - 1 - e)
    fixed_s = f"{x:.{nd}f}"
    return fixed_s if len(fixed_s) <= len(sci_s) else sci_s


GZIP_LEVEL = 6  # R's gzfile() default (writeXStringSet compress = TRUE)


def write_fasta_gz_batch(paths, name_ptrs, name_lens, seq_ptrs, seq_lens, rc=False, level=None, threads=0):
    """reads/<serial>.fasta.gz of many reads in one library call
    (nt_write_fasta_gz: formatting, reverse complement and gzip in C++ on the
    host threads; the GIL is dropped).  name/seq: host addresses and lengths
    (the reader's chunk buffers, valid while the chunk is kept); rc: write the
    reverse complements (--rc).  level: NT_GZIP_LEVEL, else 6."""
    import numpy as np
    from ._lib import NanoTelError, lib
    n = len(paths)
    if n == 0:
        return
    if level is None:
        level = int(os.environ.get("NT_GZIP_LEVEL", GZIP_LEVEL))
    pb = [os.fsencode(p) for p in paths]
    parr = (ctypes.c_char_p * n)(*pb)
    arrs = [np.ascontiguousarray(a, np.uint64) for a in (name_ptrs, name_lens, seq_ptrs, seq_lens)]
    rcv = np.full(n, 1 if rc else 0, np.uint8)
    bad = ctypes.c_uint64(0)
    e = lib().nt_write_fasta_gz(ctypes.cast(parr, ctypes.c_void_p), arrs[0].ctypes.data, arrs[1].ctypes.data,
                                arrs[2].ctypes.data, arrs[3].ctypes.data, rcv.ctypes.data, n, int(level),
                                int(threads), ctypes.byref(bad))
    if e == -11:
        raise OSError(f"NanoTel: cannot write {paths[bad.value]}")
    if e != 0:
        raise NanoTelError(e, f"nt_write_fasta_gz ({paths[bad.value] if bad.value < n else ''})")


def write_fasta_gz(path, name, seq, width=80):
    """writeXStringSet(x, path, compress = TRUE): '>' name, 80-column lines,
    gzip at R's gzfile() default level 6.  One buffer, one zlib call (which
    drops the GIL, so the driver writes a chunk's reads on a thread pool)."""
    parts = [b">" + name.encode()]
    parts += [seq[i:i + width] for i in range(0, len(seq), width)]
    data = b"\n".join(parts) + b"\n"
    with open(path, "wb") as f:
        f.write(gzip.compress(data, compresslevel=6, mtime=0))
