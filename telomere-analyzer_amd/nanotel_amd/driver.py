"""The NanoTel run driver over the MI355X hot path.

Mirrors run_future_worker_chuncks + the main script of NanoTel.R
(NanoTel.R:2171-2268, 2304-2433): stream the input in `nrec`-record chunks,
scan + call every chunk on the GPU (one nt_analyze_host per chunk, which
replaces the 8 forked search_patterns of NanoTel.R:2234-2258), assign serials
(A15), write reads/<serial>.fasta.gz for telomeric reads (NanoTel.R:1869-1873),
then <basename>_summary.csv, reads_ids.txt and log/run.log (NanoTel.R:2340-2433).

With torch.distributed initialised (one process per GPU), chunks are dealt
round-robin to ranks and the serials are fixed by one all_reduce (shard.py);
rank 0 writes the summary.  --use_filter runs the edge pre-filter on the GPU
(nt_filter_host, NanoTel.R:2083-2163, 2227-2232) and scans the kept reads
only.  --analysis writes the filtered/sorted summary and the results text
(analysis.py).  Every telomeric read gets the reference's three density plots
(plots.py: single_read_plots*/read<serial>.jpeg|eps) unless plot=False.
"""
import ctypes
import math
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import plots, shard
from .analysis import _keep_first, write_analysis
from .api import NanoTel, rows_columns, rows_csv
from .io import Reader, csv_field, format_double, format_int, r_as_character, write_fasta_gz, write_fasta_gz_batch
from .runlog import RunLog, r_time
from . import __version__

VERSION = "Telomere Analyzer  version v1.1.9-beta 2026-02-19"

BASE_COLUMNS = ["Serial", "sequence_ID", "sequence_length", "telo_density", "Telomere_start",
                "Telomere_end", "Telomere_length", "telo_density_mismatch", "Telomere_start_mismatch",
                "Telomere_end_mismatch", "Telomere_length_mismatch"]
TVR_COLUMNS = ["telo_density_mismatch_tvr", "Telomere_start_mismatch_tvr", "Telomere_end_mismatch_tvr",
               "Telomere_length_mismatch_tvr"]

_COMP = bytes.maketrans(b"ACGTMRWSYKVHDBNacgtmrwsykvhdbn", b"TGCAKYWSRMBDHVNtgcakywsrmbdhvn")


def reverse_complement(seq):
    """Biostrings reverseComplement on bytes (A14; the written reads are the
    RC'd reads under --rc, NanoTel.R:2219-2221)."""
    return seq.translate(_COMP)[::-1]


def columns(tvr):
    return BASE_COLUMNS + (TVR_COLUMNS if tvr else [])


def chunk_rows(res, names, lengths, serials, order, n_pass):
    """Summary rows of one chunk in the reference's row order (analyze_read's
    row, NanoTel.R:1920-1974) from the C-ABI's column builder
    (nt_rows_columns): per pass density/start/end/length, None (NA) when the
    pass found no telomere (start == -1)."""
    c = rows_columns(res, lengths, serials, order, n_pass)
    rows = []
    for i, j in enumerate(order):
        row = [float(c["serial"][i]), names[int(j)], int(c["length"][i])]
        for p in range(n_pass):
            if c["na"][p, i]:
                row += [None, None, None, None]
            else:
                row += [float(c["density"][p, i]), int(c["start"][p, i]), int(c["end"][p, i]),
                        int(c["width"][p, i])]
        rows.append(row)
    return rows


class ChunkRows:
    """One chunk's summary rows: their summary.csv and reads_ids.txt lines
    (nt_rows_csv, C++) and their columns (nt_rows_columns) -- what the ranks
    gather to rank 0 (pickled, in chunk order)."""

    def __init__(self, csv, ids, cols):
        self.csv, self.ids, self.cols = csv, ids, cols

    def __len__(self):
        return int(self.cols["serial"].size)


def _chunk_payload(rows, lengths):
    """What a rank sends rank 0 for one of its chunks, once its group round is
    done: the rows' summary.csv and reads_ids.txt bytes, and for run.log the
    value counts of the chunk's read lengths and of its rows' length / width
    columns (not the columns: rank 0 never holds a run's rows).  rows: a
    ChunkRows, or None when --use_filter kept no read of the chunk."""
    from .runlog import ValueCounts
    p = {"lengths": ValueCounts().add(lengths), "csv": b"", "ids": b"", "n": 0}
    if rows is not None and len(rows):
        c = rows.cols
        p.update(csv=rows.csv, ids=rows.ids, n=len(rows), row_len=ValueCounts().add(c["length"]))
        w = []
        for q in range(c["width"].shape[0]):
            v = c["width"][q].astype(np.float64)
            v[c["na"][q]] = np.nan
            w.append(ValueCounts().add(v))
        p["width"] = w
    return p


class SummarySink:
    """Rank 0's end of the row stream: every group round's chunks arrive in
    chunk order and are appended to <basename>_summary.csv and reads_ids.txt
    (written as *.partial, renamed when the run succeeds: the reference writes
    them at the end, NanoTel.R:2430-2433, so a failed run leaves none); run.log
    gets its summaries from value counts (len(), column()).  Memory: one group
    round's rows at a time, plus the rows --analysis keeps (those passing its
    first filter, NanoTel.R:2442-2443)."""

    def __init__(self, save_path, barcode, tvr, n_pass, analysis=False):
        from .runlog import ValueCounts
        self.n_pass = n_pass
        self.paths = (os.path.join(save_path, f"{barcode}_summary.csv"), os.path.join(save_path, "reads_ids.txt"))
        self._csv = open(self.paths[0] + ".partial", "wb")
        self._ids = open(self.paths[1] + ".partial", "wb")
        self._csv.write((",".join(columns(tvr)) + "\n").encode())  # write_csv's header
        self.lengths, self.row_len = ValueCounts(), ValueCounts()
        self.width = [ValueCounts() for _ in range(n_pass)]
        self.n_rows = 0
        self.kept = [] if analysis else None
        self.rounds, self.max_round_bytes, self._round = 0, 0, 0

    def end_round(self):
        """A group round's rows are in: the most row bytes one round brought."""
        self.rounds += 1
        self.max_round_bytes = max(self.max_round_bytes, self._round)
        self._round = 0

    def add(self, p):
        self._round += len(p["csv"]) + len(p["ids"])
        self._csv.write(p["csv"])
        self._ids.write(p["ids"])
        self.lengths.add(p["lengths"])
        if p["n"]:
            self.n_rows += p["n"]
            self.row_len.add(p["row_len"])
            for q in range(self.n_pass):
                self.width[q].add(p["width"][q])
            if self.kept is not None:
                self.kept += [r for r in _csv_rows(p["csv"], p["ids"], self.n_pass) if _keep_first(r)]

    def __len__(self):
        return self.n_rows

    def column(self, key, p=None):
        """run.log's columns as value counts: length (the rows' read lengths),
        width (pass p's telomere lengths, NA for a pass without one)."""
        return self.row_len if key == "length" else self.width[p]

    def rows(self):
        """The rows --analysis keeps (its first filter applied)."""
        return self.kept

    def finish(self, ok):
        self._csv.close()
        self._ids.close()
        for f in self.paths:
            if ok:
                os.replace(f + ".partial", f)
            else:
                os.remove(f + ".partial")


def _csv_rows(csv, ids, n_pass):
    """summary.csv lines back into rows [Serial, sequence_ID, sequence_length,
    (density, start, end, length) per pass], None for NA: --analysis reads
    what was written (the numbers round-trip: shortest round-trip doubles)."""
    names = ids.decode("utf-8", "replace").split("\n")
    out = []
    for i, line in enumerate(csv.decode("utf-8", "replace").split("\n")[:-1]):
        f = _split_csv_line(line)
        row = [float(f[0]), names[i], int(f[2])]
        for k in range(n_pass):
            d, a, e, w = f[3 + 4 * k:7 + 4 * k]
            row += [None] * 4 if d == "NA" else [float(d), int(a), int(e), int(w)]
        out.append(row)
    return out


def _split_csv_line(line):
    """Fields of one write_csv line (a sequence_ID may be quoted, with "" for ")."""
    import csv as _csv
    return next(_csv.reader([line]))


def format_row(row, sci_threshold=None):
    out = [format_double(row[0], sci_threshold), csv_field(row[1]), format_int(row[2])]
    for k in range(3, len(row), 4):
        d, s, e, w = row[k:k + 4]
        out += [format_double(d) if d is not None else "NA", format_int(s), format_int(e), format_int(w)]
    return ",".join(out)


def write_summary_csv(path, rows, tvr, sci_threshold=None):
    """write_csv(df_summary, <basename>_summary.csv) (NanoTel.R:2430-2432)."""
    with open(path, "w", newline="") as f:
        f.write(",".join(columns(tvr)) + "\n")
        for r in rows:
            f.write(format_row(r, sci_threshold) + "\n")


def _write_run_log(save_path, t0, input_path, files, patterns, tvr_patterns, rc, subseq_length, min_density,
                   lengths, rows, tvr):
    """<save_path>/log/run.log: the messages of NanoTel.R:2347-2427 and 2510-2514
    in logr's layout (runlog.py), in the order the reference prints them."""
    import torch
    log = RunLog(save_path, t0, versions=f"nanotel_amd {__version__}; torch {torch.__version__}; "
                                         f"HIP {getattr(torch.version, 'hip', None)}")
    log.print(VERSION)
    log.print(f"Work started at: {r_time(t0)}")
    log.print("############### The input argumetns for this run: ################")
    if rc:
        log.print("Reverse complement was applied on the input reads.")
    log.print(f"The patterns to search: {patterns}")
    log.print(f"The sub-sequence length  is: {subseq_length}")
    log.print(f"The minimal density for a telomeric subseq: {r_as_character(float(min_density))}")
    if tvr:
        log.print(f"Additional Telomere variant repeats patterns were added: {tvr_patterns}")
    log.print("##################################################################")
    log.print("The input files:")
    for p in (files if os.path.isdir(input_path) else [input_path]):
        log.print(p)
    n = lengths.n
    log.print(f"Total reads in sample: {n}")
    log.print("Summary statistics of the sample reads length:")
    log.summary(lengths)
    log.print(f"Number of reads which identified as Telomeric: {len(rows)}")
    pct = r_as_character(round(100 * len(rows) / n, 2)) if n else "NaN"
    log.print(f"% of total reads: {pct}%")
    log.print("Summary statistics for the Telomeric reads:")
    log.print("reads length:")
    log.summary(rows.column("length"))
    log.print("Telomere length:")
    log.summary(rows.column("width", 0))
    log.print("Telomere length with 1 mismatch allowed:")
    log.summary(rows.column("width", 1))
    if tvr:
        log.print("Telomere length with 1 mismatch allowed + tvr patterns.:")
        log.summary(rows.column("width", 2))
    log.print(f"Work ended at: {r_time()}")
    log.close()  # log_close(footer = FALSE)


def _peak_rss_kb():
    """This process's peak resident set (VmHWM: per address space, so a
    spawned rank reports its own, not its parent's as ru_maxrss would)."""
    try:
        with open("/proc/self/status") as f:
            for line in f:
                if line.startswith("VmHWM:"):
                    return int(line.split()[1])
    except OSError:
        pass
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss


def _write_read(path, name, seq, rc):
    write_fasta_gz(path, name, reverse_complement(seq) if rc else seq)


def _plot_pool():
    """Spawned (not forked: this process holds a HIP context) plot workers,
    one per host core of the GPU's share, at most 16; they import only
    plots.py and never touch the GPU."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    return ProcessPoolExecutor(min(16, os.cpu_count() or 1), mp_context=mp.get_context("spawn"))


def _plot_rows(res, order):
    """The rows of `order` that get plots (reads with at least one window)."""
    return [int(j) for j in order if int(res["n_windows"][int(j)]) != 0]


def _plot_jobs(nt, res, order, lens, ser, save_path):
    """Arguments of plots.write_read_plots for every row of a chunk (the three
    single-read plots of analyze_read, NanoTel.R:1876-1912)."""
    jobs = []
    for j in order:
        j = int(j)
        n = int(lens[j])
        if int(res["n_windows"][j]) == 0:
            continue
        tabs = [plots.window_table(n, nt.subseq_length, nt.window_counts(res, j, p)) for p in range(nt.n_pass)]
        se = [(int(res["start"][j, p]), int(res["end"][j, p])) for p in range(nt.n_pass)]
        kw = {}
        if nt.n_pass == 3:
            kw = dict(subs_tvr=tabs[2], tvr_start=se[2][0], tvr_end=se[2][1])
        jobs.append(((save_path, r_as_character(float(ser[j])), n, tabs[0], tabs[1], se[0][0], se[0][1],
                      se[1][0], se[1][1]), kw))
    return jobs


# One device call covers several of the reference's nrec-record chunks (they
# stay the units of serials and rows): the calling kernel specialised for the
# patterns runs on batches of >= 65,536 reads (nt_host.cpp), so a rank's block
# of a group is ceil(65536 / nrec) chunks, at most kGroupRounds, scanned in
# calls of at most kGroupBases bases.
kCallReads = 65536
kGroupRounds = 16
kGroupBases = 4_000_000_000


def _group_rounds(nrec):
    """Chunks per block (NT_GROUP_CHUNKS overrides: small blocks spread small
    test inputs over the ranks)."""
    if os.environ.get("NT_GROUP_CHUNKS"):
        return max(1, int(os.environ["NT_GROUP_CHUNKS"]))
    return max(1, min(kGroupRounds, -(-kCallReads // max(1, nrec))))


class _View(dict):
    """One chunk's slice of a grouped result (window-count offsets stay global)."""


class _LazyNames(dict):
    """names[j] of a chunk's rows, decoded from the reader's buffer on first use."""

    def __init__(self, name_of):
        super().__init__()
        self._of = name_of

    def __missing__(self, j):
        v = self[j] = self._of(int(j))
        return v


def _scan_group(nt, chunks, use_filter, log, want_windows=False):
    """Scan + call the reads of several chunks in as few device calls as
    possible -- one per kGroupBases bases (after --use_filter, per chunk, when
    on).  Returns per chunk (rel_serials, row_order, rel_max, result view,
    name_of(j), lengths) over the reads that were scanned (the view holds the
    reads' name and sequence addresses in the reader's chunk buffers); rel_max
    is shard.SKIPPED for a chunk that --use_filter emptied."""
    parts = []
    for ch in chunks:
        idx = np.arange(ch.n)
        if use_filter:
            idx = np.flatnonzero(nt.filter_chunk(ch))
            if idx.size == 0:
                log("No read have passed the filteration at run_with_rc_and_filter!")
        parts.append((ch, idx))
    calls, cur, bases = [], [], 0  # consecutive chunks, at most kGroupBases bases a call (at least one chunk)
    for ch, idx in parts:
        b = int(ch.lengths[idx].sum()) if idx.size else 0
        if cur and bases + b > kGroupBases:
            calls.append(cur)
            cur, bases = [], 0
        cur.append((ch, idx))
        bases += b
    if cur:
        calls.append(cur)
    out = []
    for call in calls:
        ptrs = np.concatenate([ch.pointers()[idx] for ch, idx in call])
        lens = np.concatenate([ch.lengths[idx] for ch, idx in call])
        res = nt.analyze_pointers(ptrs, lens, want_windows=want_windows) if ptrs.size else None
        a = 0
        for ch, idx in call:
            b = a + idx.size
            if idx.size == 0:
                out.append((None, np.zeros(0, np.int64), shard.SKIPPED, None, None, lens[:0]))
                continue
            v = _View({k: res[k][a:b] for k in ("start", "end", "density", "flags", "width", "telomeric")
                       if k in res})
            if want_windows:
                v["win_off"], v["n_windows"], v["win_counts"] = res["win_off"][a:b], res["n_windows"][a:b], \
                    res["win_counts"]
            np_, nl_ = ch.name_pointers()
            v["name_ptrs"], v["name_lens"] = np_[idx], nl_[idx]
            v["seq_ptrs"] = ch.pointers()[idx]
            rel, order, rmax = shard.chunk_relative(v["telomeric"])
            name_of = (lambda c, ix: (lambda j: c.name(int(ix[j]))))(ch, idx)
            out.append((rel, order, rmax, v, name_of, lens[a:b]))
            a = b
    return out


class _Prefetch:
    """The next chunk is read on a worker thread while the current ones are
    scanned (the C++ reader keeps the last chunks valid, nt_reader_keep, and
    ctypes drops the GIL).

    Sharded ingest (plan.sharded): only this rank's chunks are read, in order,
    with one seek at the start of each of its blocks.  Otherwise the whole
    stream is read and the chunks this rank does not scan are passed over with
    the reader's count-only skip path (record boundaries and lengths, no copies)."""

    def __init__(self, rdr, nrec, own=lambda k: True, plan=None, g=1, world=1, rank=0):
        self._rdr, self._nrec, self._own = rdr, nrec, own
        self._plan = plan if plan is not None and plan.sharded else None
        self._k = 0
        if self._plan is not None:
            n = self._plan.n_chunks
            G = g * world
            self._seq = [k for t0 in range(0, n, G) for k in range(t0 + rank * g, min(t0 + (rank + 1) * g, n))]
            self._i = 0
            self._g = g
            blocks = [(k, min(k + g, n)) for k in self._seq[::g]]
            files = sorted({f for k0, k1 in blocks for f in range(*self._span(k0, k1))})
            rdr.plan(files)
        self._ex = ThreadPoolExecutor(1)
        self._f = self._ex.submit(self._read)

    def _span(self, k0, k1):
        f0, f1 = self._plan.files_of(k0, k1, self._nrec)
        return f0, f1 + 1

    def _read(self):
        if self._plan is not None:
            if self._i >= len(self._seq):
                return None
            k = self._seq[self._i]
            self._i += 1
            if k % self._g == 0:  # a block's first chunk
                self._plan.seek(self._rdr, k)
            ch = self._rdr.next_chunk(self._nrec)
            want = self._plan.chunk_len(k, self._nrec)
            if ch is None or ch.n != want:
                raise RuntimeError(f"NanoTel: sharded ingest read {0 if ch is None else ch.n} records "
                                   f"of chunk {k + 1}, expected {want}")
            return ch
        k = self._k
        self._k += 1
        return self._rdr.next_chunk(self._nrec) if self._own(k) else self._rdr.skip_chunk(self._nrec)

    def next_chunk(self):
        if self._f is None:
            return None
        ch = self._f.result()
        self._f = self._ex.submit(self._read) if ch is not None else None
        return ch

    def close(self):
        if self._f is not None:
            self._f.cancel()
            try:
                self._f.result()
            except Exception:  # noqa: BLE001 -- a read error after the last chunk used
                pass
            self._f = None
        self._ex.shutdown()


def _targets(ser, order):
    """Rows of a chunk whose reads/plots are written now, and the last row with
    a -Inf serial.  Once a chunk without rows leaves serial_start at -Inf
    (max(numeric(0)) + 1, NanoTel.R:2258) every later row is -Inf and all of
    them name reads/-Inf.fasta.gz and read-Inf.*: concurrent writers would
    interleave there, so those rows are held back and only the last one in
    stream order is written, at the end of the run (the reference keeps the
    last-written read)."""
    now, last_inf = [], None
    for j in order:
        j = int(j)
        if math.isinf(float(ser[j])):
            last_inf = j
        else:
            now.append(j)
    return now, last_inf


def run(input_path, save_path, patterns, fmt="fastq", nrec=10000, rc=False, min_density=0.6,
        subseq_length=100, check_right_edge=False, tvr_patterns=None, legacy_no_ext=False,
        device=0, write_reads=True, sci_threshold=None, use_filter=False, analysis=False,
        plot=True, plot_jpeg=True, log=print, stats=None):
    """Run the pipeline; returns (the run's SummarySink: len() = rows, the
    run.log columns as value counts; the read lengths' value counts) on rank
    0, (None, None) elsewhere.  stats: a dict filled with the run's phase
    times (seconds)."""
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank() if dist_on else 0
    world = dist.get_world_size() if dist_on else 1
    # RCCL (backend "nccl") reduces device tensors, gloo host ones: every
    # collective below runs on coll_dev
    coll_dev = shard.collective_device() if dist_on else None
    os.makedirs(save_path, exist_ok=True)
    reads_dir = os.path.join(save_path, "reads")
    os.makedirs(reads_dir, exist_ok=True)
    if plot:  # create_dirs (NanoTel.R:1978-1996)
        os.makedirs(os.path.join(save_path, "single_read_plots"), exist_ok=True)
        os.makedirs(os.path.join(save_path, "single_read_plots_adj"), exist_ok=True)
    nt = NanoTel(patterns=patterns, tvr_patterns=tvr_patterns, subseq_length=subseq_length,
                 min_density=min_density, check_right_edge=check_right_edge, rc=rc,
                 legacy_no_ext=legacy_no_ext, device=device)
    tvr = tvr_patterns is not None
    rdr = Reader(input_path, fmt)
    files = rdr.files()
    g = _group_rounds(nrec)  # chunks per block: a rank's chunks of one group
    G = g * world            # chunks per group (one collective per group)
    rdr.keep(g + 2)          # this rank's chunks of a group stay valid, plus the one read ahead
    t0 = time.time()
    tm = {"setup": 0.0, "index": 0.0, "read_wait": 0.0, "scan": 0.0, "rows_files": 0.0, "collectives": 0.0}
    # sharded ingest: the ranks find the chunk starts together (each indexes
    # 1/N of the input) and each reads only its own chunks; otherwise every
    # rank reads the stream and passes over the others' chunks
    ti = time.perf_counter()
    try:
        plan = shard.ingest_plan(rdr, nrec, rank, world, device=coll_dev, log=log) if dist_on \
            else shard.IngestPlan(reason="one rank")
    except Exception:  # every rank raises here (the plan's exchange carries the error flag)
        rdr.close()
        nt.close()
        raise
    tm["index"] = time.perf_counter() - ti
    # chunk k of the stream is scanned by rank (k // g) % world: groups of
    # `world` blocks of g chunks
    src = _Prefetch(rdr, nrec, own=lambda c: shard.block_owner(c, g, world) == rank, plan=plan, g=g,
                    world=world, rank=rank)
    writers = ThreadPoolExecutor(min(16, os.cpu_count() or 1)) if (write_reads or plot) else None
    plotters = None  # worker processes for the plots of large chunks (Python drawing holds the GIL)
    pending = []
    barcode = os.path.basename(os.path.normpath(os.path.abspath(input_path)))
    sink = SummarySink(save_path, barcode, tvr, nt.n_pass, analysis) if rank == 0 else None
    held = None  # (chunk, read args, plot job) of this rank's last -Inf row (see _targets)
    k = 0  # global chunk index of the group's first chunk
    s_next, m_run = 1.0, shard.NEG_INF  # serial_start of the next chunk, running max(Serial)
    failure = None
    # groups of G chunks: rank r scans block r of each group (its device calls,
    # split at kGroupBases bases); one all_reduce per group fixes the
    # serial_starts (and carries an error flag, so that a rank that fails stops
    # every rank at the same group instead of leaving them blocked in the next
    # collective).  The ranks agree on the groups: the plan's chunk count, or
    # (unsharded) the same stream read by every rank.
    tm["setup"] = time.time() - t0 - tm["index"]
    while True:
        own = []  # (chunk's place in the group, chunk)
        n_grp, ended = 0, False
        try:
            if plan.sharded:
                n_grp = min(G, plan.n_chunks - k)
                ended = k + G >= plan.n_chunks
                for c in range(k + rank * g, min(k + (rank + 1) * g, plan.n_chunks)):
                    tr = time.perf_counter()
                    ch = src.next_chunk()
                    tm["read_wait"] += time.perf_counter() - tr
                    own.append((c - k, ch))
            else:
                for pos in range(G):
                    tr = time.perf_counter()
                    ch = src.next_chunk()
                    tm["read_wait"] += time.perf_counter() - tr
                    if ch is None:
                        ended = True
                        break
                    if shard.block_owner(k + pos, g, world) == rank:
                        own.append((pos, ch))
                    n_grp += 1
            for pos, ch in own:
                log(f"processing chunk {k + pos + 1} ...")
            ts = time.perf_counter()
            scanned = _scan_group(nt, [ch for _, ch in own], use_filter, log, want_windows=plot)
            tm["scan"] += time.perf_counter() - ts
        except Exception as ex:  # noqa: BLE001 -- re-raised after the collective
            failure, scanned = ex, []
        local = {own[i][0]: scanned[i][2] for i in range(len(scanned))}
        tc = time.perf_counter()
        maxima, failed = shard.exchange_rel_max(local, G, device=coll_dev, failed=failure is not None)
        tm["collectives"] += time.perf_counter() - tc
        if failed:
            break
        starts = np.empty(n_grp, np.float64)
        for r in range(n_grp):  # the reference's recurrence, chunk by chunk
            starts[r], s_next, m_run = shard.advance(s_next, m_run, float(maxima[r]))
        tw = time.perf_counter()
        payload = {}  # this group's chunks, for rank 0
        try:
            for (pos, ch), (rel, order, _, res, name_of, lens) in zip(own, scanned):
                if res is None:  # --use_filter kept no read of this chunk
                    payload[k + pos] = _chunk_payload(None, ch.lengths)
                    continue
                ser = shard.assign_chunk_serials(rel, starts[pos])
                cols = rows_columns(res, lens, ser, order, nt.n_pass)
                csv, ids = rows_csv(cols, res["name_ptrs"][order], res["name_lens"][order], nt.n_pass,
                                    sci_threshold)
                payload[k + pos] = _chunk_payload(ChunkRows(csv, ids, cols), ch.lengths)
                names = _LazyNames(name_of)
                for f in pending:  # the previous chunk's files (errors surface here)
                    f.result()
                pending = []
                now, last_inf = _targets(ser, order)
                jobs = _plot_jobs(nt, res, order, lens, ser, save_path) if plot else []
                job_of = {int(j): jb for j, jb in zip(_plot_rows(res, order), jobs)} if plot else {}
                if last_inf is not None:
                    seq = ctypes.string_at(int(res["seq_ptrs"][last_inf]), int(lens[last_inf])) if write_reads else None
                    held = (k + pos, (names[last_inf], seq, rc), job_of.get(last_inf))
                if write_reads and now:  # one library call a chunk: formatting + gzip on the host threads
                    sel = np.asarray(now, np.int64)
                    paths = [os.path.join(reads_dir, f"{r_as_character(float(ser[j]))}.fasta.gz") for j in now]
                    pending.append(writers.submit(write_fasta_gz_batch, paths, res["name_ptrs"][sel],
                                                  res["name_lens"][sel], res["seq_ptrs"][sel], lens[sel], rc))
                if plot:
                    jobs = [job_of[j] for j in now if j in job_of]
                    if len(jobs) >= 64 and plotters is None:
                        plotters = _plot_pool()
                    pool = plotters if len(jobs) >= 64 else writers
                    pending += [pool.submit(plots.write_read_plots, *a, jpeg=plot_jpeg, **kw) for a, kw in jobs]
        except Exception as ex:  # noqa: BLE001
            failure = ex
        tm["rows_files"] += time.perf_counter() - tw
        # the group's rows to rank 0 now, in chunk order (every rank joins, a
        # failed one with what it has: the next round's exchange stops them all)
        tc = time.perf_counter()
        parts = shard.gather_chunks(payload)
        del payload
        if sink is not None:
            for p in parts:
                sink.add(p)
            sink.end_round()
        tm["collectives"] += time.perf_counter() - tc
        k += n_grp
        if ended:
            break
    try:
        for f in pending:
            f.result()
        # the last -Inf row of the whole stream: written by the rank that holds it
        last = shard.max_over_ranks(held[0] if held else -1, device=coll_dev)
        if held is not None and held[0] == last:
            name, seq, rcf = held[1]
            if write_reads:
                _write_read(os.path.join(reads_dir, "-Inf.fasta.gz"), name, seq, rcf)
            if plot and held[2] is not None:
                a, kw = held[2]
                plots.write_read_plots(*a, jpeg=plot_jpeg, **kw)
    except Exception as ex:  # noqa: BLE001
        failure = failure or ex
    if writers is not None:
        writers.shutdown()
    if plotters is not None:
        plotters.shutdown()
    src.close()
    if shard.any_rank(failure is not None, device=coll_dev):
        rdr.close()
        nt.close()
        if sink is not None:
            sink.finish(False)
        if failure is not None:
            raise failure
        raise RuntimeError("NanoTel: another rank failed (see its error)")
    t_end = time.time()
    if stats is not None:
        stats.update(tm)
        stats["ingest"] = plan.mode or "unsharded"
        stats["ingest_reason"] = plan.reason
        stats["bytes_parsed"], stats["bytes_inflated"] = rdr.stats()
        stats.update({"host_" + k: v for k, v in nt.host_times().items()} if hasattr(nt, "host_times") else {})
        stats["groups_rounds"] = g
        stats["peak_rss_kb"] = _peak_rss_kb()
        if sink is not None:
            stats["rows_rounds"], stats["rows_max_round_bytes"] = sink.rounds, sink.max_round_bytes
    tc = time.time()
    rdr.close()
    tc2 = time.time()
    nt.close()
    if stats is not None:  # (inside "final")
        stats["final_close_reader"] = tc2 - tc
        stats["final_close_ctx"] = time.time() - tc2
    if rank != 0:
        return None, None
    # write_csv / write_lines (NanoTel.R:2430-2433): streamed, complete now
    sink.finish(True)
    if analysis:  # --analysis post-processing (NanoTel.R:2437-2508)
        write_analysis(save_path, barcode, sink.rows(), columns(tvr), format_row, sci_threshold)
    _write_run_log(save_path, t0, input_path, files, patterns, tvr_patterns, rc, subseq_length, min_density,
                   sink.lengths, sink, tvr)
    if stats is not None:
        stats["final"] = time.time() - t_end
        stats["total"] = time.time() - t0
    return sink, sink.lengths
