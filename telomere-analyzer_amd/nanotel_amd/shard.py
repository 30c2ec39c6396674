"""Multi-GPU sharding of NanoTel's chunk stream.

The reference reads its input as a stream of `nrec`-record chunks
(run_future_worker_chuncks, NanoTel.R:2171-2268); reads are independent, so
chunks are dealt round-robin to ranks (one process per GPU) and scanned with no
collective on the data path.  The only cross-chunk dependency of the output is
the Serial column (A15):

  * inside a chunk, serials are offsets from the chunk's serial_start that
    depend only on that chunk's telomeric flags (the 8-way split,
    NanoTel.R:2234-2254) -- nt_assign_serials with serial_start = 0;
  * serial_start(chunk k+1) = max(Serial of chunks <= k) + 1, which is -Inf
    while no row exists yet (max(numeric(0)), NanoTel.R:2258).

So each rank publishes, per chunk it owns, the chunk's largest relative serial
(-Inf for a chunk without rows); one all-reduce(MAX) of that n_chunks vector
(8 bytes per chunk; every other rank contributes -Inf) gives every rank all of
them, and the serial_starts follow from a sequential scan that reproduces the
reference's fp64 arithmetic exactly.  Rows then go to rank 0 in chunk order.
"""
import os

import numpy as np

from .api import assign_serials

NEG_INF = float("-inf")


def owner(chunk, world):
    """Rank that scans chunk `chunk` (round-robin)."""
    return chunk % world


def local_chunks(n_chunks, rank, world):
    return list(range(rank, n_chunks, world))


def chunk_relative(is_telo):
    """Serials of one chunk relative to serial_start = 0.

    Returns (rel_serials (n,) float64, NaN for non-telomeric reads;
    row_order (rows,) int64 -- the reference's group-major row order;
    rel_max float: largest relative serial, -Inf without rows)."""
    ser, order, _, mx = assign_serials(is_telo, serial_start=0.0, max_serial=NEG_INF)
    return ser, order, mx


# rel_max of a chunk that --use_filter emptied: the reference `next`s past it
# (NanoTel.R:2229-2231), so serial_start is not recomputed.  Relative maxima
# are -Inf or >= 0, so -1 survives the all_reduce(MAX) with -Inf elsewhere.
SKIPPED = -1.0


def advance(s, m, rel_max):
    """One chunk of the reference's serial recurrence: returns (this chunk's
    serial_start, next serial_start, running max(Serial)).
    M = max(M, S + rel_max); S' = M + 1 (NanoTel.R:2258), same fp64 operations;
    a SKIPPED chunk leaves S and M unchanged."""
    if rel_max == SKIPPED:
        return s, s, m
    v = s + rel_max
    if v > m:
        m = v
    return s, m + 1.0, m


def serial_starts(rel_max):
    """serial_start of every chunk from the chunks' relative maxima, in chunk
    order: S_0 = 1; M_k = max(M_{k-1}, S_k + rel_max_k); S_{k+1} = M_k + 1."""
    starts = np.empty(len(rel_max), np.float64)
    s, m = 1.0, NEG_INF
    for k, r in enumerate(rel_max):
        starts[k], s, m = advance(s, m, float(r))
    return starts


def _collective(group=None):
    """Whether the collectives run: a process group of more than one rank, or
    of one rank with NT_DIST_FORCE=1 (exercises the RCCL path on one GPU)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return False
    return dist.get_world_size(group) > 1 or os.environ.get("NT_DIST_FORCE") == "1"


def exchange_rel_max(local, n_chunks, group=None, device=None, failed=False):
    """All ranks' per-chunk relative maxima: local = {chunk: rel_max} for the
    chunks this rank owns.  One all_reduce(MAX) over an n_chunks float64
    vector plus one error flag (gloo on CPU tensors, RCCL on device tensors).
    Returns (maxima, any rank failed): a rank that failed publishes the flag
    so that every rank stops at this collective."""
    import torch
    import torch.distributed as dist
    t = torch.full((n_chunks + 1,), NEG_INF, dtype=torch.float64,
                   device=device if device is not None else "cpu")
    for k, v in local.items():
        t[k] = v
    t[n_chunks] = 1.0 if failed else 0.0
    if _collective(group):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    a = t.cpu().numpy()
    return a[:n_chunks], bool(a[n_chunks] > 0.0)


def collective_device(group=None):
    """Where this process group's collectives reduce: a device tensor for RCCL
    (backend "nccl" -- it refuses host tensors), None (host) for gloo."""
    import torch
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return None


def max_over_ranks(x, group=None, device=None):
    """max over the ranks of an integer (one all_reduce; on `device` for
    RCCL, see collective_device)."""
    import torch
    import torch.distributed as dist
    if not _collective(group):
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64, device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def any_rank(flag, group=None, device=None):
    """True on every rank if `flag` is true on any."""
    return max_over_ranks(1 if flag else 0, group, device) > 0


def assign_chunk_serials(rel, start):
    """Absolute serials of one chunk: start + relative offsets (NaN stays)."""
    return start + rel


def gather_rows(local_rows, group=None, dst=0):
    """Gather {chunk: rows} from every rank to dst; returns the rows
    concatenated in chunk order on dst (None elsewhere)."""
    import torch.distributed as dist
    if not _collective(group):
        return [r for _, rows in sorted(local_rows.items()) for r in rows]
    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(local_rows, out, dst=dst, group=group)
    if out is None:
        return None
    merged = {}
    for part in out:
        merged.update(part)
    return [r for _, rows in sorted(merged.items()) for r in rows]


def gather_chunks(local, group=None, dst=0):
    """Gather {chunk: value} from every rank to dst; returns the values in
    chunk order on dst (None elsewhere)."""
    import torch.distributed as dist
    if not _collective(group):
        return [v for _, v in sorted(local.items())]
    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(local, out, dst=dst, group=group)
    if out is None:
        return None
    merged = {}
    for part in out:
        merged.update(part)
    return [v for _, v in sorted(merged.items())]


def block_owner(chunk, g, world):
    """Rank that scans chunk `chunk`: blocks of g consecutive chunks dealt
    round-robin (group t = chunks [t g world, (t+1) g world); rank r owns the
    r-th block of every group), so a rank's chunks of a group are one
    contiguous run of records and a sharded reader seeks once per group."""
    return (chunk // g) % world


class IngestPlan:
    """Where every nrec-record chunk of the input starts, found by the ranks
    together from 1/N of the input each (nt_reader_shard_range /
    nt_reader_count_files), so that each rank reads only the chunks it scans
    (DESIGN.md §7).  Chunk k is still records [k nrec, (k+1) nrec) of the
    whole stream (run_future_worker_chuncks, NanoTel.R:2207-2254), so the
    serials (A15) do not change.

    mode "range": all files plain -- chunk starts are byte offsets of the
    concatenated files; "files": gzip parts -- chunk starts are (file, record
    within the file); None: unsharded (one rank, a single gzip stream, or a
    failed resynchronisation): every rank reads the whole stream and passes
    over the chunks it does not scan (nt_reader_skip)."""

    def __init__(self, mode=None, n_chunks=None, total=None, starts=None, file_first=None, reason=""):
        self.mode, self.n_chunks, self.total = mode, n_chunks, total
        self.starts = starts          # range: (n_chunks,) byte offsets; files: (n_chunks, 2) (file, skip)
        self.file_first = file_first  # range: files' first byte offsets; files: files' first record index
        self.reason = reason
        self.index_s = 0.0

    @property
    def sharded(self):
        return self.mode is not None

    def chunk_len(self, k, nrec):
        return min(nrec, self.total - k * nrec)

    def seek(self, rdr, k):
        """Move the reader to chunk k's first record."""
        if self.mode == "range":
            rdr.seek_byte(int(self.starts[k]))
        else:
            rdr.seek_record(int(self.starts[k, 0]), int(self.starts[k, 1]))

    def files_of(self, k0, k1, nrec):
        """The files holding records of chunks [k0, k1) (an inclusive index range)."""
        if self.mode == "range":
            a = int(self.starts[k0])
            b = int(self.starts[k1]) - 1 if k1 < self.n_chunks else int(self.file_first[-1]) - 1
            f0 = int(np.searchsorted(self.file_first, a, side="right")) - 1
            f1 = int(np.searchsorted(self.file_first, max(a, b), side="right")) - 1
        else:
            r0, r1 = k0 * nrec, min(k1 * nrec, self.total) - 1
            f0 = int(np.searchsorted(self.file_first, r0, side="right")) - 1
            f1 = int(np.searchsorted(self.file_first, r1, side="right")) - 1
            f1 = max(f0, f1)
        return f0, f1


def _all_sum(vec, device):
    """Elementwise sum over the ranks of an int64 vector (one all_reduce)."""
    import torch
    import torch.distributed as dist
    t = torch.as_tensor(np.ascontiguousarray(vec, np.int64), device=device if device is not None else "cpu")
    if _collective():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def ingest_plan(rdr, nrec, rank, world, device=None, log=None):
    """The ranks' chunk starts (collective: every rank calls it).  See IngestPlan."""
    import time
    t0 = time.perf_counter()
    if world <= 1 or os.environ.get("NT_SHARD_INGEST", "1") == "0":
        return IngestPlan(reason="one rank" if world <= 1 else "NT_SHARD_INGEST=0")
    from ._lib import NanoTelError
    files = rdr.files()
    # the layout (a stat of every file) can fail on one rank only: its failure
    # goes through the same flag exchange as the reads below, so that no rank
    # waits in a collective the failing one never joins
    lay_err, plain, total_bytes = None, False, 0
    try:
        plain, total_bytes = rdr.layout()
    except (NanoTelError, OSError) as ex:
        lay_err = ex
    if _all_sum(np.array([1 if lay_err is not None else 0], np.int64), device)[0]:
        raise lay_err if lay_err is not None else RuntimeError("NanoTel: another rank failed to read the input")
    if plain:
        a, b = total_bytes * rank // world, total_bytes * (rank + 1) // world
        row, err = np.zeros((world, 4), np.int64), None
        try:
            pos, first, nxt = rdr.shard_range(a, b)
            row[rank] = (pos.size, first, nxt, 0)
        except NanoTelError as ex:
            pos, err = np.zeros(0, np.uint64), ex
            row[rank] = (0, 0, 0, 1)
        row = _all_sum(row.ravel(), device).reshape(world, 4)
        if row[:, 3].any():
            raise err if err is not None else RuntimeError("NanoTel: another rank failed to read the input")
        if any(row[r, 1] != row[r - 1, 2] for r in range(1, world)):
            plan = IngestPlan(reason="resynchronisation mismatch (a FASTQ quality line shaped like a header)")
        else:
            counts = row[:, 0]
            total = int(counts.sum())
            n_chunks = -(-total // nrec)
            g0 = int(counts[:rank].sum())
            first_local = (-g0) % nrec
            idx = np.arange(first_local, pos.size, nrec)
            starts = np.zeros(n_chunks, np.int64)
            if idx.size:
                starts[(g0 + idx) // nrec] = pos[idx].astype(np.int64)
            starts = _all_sum(starts, device)
            sizes = np.array([os.path.getsize(f) for f in files], np.int64)
            ff = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
            plan = IngestPlan("range", n_chunks, total, starts, ff)
    elif len(files) < 2:
        plan = IngestPlan(reason="a single gzip stream (inflated from its start by every rank)")
    else:
        own = np.arange(rank, len(files), world, dtype=np.uint64)
        vec, err = np.zeros(len(files) + 1, np.int64), None
        try:
            vec[own.astype(np.int64)] = rdr.count_files(own).astype(np.int64)
        except NanoTelError as ex:
            err = ex
            vec[-1] = 1
        vec = _all_sum(vec, device)
        if vec[-1]:
            raise err if err is not None else RuntimeError("NanoTel: another rank failed to read the input")
        counts = vec[:-1]
        total = int(counts.sum())
        n_chunks = -(-total // nrec)
        ff = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)  # files' first record index
        first = np.arange(n_chunks, dtype=np.int64) * nrec
        f = np.searchsorted(ff, first, side="right") - 1
        plan = IngestPlan("files", n_chunks, total, np.stack([f, first - ff[f]], axis=1), ff)
    plan.index_s = time.perf_counter() - t0
    if log is not None and not plan.sharded:
        log(f"ingest not sharded: {plan.reason}")
    return plan


def sequential_serials(flags_per_chunk):
    """Reference recurrence run chunk by chunk in one process (the oracle for
    the sharded path): list of per-chunk absolute serial arrays."""
    ss, mx = 1.0, NEG_INF
    out = []
    for f in flags_per_chunk:
        ser, _, ss, mx = assign_serials(f, serial_start=ss, max_serial=mx)
        out.append(ser)
    return out
