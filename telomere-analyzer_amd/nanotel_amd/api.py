"""Host-side mirror of NanoTel's per-chunk interface over the HIP C-ABI.

`NanoTel` owns one device context and one compiled pattern program
(extract_patterns, NanoTel.R:2322-2334).  `NanoTel.analyze()` is the
per-chunk replacement of search_patterns' loop over analyze_read
(NanoTel.R:2001-2078, 1774-1976): one kernel launch for the whole chunk.
"""
import ctypes

import numpy as np

from ._lib import (NanoTelError, NtBatch, NtOut, NtParams, NtProgramInfo, NtSynthParams, lib,
                   ROW_DONE, ROW_TELOMERIC)


def _check(rc, ctx=None):
    if rc < 0:
        msg = lib().nt_last_error(ctx).decode() if ctx else ""
        raise NanoTelError(rc, msg)
    return rc


def window_count(n, subseq_length=100):
    """split_telo window count (NanoTel.R:199-227)."""
    return lib().nt_window_count(int(n), int(subseq_length))


def window_rows(nw):
    """Windows of a read's padded count row (nw rounded up to a multiple of 64;
    scalar or numpy array): the win_counts / win_off layout, nt_common.h."""
    if isinstance(nw, np.ndarray):
        return (nw + 63) // 64 * 64
    return lib().nt_window_rows(int(nw))


def read_blocks(n):
    """32-base blocks of a read's slot in the plane buffer (2*ceil(n/64));
    slots start at even block offsets (16-byte segments)."""
    return lib().nt_read_blocks(int(n))


class NanoTel:
    """One GPU context + compiled --patterns/--tvr_patterns/flags."""

    def __init__(self, patterns, tvr_patterns=None, subseq_length=100, min_density=0.6,
                 check_right_edge=False, rc=False, legacy_no_ext=False, device=0):
        L = lib()
        h = ctypes.c_void_p()
        rc_ = L.nt_create(int(device), ctypes.byref(h))
        if rc_ != 0 or not h.value:
            raise NanoTelError(rc_, "nt_create failed (no GPU visible?)")
        self._h = h
        self._pat_b = patterns.encode() if isinstance(patterns, str) else patterns
        self._tvr_b = None if tvr_patterns is None else (
            tvr_patterns.encode() if isinstance(tvr_patterns, str) else tvr_patterns)
        self.params = NtParams(self._pat_b, self._tvr_b, int(subseq_length), float(min_density),
                               int(bool(check_right_edge)), int(bool(rc)), int(bool(legacy_no_ext)))
        info = NtProgramInfo()
        _check(L.nt_compile(self._h, ctypes.byref(self.params), ctypes.byref(info)), self._h)
        self.n_pass = info.n_pass
        self.n_pat = info.n_pat
        self.n_tvr = info.n_tvr
        self.n_hits = info.n_hits
        self.raw_p1 = bool(info.raw_p1)
        # scan kernel specialised for these patterns at run time (hiprtc), or
        # the ahead-of-time kernels (NT_JIT=0 / hiprtc unavailable)
        self.jit = bool(info.jit)
        # bundled reads take the bundle scan (the reads transposed 32 to a bundle)
        self.tscan = bool(info.tscan)
        self.count_bytes = int(info.count_bytes)  # window counts: uint8 (subseq_length <= 170) or uint16
        self.count_dtype = np.uint8 if self.count_bytes == 1 else np.uint16
        self.subseq_length = int(subseq_length)

    # ------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().nt_destroy(self._h)
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

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_handle):
        _check(lib().nt_set_stream(self._h, ctypes.c_void_p(stream_handle)), self._h)

    def set_profiling(self, on=True):
        _check(lib().nt_set_profiling(self._h, int(bool(on))), self._h)

    def kernel_times(self):
        """(calls, scan_ms, call_ms): summed HIP-event spans of the scan and the
        calling kernels over the scan_call()s since the previous query."""
        a, b = ctypes.c_double(), ctypes.c_double()
        n = _check(lib().nt_kernel_times(self._h, ctypes.byref(a), ctypes.byref(b)), self._h)
        return int(n), a.value, b.value

    def kernel_launches(self):
        """Scan-kernel launches behind the last kernel_times() (a bundle scan in
        ranges launches once per range): scan_ms / this = one launch."""
        return int(_check(lib().nt_kernel_launches(self._h), self._h))

    def call_kernel_times(self):
        """(calling launches, their summed own span in ms) behind the last
        kernel_times(): events on the stream each calling kernel ran on."""
        ms = ctypes.c_double()
        n = _check(lib().nt_call_kernel_times(self._h, ctypes.byref(ms)), self._h)
        return int(n), ms.value

    def call_launch_counts(self):
        """Calling-kernel launches since creation: (ahead-of-time, specialised)."""
        out = (ctypes.c_int64 * 2)()
        _check(lib().nt_call_launch_counts(self._h, out), self._h)
        return int(out[0]), int(out[1])

    def call_jit(self):
        """True if the last scan_call() ran the calling kernel specialised for
        the patterns (hiprtc), False for the ahead-of-time one."""
        return bool(lib().nt_call_jit_state(self._h))

    def host_times(self):
        """nt_host_times: cumulative seconds of the host path's phases."""
        t = np.zeros(6, np.float64)
        _check(lib().nt_host_times(self._h, t.ctypes.data), self._h)
        return dict(zip(("layout", "pack", "plan", "upload", "device", "checks"), t.tolist()))

    def call_jit_wait(self):
        """Wait for the background build of the calling kernel specialised for
        the patterns (started by nt_compile); True when it is available."""
        return bool(_check(lib().nt_call_jit_wait(self._h), self._h))

    def synchronize(self):
        _check(lib().nt_synchronize(self._h), self._h)

    def set_pipelined(self, on=True):
        """nt_set_pipelined: a scan_call() returns with its last bundle range's
        calling still running beside the next call's scan; outputs are
        complete after join() / synchronize().  Consecutive calls need their
        own output buffers."""
        _check(lib().nt_set_pipelined(self._h, int(bool(on))), self._h)

    def wait_call(self, back=0):
        """nt_wait_call: the context stream waits until the calling of the call
        `back` calls before the latest one is done (its inputs may then be
        overwritten by work enqueued on the context stream)."""
        _check(lib().nt_wait_call(self._h, int(back)), self._h)

    def join(self):
        """nt_join: the launch stream waits for every calling launched so far."""
        _check(lib().nt_join(self._h), self._h)

    # ------------------------------------------------------------------
    def analyze(self, seqs, want_windows=False, want_hits=False):
        """Scan + call every read of a chunk (host buffers in, host arrays out).

        Returns a dict of numpy arrays: start/end (n,3) int32 (1-based, -1 =
        no telomere), density (n,3) float64, flags (n,) uint8, width (n,3),
        telomeric (n,) bool [, win_counts (flat, count_dtype), win_off (n,) ]
        [, hits (n, n_hits) uint32].
        """
        bseqs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        n = len(bseqs)
        ptrs = (ctypes.c_char_p * max(1, n))(*bseqs)
        lens = np.array([len(b) for b in bseqs], np.uint64)
        return self._analyze(ctypes.addressof(ptrs), lens, n, want_windows, want_hits)

    def analyze_pointers(self, ptrs, lens, want_windows=False, want_hits=False):
        """analyze() of reads given as host addresses (a uint64 array of
        `const char*`, e.g. several reader chunks' sequences joined) and lengths."""
        ptrs = np.ascontiguousarray(ptrs, np.uint64)
        return self._analyze(ptrs.ctypes.data, lens, int(ptrs.size), want_windows, want_hits)

    def analyze_chunk(self, chunk, want_windows=False, want_hits=False):
        """analyze() of an io.Reader chunk, zero-copy (the reader's buffers)."""
        return self._analyze(chunk.seq_ptrs, chunk.lengths, chunk.n, want_windows, want_hits)

    def _analyze(self, ptrs_addr, lens, n, want_windows, want_hits):
        out = {
            "start": np.full((n, 3), -1, np.int32),
            "end": np.full((n, 3), -1, np.int32),
            "density": np.zeros((n, 3), np.float64),
            "flags": np.zeros(n, np.uint8),
        }
        if n == 0:
            out["width"] = np.zeros((0, 3), np.int64)
            out["telomeric"] = np.zeros(0, bool)
            return out
        lens = np.ascontiguousarray(lens, np.uint64)
        wc = None
        if want_windows:
            nw = np.array([window_count(int(x), self.subseq_length) for x in lens], np.int64)
            rows = window_rows(nw)  # padded rows (nt_common.h): 16-byte aligned
            win_off = np.zeros(n, np.int64)
            win_off[1:] = np.cumsum(rows)[:-1]
            wc = np.zeros(max(1, int(rows.sum()) * self.n_pass), self.count_dtype)
            out["win_off"] = win_off
            out["n_windows"] = nw
        hits = np.zeros((n, max(1, self.n_hits)), np.uint32) if want_hits else None
        rc = lib().nt_analyze_host(
            self._h, ctypes.c_void_p(ptrs_addr), lens.ctypes.data, n,
            out["start"].ctypes.data, out["end"].ctypes.data, out["density"].ctypes.data,
            out["flags"].ctypes.data, None if wc is None else wc.ctypes.data,
            None if hits is None else hits.ctypes.data)
        _check(rc, self._h)
        out["width"] = out["end"].astype(np.int64) - out["start"].astype(np.int64) + 1
        out["telomeric"] = (out["flags"] & ROW_TELOMERIC) != 0
        assert np.all(out["flags"] & ROW_DONE), "kernel did not process every read"
        if wc is not None:
            out["win_counts"] = wc
        if hits is not None:
            out["hits"] = hits[:, :self.n_hits]
        return out

    def filter(self, seqs):
        """--use_filter decision per read (bool array; True = kept), reads in
        input orientation (the context's rc is applied as in analyze())."""
        bseqs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        n = len(bseqs)
        ptrs = (ctypes.c_char_p * max(1, n))(*bseqs)
        lens = np.array([len(b) for b in bseqs], np.uint64)
        return self._filter(ctypes.addressof(ptrs), lens, n)

    def filter_chunk(self, chunk):
        """filter() of an io.Reader chunk, zero-copy."""
        return self._filter(chunk.seq_ptrs, chunk.lengths, chunk.n)

    def _filter(self, ptrs_addr, lens, n):
        keep = np.zeros(max(1, n), np.uint8)
        if n:
            lens = np.ascontiguousarray(lens, np.uint64)
            _check(lib().nt_filter_host(self._h, ctypes.c_void_p(ptrs_addr), lens.ctypes.data, n,
                                        keep.ctypes.data), self._h)
        return keep[:n].astype(bool)

    def window_counts(self, res, read, p):
        """Window counts of pass p for read `read` from an analyze(want_windows) result."""
        nw = int(res["n_windows"][read])
        off = int(res["win_off"][read]) * self.n_pass + p * int(window_rows(nw))
        return res["win_counts"][off:off + nw]

    # ------------------------------------------------------------------
    def scan_call_device(self, planes, blk_off, lengths, win_off, n_reads, n_windows, max_len, start,
                         end, density, flags, win_counts, hits=0, exc_off=0, exc_pos=0, exc_code=0,
                         bundles=None):
        """Device-resident hot path: all pointer arguments are device pointers
        (ints); n_windows = sum of the window rows (window_rows).  bundles: a DeviceBundles
        (a bundle_plan's lists on the device) or None (per-read scan only).
        Asynchronous on the context stream (see set_stream)."""
        B = self._batch(planes, blk_off, lengths, win_off, n_reads, n_windows, exc_off, exc_pos, exc_code,
                        bundles)
        O = NtOut(win_counts or None, start, end, density, flags, hits or None)
        _check(lib().nt_scan_call(self._h, ctypes.byref(B), ctypes.byref(O), int(max_len)), self._h)

    @staticmethod
    def _batch(planes, blk_off, lengths, win_off, n_reads, n_windows, exc_off=0, exc_pos=0, exc_code=0,
               bundles=None):
        b = bundles
        return NtBatch(planes, blk_off, lengths, win_off, exc_off or None, exc_pos or None,
                       exc_code or None, int(n_reads), int(n_windows),
                       b.bnd_read if b else None, b.n_bundles if b else 0, (b.list or None) if b else None,
                       b.n_list if b else 0)

    def exc_marks(self, lengths, exc_off, exc_pos):
        """nt_exc_marks on host arrays: uint8 per read, 1 = its non-ACGT letters
        reach more than NT_EXC_WINDOWS windows (keep it on the per-read scan:
        pass the result to bundle_plan)."""
        ln = np.ascontiguousarray(lengths, np.uint32)
        eo = np.ascontiguousarray(exc_off, np.uint32)
        ep = np.ascontiguousarray(exc_pos, np.uint32)
        out = np.zeros(max(1, ln.size), np.uint8)
        _check(lib().nt_exc_marks(self._h, ln.ctypes.data, eo.ctypes.data, ep.ctypes.data if ep.size else None,
                                  ln.size, out.ctypes.data), self._h)
        return out[:ln.size]

    def bundle_plan(self, lengths, has_exc=None, blk_off=None):
        """nt_bundle_plan on host arrays: returns a BundlePlan (numpy arrays).
        blk_off (the batch's block offsets; None = the caller vouches that
        every bundle's planes lie within 2 GiB): bundles spread wider go to the
        per-read scan."""
        ln = np.ascontiguousarray(lengths, np.uint32)
        n = ln.size
        nbmax = (n + 31) // 32
        bread = np.zeros(max(1, nbmax * 32), np.uint32)
        lst = np.zeros(max(1, n), np.uint32)
        hx = None if has_exc is None else np.ascontiguousarray(has_exc, np.uint8)
        bo = None if blk_off is None else np.ascontiguousarray(blk_off, np.uint64)
        nb, nl = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().nt_bundle_plan(self._h, ln.ctypes.data, None if bo is None else bo.ctypes.data,
                                    None if hx is None else hx.ctypes.data, n, bread.ctypes.data, ctypes.byref(nb),
                                    lst.ctypes.data, ctypes.byref(nl)), self._h)
        return BundlePlan(bread[:nb.value * 32], lst[:nl.value])

    def synth_device(self, sp, n_reads, planes_ptr):
        _check(lib().nt_synth_device(self._h, ctypes.byref(sp), int(n_reads), planes_ptr), self._h)

    def rc_device(self, planes_in, planes_out, blk_off_ptr, len_ptr, n_reads):
        """nt_rc_device: planes_out = the reverse complement of every read of
        planes_in (device pointers, same layout; A/C/G/T reads)."""
        _check(lib().nt_rc_device(self._h, planes_in, planes_out, blk_off_ptr, len_ptr, int(n_reads)), self._h)

    def uniform_layout_device(self, n_reads, read_len, blk_off_ptr, len_ptr, win_off_ptr):
        _check(lib().nt_uniform_layout_device(self._h, int(n_reads), int(read_len), self.subseq_length,
                                              blk_off_ptr, len_ptr, win_off_ptr), self._h)


class BundlePlan:
    """Host result of nt_bundle_plan: bnd_read (n_bundles*32 u32, ~0 = empty
    slot) and list (the reads left to the per-read scan)."""

    def __init__(self, bnd_read, lst):
        self.bnd_read, self.list = bnd_read, lst
        self.n_bundles = len(bnd_read) // 32


class DeviceBundles:
    """Device pointers (ints) of a BundlePlan for scan_call_device."""

    def __init__(self, bnd_read, n_bundles, lst, n_list):
        self.bnd_read, self.n_bundles, self.list, self.n_list = bnd_read, n_bundles, lst, n_list


def jit_prebuild(patterns, tvr_patterns=None, subseq_length=100, min_density=0.6, check_right_edge=False,
                 rc=False, arch="gfx950"):
    """nt_jit_prebuild (no device): the kernels specialised for this parameter
    set go into the on-disk code-object cache (jitcache/ beside the library)."""
    pat = patterns.encode() if isinstance(patterns, str) else patterns
    tvr = None if tvr_patterns is None else (tvr_patterns.encode() if isinstance(tvr_patterns, str)
                                             else tvr_patterns)
    prm = NtParams(pat, tvr, int(subseq_length), float(min_density), int(bool(check_right_edge)), int(bool(rc)), 0)
    _check(lib().nt_jit_prebuild(ctypes.byref(prm), arch.encode()))


def synth_params(seed=20260501, first_read=0, read_len=50000, p_tract=0.5, sub_rate=0.02,
                 variant_rate=0.0, tract_min=1000, tract_max=15000, rc_layout=False):
    return NtSynthParams(int(seed), int(first_read), int(read_len), float(p_tract), float(sub_rate),
                         float(variant_rate), int(tract_min), int(tract_max), int(bool(rc_layout)))


def synth_read_ascii(sp, index):
    """Host twin of the device generator (nt_rng.h): read `first_read + index`."""
    buf = ctypes.create_string_buffer(int(sp.read_len))
    _check(lib().nt_synth_ascii(ctypes.byref(sp), int(index), buf))
    return buf.raw[:int(sp.read_len)].decode()


def assign_serials(is_telo, serial_start=1.0, max_serial=float("-inf")):
    """A15 for one chunk: returns (serials, row_order, next_serial_start, max_serial)."""
    t = np.ascontiguousarray(np.asarray(is_telo, dtype=np.uint8))
    n = t.size
    ser = np.zeros(max(1, n), np.float64)
    order = np.zeros(max(1, n), np.int64)
    ss = ctypes.c_double(serial_start)
    mx = ctypes.c_double(max_serial)
    rows = lib().nt_assign_serials(t.ctypes.data if n else None, n, ctypes.byref(ss), ctypes.byref(mx),
                                   ser.ctypes.data, order.ctypes.data)
    _check(rows)
    return ser[:n], order[:rows], ss.value, mx.value


NA_INT32 = -(1 << 31)  # R's NA_integer_ (NT_NA_INT32)
NA_REAL_BITS = 0x7FF00000000007A2  # R's NA_real_ (NT_NA_REAL_BITS)


def rows_columns(res, lengths, serials, order, n_pass):
    """nt_rows_columns: the chunk's rows (row i = read order[i]) as the columns
    of analyze_read's data.frame (NanoTel.R:1820-1837, 1926-1974), with R's NA
    values where a pass found no telomere.  Returns a dict: serial (rows,)
    float64, length (rows,) int32, density / start / end / width (n_pass, rows)
    and na (n_pass, rows) bool."""
    n = int(res["start"].shape[0])
    order = np.ascontiguousarray(order, np.int64)
    rows = int(order.size)
    start = np.ascontiguousarray(res["start"], np.int32)
    end = np.ascontiguousarray(res["end"], np.int32)
    dens = np.ascontiguousarray(res["density"], np.float64)
    lens = np.ascontiguousarray(lengths, np.uint64)
    ser = np.ascontiguousarray(serials, np.float64)
    assert start.shape == (n, 3) and end.shape == (n, 3) and dens.shape == (n, 3) and lens.size == n
    out = {"serial": np.zeros(max(1, rows), np.float64), "length": np.zeros(max(1, rows), np.int32),
           "density": np.zeros((n_pass, max(1, rows)), np.float64)}
    for k in ("start", "end", "width"):
        out[k] = np.zeros((n_pass, max(1, rows)), np.int32)
    got = lib().nt_rows_columns(start.ctypes.data, end.ctypes.data, dens.ctypes.data, lens.ctypes.data, n,
                                int(n_pass), ser.ctypes.data, order.ctypes.data, rows,
                                out["serial"].ctypes.data, out["length"].ctypes.data, out["density"].ctypes.data,
                                out["start"].ctypes.data, out["end"].ctypes.data, out["width"].ctypes.data)
    _check(got)
    for k in out:
        out[k] = out[k][..., :rows]
    out["na"] = out["start"] == NA_INT32
    return out


def rows_csv(cols, name_ptrs, name_lens, n_pass, sci_threshold=None, ids=True):
    """nt_rows_csv: (summary.csv lines, reads_ids.txt lines) as bytes for the
    columns of rows_columns(); name_ptrs / name_lens: each row's sequence_ID
    (host addresses and lengths, in row order)."""
    rows = int(cols["serial"].size)
    if rows == 0:
        return b"", b""
    name_ptrs = np.ascontiguousarray(name_ptrs, np.uint64)
    name_lens = np.ascontiguousarray(name_lens, np.uint64)
    cap = int(2 * name_lens.sum()) + rows * (3 + (3 + 4 * n_pass) * 40)
    out = np.empty(cap, np.uint8)
    ids_out = np.empty(int(name_lens.sum()) + rows, np.uint8) if ids else None
    ib = ctypes.c_uint64()
    c = {k: np.ascontiguousarray(cols[k]) for k in ("serial", "length", "density", "start", "end", "width")}
    n = lib().nt_rows_csv(c["serial"].ctypes.data, c["length"].ctypes.data, c["density"].ctypes.data,
                          c["start"].ctypes.data, c["end"].ctypes.data, c["width"].ctypes.data, rows, int(n_pass),
                          name_ptrs.ctypes.data, name_lens.ctypes.data,
                          float(sci_threshold) if sci_threshold else 0.0, out.ctypes.data, cap,
                          None if ids_out is None else ids_out.ctypes.data, 0 if ids_out is None else ids_out.size,
                          ctypes.byref(ib))
    _check(n)
    return out[:n].tobytes(), (ids_out[:ib.value].tobytes() if ids_out is not None else b"")
