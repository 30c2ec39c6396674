"""ctypes binding of the CPU oracle (oracle/_build/libnanotel_oracle.so).

Test infrastructure only: the oracle is the checker, never the product.
"""
import ctypes
import math
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "libnanotel_oracle.so")


class NtoRow(ctypes.Structure):
    _fields_ = [
        ("start", ctypes.c_int32 * 3),
        ("end", ctypes.c_int32 * 3),
        ("width", ctypes.c_int64 * 3),
        ("density", ctypes.c_double * 3),
        ("na", ctypes.c_int32 * 3),
        ("n_pass", ctypes.c_int32),
        ("telomeric", ctypes.c_int32),
        ("n_windows", ctypes.c_int64),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "nanotel_oracle.c")
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        L = ctypes.CDLL(LIB_PATH)
        L.nto_patterns_new.restype = ctypes.c_void_p
        L.nto_patterns_new.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        L.nto_patterns_free.argtypes = [ctypes.c_void_p]
        L.nto_patterns_npass.argtypes = [ctypes.c_void_p]
        L.nto_patterns_count.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.nto_window_count.restype = ctypes.c_int64
        L.nto_window_count.argtypes = [ctypes.c_int64, ctypes.c_int]
        L.nto_match_pattern.restype = ctypes.c_int64
        L.nto_match_pattern.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int64]
        L.nto_reverse_complement.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        L.nto_analyze_read.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(NtoRow), ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_uint32)]
        L.nto_filter_read.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_double,
                                      ctypes.c_int]
        L.nto_assign_serials.restype = ctypes.c_int64
        L.nto_assign_serials.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__(f"oracle error {code}")
        self.code = code


class Patterns:
    def __init__(self, patterns, tvr_patterns=None):
        err = ctypes.c_int(0)
        self.h = lib().nto_patterns_new(patterns.encode(), None if tvr_patterns is None else tvr_patterns.encode(),
                                        ctypes.byref(err))
        if not self.h:
            raise OracleError(err.value)
        self.npass = lib().nto_patterns_npass(self.h)
        self.n_pat = lib().nto_patterns_count(self.h, 0)
        self.n_tvr = lib().nto_patterns_count(self.h, 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().nto_patterns_free(self.h)
            self.h = None


def window_count(n, L=100):
    return lib().nto_window_count(n, L)


def match_pattern(pattern, subject, k=0, fixed=True):
    n = len(subject)
    cap = n + 64
    buf = (ctypes.c_int32 * cap)()
    cnt = lib().nto_match_pattern(pattern.encode(), subject.encode(), n, k, int(fixed), buf, cap)
    if cnt < 0:
        raise OracleError(cnt)
    return list(buf[:cnt])


def reverse_complement(seq):
    b = ctypes.create_string_buffer(seq.encode(), len(seq))
    rc = lib().nto_reverse_complement(b, len(seq))
    if rc:
        raise OracleError(rc)
    return b.raw[:len(seq)].decode()


def analyze_read(seq, pats, L=100, min_density=0.6, right_edge=False, legacy_no_ext=False,
                 want_windows=False, want_hits=False):
    """Returns dict(row fields [+ win_counts per pass] [+ hits])."""
    n = len(seq)
    row = NtoRow()
    nw = window_count(n, L) if n > 0 else 0
    wc = (ctypes.c_uint32 * max(1, pats.npass * nw))() if want_windows else None
    hc = (ctypes.c_uint32 * max(1, 2 * pats.n_pat + pats.n_tvr))() if want_hits else None
    rc = lib().nto_analyze_read(seq.encode(), n, pats.h, L, min_density, int(right_edge), int(legacy_no_ext),
                                ctypes.byref(row), wc, hc)
    if rc:
        raise OracleError(rc)
    out = {
        "n_pass": row.n_pass,
        "telomeric": bool(row.telomeric),
        "start": list(row.start[:row.n_pass]),
        "end": list(row.end[:row.n_pass]),
        "width": list(row.width[:row.n_pass]),
        "density": list(row.density[:row.n_pass]),
        "na": [bool(x) for x in row.na[:row.n_pass]],
        "n_windows": row.n_windows,
    }
    if want_windows:
        out["win_counts"] = [list(wc[p * nw:(p + 1) * nw]) for p in range(row.n_pass)]
    if want_hits:
        out["hits"] = list(hc[:2 * pats.n_pat + pats.n_tvr])
    return out


def filter_read(seq, pats, min_density=0.6, right_edge=False):
    """--use_filter decision for one read in scan orientation (True = kept)."""
    rc = lib().nto_filter_read(seq.encode(), len(seq), pats.h, min_density, int(right_edge))
    if rc < 0:
        raise OracleError(rc)
    return bool(rc)


def assign_serials(is_telo, serial_start=1.0, max_serial=-math.inf):
    n = len(is_telo)
    t = (ctypes.c_uint8 * max(1, n))(*[1 if x else 0 for x in is_telo])
    ss = ctypes.c_double(serial_start)
    mx = ctypes.c_double(max_serial)
    ser = (ctypes.c_double * max(1, n))()
    order = (ctypes.c_int64 * max(1, n))()
    rows = lib().nto_assign_serials(t, n, ctypes.byref(ss), ctypes.byref(mx), ser, order)
    return list(ser[:n]), list(order[:rows]), ss.value, mx.value


def read_fasta(path):
    names, seqs, cur = [], [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\r\n")
            if line.startswith(">"):
                if names:
                    seqs.append("".join(cur))
                names.append(line[1:])
                cur = []
            else:
                cur.append(line.strip())
    if names:
        seqs.append("".join(cur))
    return names, seqs
