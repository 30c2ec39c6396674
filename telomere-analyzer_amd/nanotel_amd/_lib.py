"""ctypes binding of the in-tree HIP library (libnanotel.so, include/nanotel.h).

The library is the product: there is no CPU fallback.  If it is missing, or no
GPU is visible when a device call is made, the calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnanotel.so")

NT_OK = 0
ERRORS = {
    -1: "NT_E_ARG", -2: "NT_E_PATTERN", -3: "NT_E_LETTER", -4: "NT_E_EMPTY_READ",
    -5: "NT_E_RIGHT_EMPTY", -6: "NT_E_NEG_WIDTH", -7: "NT_E_HIP", -8: "NT_E_NOMEM",
    -9: "NT_E_LIMIT", -10: "NT_E_STATE", -11: "NT_E_IO",
}

ROW_TELOMERIC = 0x01
ROW_ERR_ALIGN = 0x10
ROW_DONE = 0x80


def row_na(p):
    return 0x02 << p


class NanoTelError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code
        self.name = ERRORS.get(code, str(code))


class NtParams(ctypes.Structure):
    _fields_ = [
        ("patterns", ctypes.c_char_p),
        ("tvr_patterns", ctypes.c_char_p),
        ("subseq_length", ctypes.c_int32),
        ("min_density", ctypes.c_double),
        ("check_right_edge", ctypes.c_int32),
        ("rc", ctypes.c_int32),
        ("legacy_no_ext", ctypes.c_int32),
    ]


class NtProgramInfo(ctypes.Structure):
    _fields_ = [("n_pass", ctypes.c_int32), ("n_pat", ctypes.c_int32), ("n_tvr", ctypes.c_int32),
                ("n_hits", ctypes.c_int32), ("raw_p1", ctypes.c_int32), ("jit", ctypes.c_int32),
                ("tscan", ctypes.c_int32), ("count_bytes", ctypes.c_int32)]


class NtBatch(ctypes.Structure):
    _fields_ = [
        ("planes", ctypes.c_void_p), ("blk_off", ctypes.c_void_p), ("len", ctypes.c_void_p),
        ("win_off", ctypes.c_void_p), ("exc_off", ctypes.c_void_p), ("exc_pos", ctypes.c_void_p),
        ("exc_code", ctypes.c_void_p), ("n_reads", ctypes.c_uint64), ("n_windows", ctypes.c_uint64),
        # bundle scan (optional): the bundles' reads, the reads left to the per-read scan
        ("bnd_read", ctypes.c_void_p), ("n_bundles", ctypes.c_uint64), ("list", ctypes.c_void_p),
        ("n_list", ctypes.c_uint64),
    ]


class NtOut(ctypes.Structure):
    _fields_ = [
        ("win_counts", ctypes.c_void_p), ("start", ctypes.c_void_p), ("end", ctypes.c_void_p),
        ("density", ctypes.c_void_p), ("flags", ctypes.c_void_p), ("hits", ctypes.c_void_p),
    ]


class NtSynthParams(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64), ("first_read", ctypes.c_uint64), ("read_len", ctypes.c_uint64),
        ("p_tract", ctypes.c_double), ("sub_rate", ctypes.c_double), ("variant_rate", ctypes.c_double),
        ("tract_min", ctypes.c_uint32), ("tract_max", ctypes.c_uint32), ("rc_layout", ctypes.c_int32),
    ]


# name -> (restype, argtypes); every symbol declared in include/nanotel.h
_P = ctypes.c_void_p
_U64P = ctypes.POINTER(ctypes.c_uint64)
SIGNATURES = {
    "nt_version": (ctypes.c_char_p, []),
    "nt_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "nt_destroy": (None, [_P]),
    "nt_last_error": (ctypes.c_char_p, [_P]),
    "nt_set_stream": (ctypes.c_int, [_P, _P]),
    "nt_synchronize": (ctypes.c_int, [_P]),
    "nt_set_pipelined": (ctypes.c_int, [_P, ctypes.c_int]),
    "nt_join": (ctypes.c_int, [_P]),
    "nt_wait_call": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "nt_compile": (ctypes.c_int, [_P, ctypes.POINTER(NtParams), ctypes.POINTER(NtProgramInfo)]),
    "nt_window_count": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    "nt_window_rows": (ctypes.c_uint64, [ctypes.c_int64]),
    "nt_read_blocks": (ctypes.c_uint64, [ctypes.c_uint64]),
    "nt_pack_count": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int32, _U64P, _U64P, _U64P,
                                     _U64P, _U64P]),
    "nt_pack_reads": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, _P, _P,
                                     _P, _P, _P, _P, _P]),
    "nt_exc_marks": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_uint64, _P]),
    "nt_bundle_plan": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_uint64, _P, _U64P, _P, _U64P]),
    "nt_scan_call": (ctypes.c_int, [_P, ctypes.POINTER(NtBatch), ctypes.POINTER(NtOut), ctypes.c_uint64]),
    "nt_set_profiling": (ctypes.c_int, [_P, ctypes.c_int]),
    "nt_kernel_times": (ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double)]),
    "nt_kernel_launches": (ctypes.c_int64, [_P]),
    "nt_call_kernel_times": (ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_double)]),
    "nt_call_launch_counts": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "nt_call_jit_state": (ctypes.c_int, [_P]),
    "nt_call_jit_wait": (ctypes.c_int, [_P]),
    "nt_jit_prebuild": (ctypes.c_int, [ctypes.POINTER(NtParams), ctypes.c_char_p]),
    "nt_analyze_host": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, _P, _P, _P, _P, _P, _P]),
    "nt_host_times": (ctypes.c_int, [_P, _P]),
    "nt_filter_call": (ctypes.c_int, [_P, _P, _P]),
    "nt_filter_host": (ctypes.c_int, [_P, _P, _P, ctypes.c_uint64, _P]),
    "nt_assign_serials": (ctypes.c_int64, [_P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double), _P, _P]),
    "nt_rows_columns": (ctypes.c_int64, [_P, _P, _P, _P, ctypes.c_uint64, ctypes.c_int32, _P, _P,
                                         ctypes.c_int64, _P, _P, _P, _P, _P, _P]),
    "nt_rows_csv": (ctypes.c_int64, [_P, _P, _P, _P, _P, _P, ctypes.c_int64, ctypes.c_int32, _P, _P,
                                     ctypes.c_double, _P, ctypes.c_uint64, _P, ctypes.c_uint64, _U64P]),
    "nt_reader_open": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "nt_reader_close": (None, [_P]),
    "nt_reader_file_count": (ctypes.c_uint64, [_P]),
    "nt_reader_file": (ctypes.c_char_p, [_P, ctypes.c_uint64]),
    "nt_reader_error": (ctypes.c_char_p, [_P]),
    "nt_reader_next": (ctypes.c_int64, [_P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "nt_reader_keep": (ctypes.c_int, [_P, ctypes.c_uint32]),
    "nt_reader_skip": (ctypes.c_int64, [_P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "nt_reader_layout": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), _U64P]),
    "nt_reader_shard_range": (ctypes.c_int64, [_P, ctypes.c_uint64, ctypes.c_uint64, _U64P, _U64P]),
    "nt_reader_shard_positions": (ctypes.c_int64, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    "nt_reader_count_files": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _P]),
    "nt_reader_plan": (ctypes.c_int, [_P, _P, ctypes.c_uint64]),
    "nt_reader_seek": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]),
    "nt_reader_stats": (ctypes.c_int, [_P, _U64P]),
    "nt_write_fasta_gz": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                         _U64P]),
    "nt_synth_device": (ctypes.c_int, [_P, ctypes.POINTER(NtSynthParams), ctypes.c_uint64, _P]),
    "nt_rc_device": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_uint64]),
    "nt_uniform_layout_device": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int32,
                                                _P, _P, _P]),
    "nt_synth_ascii": (ctypes.c_int, [ctypes.POINTER(NtSynthParams), ctypes.c_uint64, ctypes.c_char_p]),
}

_lib = None


def lib():
    """Load libnanotel.so (raises if it was not built: no fallback).

    One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 with
    the same SONAME (libamdhip64.so.7) as /opt/rocm's.  When torch is
    importable it is imported first, so that libnanotel binds to torch's
    already-loaded runtime and device pointers/streams are shared; a second
    runtime in the process would make torch's own initialisation fail.
    """
    global _lib
    if _lib is None:
        try:
            import torch  # noqa: F401  (load torch's libamdhip64 first)
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                              "(make -C telomere-analyzer_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib
