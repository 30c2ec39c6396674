"""The hiprtc sources of the pattern-specialised kernels build on the CPU (no
GPU needed: hiprtc only drives the compiler): the bundle scan (nt_tscan.h) and
the calling kernel (nt_call.h) for the Example's TTAGGG and for BASELINE's c4
set (2 patterns + 2 TVRs, the largest specialised calling kernel), and the
bundle scan for an 18-letter pattern (a halo of 17 positions each side).  Catches
JIT-only failures (hiprtc has no libc headers, only what nt_*.h include) before
a GPU run; the GPU tests run the same kernels for parity."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPRTC = "/opt/rocm/lib/libhiprtc.so"


def _tool():
    spec = importlib.util.spec_from_file_location("hiprtc_check", os.path.join(ROOT, "tools", "hiprtc_check.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


TTAGGG = "nt::CtPat<6, 8, 8, 1, 4, 4, 4>"
C4_PATS = "nt::CtPat<6, 8, 8, 1, 4, 4, 4>, nt::CtPat<6, 8, 2, 1, 4, 4, 4>"
C4_TVRS = "nt::CtPat<6, 8, 4, 1, 4, 4, 4>, nt::CtPat<6, 8, 8, 4, 4, 4, 4>"
# an 18-letter pattern (TAGGGTTAGGGTTAGGGT): the longest halo the walk has
LONG = "nt::CtPat<18, 8, 1, 4, 4, 4, 8, 8, 1, 4, 4, 4, 8, 8, 1, 4, 4, 4, 8>"


@pytest.mark.skipif(not os.path.exists(HIPRTC), reason="no hiprtc in this image")
@pytest.mark.parametrize("kernel,pats,tvrs", [
    ("call", TTAGGG, ""),
    ("call", C4_PATS, C4_TVRS),
    ("tscan", TTAGGG, ""),
    ("tscan", C4_PATS, C4_TVRS),
    ("tscan", LONG, ""),
])
def test_specialised_kernel_sources_build(kernel, pats, tvrs):
    t = _tool()
    src = t.call_source(pats, tvrs) if kernel == "call" else t.tscan_source(pats, tvrs)
    assert t.compile_src(src, quiet=True) == 0
