#!/usr/bin/env python3
"""Compile the hiprtc source of the pattern-specialised kernels on the CPU
(no GPU needed: hiprtc only drives the compiler) and print the log -- the
same headers and options nt_jit.cpp uses, for a pattern type list such as
"nt::CtPat<6,8,8,1,4,4,4>".  Catches JIT-only failures (hiprtc has no libc
headers) before a GPU run.

usage: tools/hiprtc_check.py "nt::CtPat<6,8,8,1,4,4,4>" [tvr list] [L] [extra options...]
       tools/hiprtc_check.py --call "<patterns>" "<tvrs>" "<patterns, eq tables>" "<tvrs, eq tables>"
         (the calling kernel, nt_call.h)
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "telomere-analyzer_amd", "csrc")


TYPEDEFS = "".join(f"typedef __hip_internal::{t} {t};\n" for t in
                   ("uint8_t", "uint16_t", "uint32_t", "uint64_t", "int32_t", "int64_t"))


def tscan_source(pats, tvrs="", L="100"):
    """The bundle scan's hiprtc source (as nt_jit.cpp jit_source builds it)."""
    src = TYPEDEFS + '#include "nt_tscan.h"\n'
    src += f"using TPats = nt::CtList<{pats}>;\nusing TTvrs = nt::CtList<{tvrs}>;\n"
    src += f"using TJit = nt::TProg<TPats, TTvrs, {L}>;\n"
    src += """
constexpr int kTsW = nt::ts_lds_words<TJit::kNP, TJit::kL>();
constexpr int kTsNW = 40960 / kTsW < 4 ? 40960 / kTsW : 4;
extern "C" __global__ void __launch_bounds__(kTsNW * 64) __attribute__((amdgpu_waves_per_eu(1)))
nt_tscan_jit(NtBatch B, NtOut O, uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue,
             uint32_t thr_full) {
  __shared__ uint32_t tsl[kTsNW * kTsW];
  nt::tscan_bundles<TJit, TPats, TTvrs>(B, O, tmask, queue, thr_full, tsl + (threadIdx.x >> 6) * kTsW);
}
"""
    return src


def call_source(pats, tvrs="", pats_eq=None, tvrs_eq=None, raw=None):
    """The calling kernel's hiprtc source (as nt_jit.cpp call_source builds it).
    raw: the program keeps P1's raw views (one fixed pattern); default: one
    pattern in the list."""
    if raw is None:
        raw = pats.count("CtPat") == 1
    pats_eq = pats if pats_eq is None else pats_eq
    tvrs_eq = tvrs if tvrs_eq is None else tvrs_eq
    return (TYPEDEFS + '#include "nt_call.h"\n'
            f"using JitCall = nt::CtCall<nt::CtList<{pats}>, nt::CtList<{tvrs}>, nt::CtList<{pats_eq}>, "
            f"nt::CtList<{tvrs_eq}>, {'true' if raw else 'false'}>;\nNT_CALL_KERNEL(nt_call_jit, JitCall)\n")


def main():
    if sys.argv[1] == "--call":
        pats, tvrs, pats_eq, tvrs_eq = (sys.argv[2:6] + ["", "", "", ""])[:4]
        sys.exit(compile_src(call_source(pats, tvrs, pats_eq, tvrs_eq), sys.argv[6:]))
    pats = sys.argv[1]
    tvrs = sys.argv[2] if len(sys.argv) > 2 else ""
    L = sys.argv[3] if len(sys.argv) > 3 else "100"
    sys.exit(compile_src(tscan_source(pats, tvrs, L), sys.argv[4:]))


def compile_src(src, extra=(), quiet=False):
    """hiprtc-compiles src for gfx950 with nt_jit.cpp's options; 0 = built."""
    import time
    names = ["nt_common.h", "nt_device.h", "nt_scan.h", "nt_tscan.h", "nt_call.h"]
    hdrs = [open(os.path.join(CSRC, n), "rb").read() for n in names]
    lib = ctypes.CDLL("/opt/rocm/lib/libhiprtc.so")
    prog = ctypes.c_void_p()
    arr = ctypes.c_char_p * len(names)
    t0 = time.time()
    rc = lib.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"nt_jit.hip", len(names),
                                 arr(*hdrs), arr(*[n.encode() for n in names]))
    assert rc == 0, rc
    opts = [b"--offload-arch=gfx950", b"-O3", b"-std=c++17", b"-ffp-contract=off", b"-mllvm",
            b"-amdgpu-sched-strategy=max-ilp"] + [x.encode() for x in extra]
    rc = lib.hiprtcCompileProgram(prog, len(opts), (ctypes.c_char_p * len(opts))(*opts))
    n = ctypes.c_size_t()
    lib.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
    log = ctypes.create_string_buffer(n.value + 1)
    lib.hiprtcGetProgramLog(prog, log)
    if not quiet or rc != 0:
        print(log.value.decode(errors="replace")[-4000:])
    print("hiprtc rc", rc, f"({time.time() - t0:.1f} s)")
    return 0 if rc == 0 else 1


if __name__ == "__main__":
    main()
