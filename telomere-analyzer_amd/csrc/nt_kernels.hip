// nt_kernels.hip -- NanoTel hot path on MI355X (gfx950 / CDNA4).
//
// Two kernels per batch:
//
//  nt_scan_kernel  -- HBM-bound, one wave per read (grid-stride).  Each lane
//     owns one 32-base word; the wave streams the read's 2-bit planes with
//     coalesced 8-byte loads through a prefetch ring, runs the bit-sliced
//     matchPattern of every pattern at the 32 starts of each word (exact and
//     <=1 mismatch in one pass, Biostrings' out-of-bound rule), builds the
//     coverage = OR of shifted hit words (trim + IRanges::reduce) and adds
//     covered bases per subseq_length window with LDS atomics
//     (analyze_subtelos / get_sub_density, NanoTel.R:717-766, 449-468).
//     Writes the uint16 window counts, the telomeric-window bitmask of every
//     pass (class -5, NanoTel.R:749-758) and the matchPattern hit counts.
//
//  nt_call_kernel  -- one LANE per read-pass (nt_call.h).  The telomere calling of
//     find_telo_position_wraper and callees (NanoTel.R:973-1155, 1692-1764,
//     843-959, 496-697) and analyze_read's row (NanoTel.R:1840-1974) from the
//     window bitmasks and counts; coverage near the called boundaries is
//     recomputed from the planes.  Sequential per read (fp64 sums in R's
//     order) but 64 reads per wave, so its instruction cost is amortised 64x.
//
// No MFMA: integer / bit work bound by HBM bandwidth.
#include <hip/hip_runtime.h>

#include "nt_common.h"
#include "nt_device.h"
#include "nt_rng.h"
#include "nt_scan.h"
#include "nt_call.h"

namespace nt {

// ============================================================ scan (AOT)
//
// Ahead-of-time scan kernels for run-time pattern sets (nt_scan.h); the
// hiprtc-specialised twin is built by nt_jit.cpp.
template <class S, bool kLds>
__global__ void __launch_bounds__(kWG)
nt_scan_kernel(const NtProgram* __restrict__ prog, const uint32_t* __restrict__ thr, NtBatch B,
               NtOut O, uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue,
               uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t wave_words, uint32_t* __restrict__ gscr) {
  extern __shared__ uint32_t smem[];
  const uint64_t gw = (uint64_t)blockIdx.x * kNWaves + (threadIdx.x >> 6);
  uint32_t* wmem = kLds ? smem + (uint64_t)(threadIdx.x >> 6) * wave_words : gscr + gw * wave_words;
  scan_reads<S, kLds>(prog, thr, B, O, tmask, queue, len_lo, len_hi, claim, nstatic, wmem);
}

// ================================================================= call
//
// The calling kernel (nt_call.h) with run-time pattern lists; the
// hiprtc-specialised twin (compile-time patterns) is built by nt_jit.cpp.
NT_CALL_KERNEL(nt_call_kernel, RtCall)
// programs with a TVR of more than 32 letters (wider neighbourhoods)
NT_CALL_KERNEL(nt_call_kernel_long, RtCallLong)

// After the per-pass calling kernels (NT_CALL_KERNEL_PASS, one launch per
// pass): the row flags of each read -- NA per pass, the errors the passes left
// in end (-2 / -3), telomeric = max width over the passes >= 30 (NanoTel.R:
// 1847-1868) -- and the -1 / -1 / 0 of the passes the program does not run,
// as the one-kernel form (Call::run) writes them.
__global__ void __launch_bounds__(256) nt_call_combine_kernel(NtBatch B, NtOut O, int np) {
  const uint64_t total = B.list ? B.n_list : B.n_reads;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total; idx += stride) {
    const uint64_t r = B.list ? (uint64_t)B.list[idx] : idx;
    if (r == 0xFFFFFFFFull) continue;
    bool span = false;  // a pass left -4: the bundle scan skipped the read (nt_call.h bundle_span_error)
    for (int p = 0; p < np; ++p) span = span || O.end[r * 3 + p] == -4;
    if ((B.blk_off[r] & 1u) || span) {  // the scan skipped this read (layout contract)
      for (int p = 0; p < 3; ++p) {
        O.start[r * 3 + p] = -1;
        O.end[r * 3 + p] = -1;
        O.density[r * 3 + p] = 0.0;
      }
      O.flags[r] = (uint8_t)(NT_FLAG_DONE | NT_FLAG_ERR_ALIGN);
      continue;
    }
    uint32_t flags = 0u;
    int w = -2147483647 - 1;
    for (int p = 0; p < np; ++p) {
      const int s0 = O.start[r * 3 + p];
      int e0 = O.end[r * 3 + p];
      if (e0 == -2 || e0 == -3) {
        flags |= e0 == -2 ? NT_FLAG_ERR_RIGHT : NT_FLAG_ERR_WIDTH;
        e0 = -1;
        O.end[r * 3 + p] = -1;
      }
      if (s0 == -1) flags |= 1u << (NT_FLAG_NA_SHIFT + p);
      w = max(w, e0 - s0 + 1);
    }
    for (int p = np; p < 3; ++p) {
      O.start[r * 3 + p] = -1;
      O.end[r * 3 + p] = -1;
      O.density[r * 3 + p] = 0.0;
    }
    if (w >= 30) flags |= NT_FLAG_TELOMERIC;
    O.flags[r] = (uint8_t)(flags | NT_FLAG_DONE);
  }
}


// ============================================================ synthetic reads

// One thread per 32-base block: bases from the counter-based generator of
// nt_rng.h (identical on the host: nt_synth_base()).
__global__ void __launch_bounds__(256)
nt_synth_kernel(NtSynth S, uint32_t* __restrict__ planes, uint64_t n_reads) {
  const uint64_t nblk = 2 * ((S.read_len + 63) / 64);  // even block slot per read
  const uint64_t total = n_reads * nblk;
  for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < total;
       g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = g / nblk, b = g - r * nblk;
    const NtSynthRead R = nt_synth_read(S, S.first_read + r);
    uint32_t lo = 0u, hi = 0u;
    for (uint32_t i = 0; i < 32; ++i) {
      const uint64_t pos = b * 32 + i;
      if (pos >= S.read_len) break;
      const uint32_t c = nt_synth_base(S, R, S.first_read + r, pos);
      lo |= (c & 1u) << i;
      hi |= ((c >> 1) & 1u) << i;
    }
    planes[2 * g] = lo;
    planes[2 * g + 1] = hi;
  }
}

__global__ void __launch_bounds__(256)
nt_layout_kernel(uint64_t n_reads, uint64_t nblk, uint64_t read_len, uint64_t nw,
                 uint64_t* __restrict__ blk_off, uint32_t* __restrict__ len,
                 uint64_t* __restrict__ win_off) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    blk_off[r] = r * nblk;
    len[r] = (uint32_t)read_len;
    win_off[r] = r * nw;
  }
}

// ================================================================ --rc
//
// reverseComplement(dna_reads) (NanoTel.R:2219-2221) of a device-resident
// batch: out read r = the reverse complement of in read r, same block
// offsets (out of place; the host path fuses it into the packer instead).
// One wave per read (grid-stride), a lane per output plane word: new word j
// = positions 32 j .. 32 j + 31 = old positions n - 1 - 32 j - i, i.e. the
// 32 old bits from e = n - 32 j - 32 (a funnel of two old words, zero before
// the read), bit-reversed; the complement flips both plane bits (A 00 <-> T
// 11, C 01 <-> G 10).  Batches with non-ACGT letters take the host packer.
__global__ void __launch_bounds__(256)
nt_rc_kernel(const uint2* __restrict__ in, uint2* __restrict__ out, const uint64_t* __restrict__ blk_off,
             const uint32_t* __restrict__ len, uint64_t n_reads) {
  const int lane = threadIdx.x & 63;
  for (uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n_reads; r += (uint64_t)gridDim.x * 4) {
    const int64_t n = len[r];
    const uint64_t bo = blk_off[r];
    const int64_t W = (n + 31) >> 5, WB = 2 * ((n + 63) >> 6);  // words of the read, of its blocks
    for (int64_t j = lane; j < WB; j += 64) {
      const int64_t e = n - 32 * j - 32;
      const int64_t k = e >> 5;  // arithmetic: -1 for the last word of a read not a multiple of 32
      const uint32_t sh = (uint32_t)(e & 31);
      uint2 v = make_uint2(0u, 0u);  // the block padding past the read: zero, as the packer leaves it
      if (j < W) {
        const uint2 a = k >= 0 ? in[bo + k] : make_uint2(0u, 0u);
        const uint2 b = k + 1 < W ? in[bo + k + 1] : make_uint2(0u, 0u);
        const uint32_t lo = __builtin_amdgcn_alignbit(b.x, a.x, sh), hi = __builtin_amdgcn_alignbit(b.y, a.y, sh);
        const int64_t m = n - 32 * j;  // positions of the word inside the read
        const uint32_t keep = m >= 32 ? 0xFFFFFFFFu : (1u << m) - 1u;
        v = make_uint2(~__builtin_bitreverse32(lo) & keep, ~__builtin_bitreverse32(hi) & keep);
      }
      out[bo + j] = v;
    }
  }
}

// ============================================================== filter
//
// --use_filter (filter_reads / filter_density, NanoTel.R:2083-2163): one lane
// per read.  Reads shorter than 1e3 are dropped; otherwise the density of
// the union of the exact fixed=FALSE matches of the patterns inside the
// 200-base edge sub-read [70, 270) (left) or [n-270, n-70) (right, 0-based)
// must reach 0.8 * min_density, i.e. covered >= thr_count (host-computed).
// The sub-read is 8 plane words from one batch of 9 independent block loads.
__global__ void __launch_bounds__(256)
nt_filter_kernel(const NtProgram* __restrict__ prog, NtBatch B, uint8_t* __restrict__ keep,
                 uint32_t thr_count, int right_edge) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < B.n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t n = B.len[r];
    if (n < 1000u) {
      keep[r] = 0;
      continue;
    }
    ReadCtx rc;
    rc.n = n;
    rc.nblk = (int32_t)((n + 31u) >> 5);
    rc.blk = reinterpret_cast<const uint2*>(B.planes) + B.blk_off[r];
    rc.n_exc = 0;
    rc.exc_pos = nullptr;
    rc.exc_code = nullptr;
    if (B.exc_off) {
      const uint32_t e0 = B.exc_off[r], e1 = B.exc_off[r + 1];
      rc.n_exc = (int32_t)(e1 - e0);
      rc.exc_pos = B.exc_pos + e0;
      rc.exc_code = B.exc_code + e0;
    }
    const int lo = right_edge ? (int)n - 270 : 70, hi = lo + 199;
    uint32_t Lw[8], Hw[8], Vw[8];
    {
      const int bb = lo >> 5;
      const uint32_t sh = (uint32_t)(lo & 31);
      uint2 blk[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) blk[t] = bb + t < rc.nblk ? rc.blk[bb + t] : make_uint2(0u, 0u);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        Lw[t] = funnel(blk[t + 1].x, blk[t].x, sh);
        Hw[t] = funnel(blk[t + 1].y, blk[t].y, sh);
        Vw[t] = range_mask((int64_t)lo + 32 * t, lo, hi);
      }
    }
    uint32_t cov[7];
#pragma unroll
    for (int h = 0; h < 7; ++h) cov[h] = 0u;
    for (int pi = 0; pi < prog->n_pat; ++pi) {
      const NtPat& P = prog->pat[pi];
      const int m = P.m;
      uint32_t x0[7];
#pragma unroll
      for (int h = 0; h < 7; ++h) x0[h] = 0xFFFFFFFFu;
      for (int j = 0; j < m; ++j) {
        // fixed=FALSE: pattern letter j matches base c iff (code & (1 << c)) != 0
        const uint32_t code = P.code[j];
        const uint32_t t0 = (code & 1u) ? ~0u : 0u, t1 = (code & 2u) ? ~0u : 0u;
        const uint32_t t2 = (code & 4u) ? ~0u : 0u, t3 = (code & 8u) ? ~0u : 0u;
#pragma unroll
        for (int h = 0; h < 7; ++h) {
          const uint32_t Ls = funnel(Lw[h + 1], Lw[h], (uint32_t)j);
          const uint32_t Hs = funnel(Hw[h + 1], Hw[h], (uint32_t)j);
          x0[h] &= bfi(Hs, bfi(Ls, t3, t2), bfi(Ls, t1, t0)) & funnel(Vw[h + 1], Vw[h], (uint32_t)j);
        }
      }
      if (rc.n_exc) {
#pragma unroll
        for (int h = 0; h < 7; ++h) {
          uint32_t a1 = 0u;
          patch_exceptions(rc, (int64_t)lo + 32 * h, lo, hi, P, false, x0[h], a1, true);
        }
      }
#pragma unroll
      for (int h = 0; h < 7; ++h) cov[h] |= spread(x0[h], h ? x0[h - 1] : 0u, m);
    }
    uint32_t c = 0;
#pragma unroll
    for (int h = 0; h < 7; ++h) c += __builtin_popcount(cov[h] & Vw[h]);
    keep[r] = c >= thr_count ? 1 : 0;
  }
}

}  // namespace nt

// ================================================================ launchers

extern "C" {

// per-wave scan scratch words for reads with at most nw_cap windows
uint32_t nt_dev_wave_words(int single, int n_hits, int np, uint32_t nw_cap) {
  const uint32_t w = (single ? 0u : (uint32_t)n_hits * 64u) + (uint32_t)(np < 2 ? 2 : np) * (nw_cap + 1u);
  return (w + 3u) & ~3u;  // 16-byte aligned per-wave areas (uint2 running counts)
}

// uint64 words of the telomeric-bitmask scratch for a batch
uint64_t nt_dev_tmask_words(uint64_t total_windows, uint64_t n_reads, int np) {
  return ((total_windows >> 6) + 2 * n_reads + 2) * 8 * (uint64_t)np;  // aux_base blocks
}

// (single, lds, one-hot, compile-time m): m = 6 covers TTAGGG-style motifs
// AOT scan variants: (pattern set, LDS?, single, one-hot, m == 6)
using nt::GenericSet;
using nt::RtOneHot;
using nt::RtTable;
using nt::SingleSet;
#define NT_SCAN_VARIANTS(X)                        \
  X(SingleSet<RtOneHot<6>>, true, 1, 1, 1)         \
  X(SingleSet<RtTable<6>>, true, 1, 0, 1)          \
  X(SingleSet<RtOneHot<0>>, true, 1, 1, 0)         \
  X(SingleSet<RtTable<0>>, true, 1, 0, 0)          \
  X(SingleSet<RtTable<0>>, false, 1, -1, -1)       \
  X(GenericSet, true, 0, -1, -1)                   \
  X(GenericSet, false, 0, -1, -1)

hipError_t nt_dev_set_lds_limit(uint32_t bytes) {
  hipError_t e = hipSuccess;
#define NT_ATTR(S, G, SI, O, M)                                                                \
  if (G && e == hipSuccess)                                                                    \
    e = hipFuncSetAttribute((const void*)nt::nt_scan_kernel<S, G>,                             \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  NT_SCAN_VARIANTS(NT_ATTR)
#undef NT_ATTR
  return e;
}

// single: 1 pattern, no TVR; one: one-hot letters; m6: 6 letters
hipError_t nt_dev_launch(const NtProgram* prog, const uint32_t* thr, const NtBatch* B,
                         const NtOut* O, uint64_t* tmask, unsigned long long* queue,
                         uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic,
                         int single, int one, int m6, int lds, uint32_t wave_words, uint32_t* gscr,
                         int grid, hipStream_t stream) {
  const size_t lds_bytes = lds ? (size_t)wave_words * 4u * nt::kNWaves : 0;
  bool done = false;
#define NT_LAUNCH(S, G, SI, O_, M)                                                             \
  if (!done && single == SI && lds == (int)G && (O_ < 0 || one == O_) && (M < 0 || m6 == M)) { \
    hipLaunchKernelGGL((nt::nt_scan_kernel<S, G>), dim3(grid), dim3(nt::kWG), lds_bytes,       \
                       stream, prog, thr, *B, *O, tmask, queue, len_lo, len_hi, claim, nstatic, wave_words,    \
                       gscr);                                                                  \
    done = true;                                                                               \
  }
  NT_SCAN_VARIANTS(NT_LAUNCH)
#undef NT_LAUNCH
  if (!done) return hipErrorInvalidValue;
  return hipGetLastError();
}

// resident 256-thread blocks per CU of the scan variant (grid sizing)
int nt_dev_scan_blocks_per_cu(int single, int one, int m6, int lds, size_t lds_bytes) {
  int nb = 0;
  bool done = false;
#define NT_OCC(S, G, SI, O_, M)                                                                \
  if (!done && single == SI && lds == (int)G && (O_ < 0 || one == O_) && (M < 0 || m6 == M)) { \
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, nt::nt_scan_kernel<S, G>, nt::kWG,   \
                                                     lds_bytes) != hipSuccess)                 \
      nb = 0;                                                                                  \
    done = true;                                                                               \
  }
  NT_SCAN_VARIANTS(NT_OCC)
#undef NT_OCC
  return nb;
}

hipError_t nt_dev_launch_call(const NtProgram* prog, const NtBatch* B, const NtOut* O,
                              const uint64_t* tmask, const uint32_t* thr, uint32_t thr_size, int fix_last,
                              int long_tvr, int call_grid, hipStream_t stream) {
  if (long_tvr)
    hipLaunchKernelGGL(nt::nt_call_kernel_long, dim3(call_grid), dim3(256), 0, stream, prog, *B, *O, tmask, thr,
                       thr_size, fix_last);
  else
    hipLaunchKernelGGL(nt::nt_call_kernel, dim3(call_grid), dim3(256), 0, stream, prog, *B, *O, tmask, thr,
                       thr_size, fix_last);
  return hipGetLastError();
}

hipError_t nt_dev_launch_combine(const NtBatch* B, const NtOut* O, int np, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(nt::nt_call_combine_kernel, dim3(grid), dim3(256), 0, stream, *B, *O, np);
  return hipGetLastError();
}

hipError_t nt_dev_launch_rc(const uint32_t* in, uint32_t* out, const uint64_t* blk_off, const uint32_t* len,
                            uint64_t n_reads, int cu_count, hipStream_t stream) {
  uint64_t grid = (n_reads + 3) / 4;
  if (grid > (uint64_t)cu_count * 32) grid = (uint64_t)cu_count * 32;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(nt::nt_rc_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, reinterpret_cast<const uint2*>(in),
                     reinterpret_cast<uint2*>(out), blk_off, len, n_reads);
  return hipGetLastError();
}

hipError_t nt_dev_launch_filter(const NtProgram* prog, const NtBatch* B, uint8_t* keep,
                                uint32_t thr_count, int right_edge, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(nt::nt_filter_kernel, dim3(grid), dim3(256), 0, stream, prog, *B, keep, thr_count,
                     right_edge);
  return hipGetLastError();
}

hipError_t nt_dev_launch_synth(const NtSynth* S, uint32_t* planes, uint64_t n_reads,
                               hipStream_t stream) {
  const uint64_t nblk = 2 * ((S->read_len + 63) / 64);
  uint64_t total = n_reads * nblk;
  uint64_t grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(nt::nt_synth_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, *S, planes,
                     n_reads);
  return hipGetLastError();
}

hipError_t nt_dev_launch_uniform_layout(uint64_t n_reads, uint64_t nblk, uint64_t read_len,
                                        uint64_t nw, uint64_t* blk_off, uint32_t* len,
                                        uint64_t* win_off, hipStream_t stream) {
  uint64_t grid = (n_reads + 255) / 256;
  if (grid > 65536) grid = 65536;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(nt::nt_layout_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, n_reads,
                     nblk, read_len, nw, blk_off, len, win_off);
  return hipGetLastError();
}

}  // extern "C"
