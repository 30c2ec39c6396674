// nt_device.h -- gfx950 device primitives for the NanoTel scan (bit-sliced
// matching on 2-bit planes, coverage spreading, exception fix-ups).
#pragma once
#ifndef __HIPCC_RTC__  // hiprtc (nt_jit.cpp) provides the HIP device runtime itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "nt_common.h"

namespace nt {

constexpr int kWave = 64;
constexpr int kWG = 256;
constexpr int kNWaves = kWG / kWave;
constexpr int kOwned = kWave - 1;  // words owned per wave-chunk (lane 0 is the carry helper)

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  return (m & a) | (~m & b);  // v_bfi_b32
}

// (hi:lo) >> s, low 32 bits (v_alignbit_b32), s in [0, 31]
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
  return __builtin_amdgcn_alignbit(hi, lo, s);
}

// Bits i of a 32-position word starting at `base` with base+i in [vlo, vhi].
__device__ __forceinline__ uint32_t range_mask(int64_t base, int64_t vlo, int64_t vhi) {
  int64_t lo = vlo - base, hi = vhi - base;
  if (hi < 0 || lo > 31 || lo > hi) return 0u;
  if (lo < 0) lo = 0;
  if (hi > 31) hi = 31;
  const uint32_t mhi = hi == 31 ? 0xFFFFFFFFu : ((1u << (uint32_t)(hi + 1)) - 1u);
  const uint32_t mlo = ~((1u << (uint32_t)lo) - 1u);
  return mhi & mlo;
}

struct ReadCtx {
  const uint2* blk;         // this read's plane blocks
  int64_t n;                // length
  int32_t nblk;             // ceil(n/32)
  const uint32_t* exc_pos;  // this read's exceptions (sorted), may be null
  const uint8_t* exc_code;
  int32_t n_exc;
};

__device__ __forceinline__ uint2 load_blk(const ReadCtx& rc, int64_t b) {
  return (b >= 0 && b < rc.nblk) ? rc.blk[b] : make_uint2(0u, 0u);
}

// The same, but the load itself is unconditional (clamped address, result
// zeroed afterwards): straight-line loads let hipcc count them with partial
// s_waitcnt vmcnt(N) instead of draining the prefetch ring with vmcnt(0).
__device__ __forceinline__ uint2 load_blk_nc(const ReadCtx& rc, int b) {
  const int bc = b < 0 ? 0 : (b >= rc.nblk ? rc.nblk - 1 : b);
  const uint2 x = rc.blk[bc];
  const bool ok = (b >= 0) & (b < rc.nblk);
  return make_uint2(ok ? x.x : 0u, ok ? x.y : 0u);
}

// Planes of the 32 positions [p, p+31] (any p; out-of-read positions read 0).
__device__ __forceinline__ void plane_at(const ReadCtx& rc, int64_t p, uint32_t& L, uint32_t& H) {
  const int64_t b = p >> 5;  // floor for negative p
  const uint32_t off = (uint32_t)(p & 31);
  const uint2 x = load_blk(rc, b), y = load_blk(rc, b + 1);
  L = funnel(y.x, x.x, off);
  H = funnel(y.y, x.y, off);
}

// Bit-sliced approximate matching of one pattern at 32 consecutive starts.
// Inputs: planes (L,H) and validity (V) of positions [base, base+63] as two
// words.  tm[j][c]: all-ones iff pattern letter j matches subject base c
// (A,C,G,T).  Invalid positions (outside the subject / window) count as
// mismatches -- Biostrings' out-of-bound rule.  a0 = starts with 0
// mismatches, a1 = <= 1.  kValid=false: every position is known valid.
template <bool kValid>
__device__ __forceinline__ void hits_step(uint32_t L0, uint32_t L1, uint32_t H0, uint32_t H1,
                                          uint32_t V0, uint32_t V1, const uint32_t* __restrict__ t,
                                          int j, uint32_t& x0, uint32_t& x1) {
  const uint32_t Ls = funnel(L1, L0, (uint32_t)j);
  const uint32_t Hs = funnel(H1, H0, (uint32_t)j);
  uint32_t q = bfi(Hs, bfi(Ls, t[3], t[2]), bfi(Ls, t[1], t[0]));
  if (kValid) q &= funnel(V1, V0, (uint32_t)j);
  x1 = (x1 & q) | x0;
  x0 &= q;
}

// kM > 0: pattern length known at compile time (fully unrolled, masks hoisted).
template <bool kValid, int kM = 0>
__device__ __forceinline__ void hits32(uint32_t L0, uint32_t L1, uint32_t H0, uint32_t H1,
                                       uint32_t V0, uint32_t V1,
                                       const uint32_t (*__restrict__ tm)[4], int m, uint32_t& a0,
                                       uint32_t& a1) {
  uint32_t x0 = 0xFFFFFFFFu, x1 = 0xFFFFFFFFu;
  if (kM) {
#pragma unroll
    for (int j = 0; j < kM; ++j) hits_step<kValid>(L0, L1, H0, H1, V0, V1, tm[j], j, x0, x1);
  } else {
    for (int j = 0; j < m; ++j) hits_step<kValid>(L0, L1, H0, H1, V0, V1, tm[j], j, x0, x1);
  }
  a0 = x0;
  a1 = x1;
}

// Coverage of 32 positions from the hit-start words of this and the previous
// 32 starts: C[p] = OR_{j<m} H[p-j]  (trimmed views, IRanges::reduce runs).
template <int kM = 0>
__device__ __forceinline__ uint32_t spread(uint32_t h, uint32_t hprev, int m) {
  uint32_t c = h;
  if (kM) {
#pragma unroll
    for (int j = 1; j < kM; ++j) c |= funnel(h, hprev, (uint32_t)(32 - j));
  } else {
    for (int j = 1; j < m; ++j) c |= funnel(h, hprev, (uint32_t)(32 - j));
  }
  return c;
}

// The same for m up to 64 (TVRs): hit words of this and the two previous 32
// starts.
template <int kM = 0>
__device__ __forceinline__ uint32_t spread_long(uint32_t h, uint32_t hp, uint32_t hpp, int m) {
  uint32_t c = h;
  if constexpr (kM > 0) {
#pragma unroll
    for (int j = 1; j < kM && j <= 32; ++j) c |= funnel(h, hp, (uint32_t)(32 - j));
#pragma unroll
    for (int j = 33; j < kM; ++j) c |= funnel(hp, hpp, (uint32_t)(64 - j));
  } else {
    for (int j = 1; j < m && j <= 32; ++j) c |= funnel(h, hp, (uint32_t)(32 - j));
    for (int j = 33; j < m; ++j) c |= funnel(hp, hpp, (uint32_t)(64 - j));
  }
  return c;
}

// ---------------------------------------------------------------- exceptions

__device__ __forceinline__ int32_t exc_lower_bound(const ReadCtx& rc, int64_t x) {
  int32_t lo = 0, hi = rc.n_exc;
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if ((int64_t)rc.exc_pos[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Biostrings DNA code of read position pos (0 <= pos < n).
__device__ __forceinline__ uint32_t code_at(const ReadCtx& rc, int64_t pos) {
  if (rc.n_exc) {
    const int32_t i = exc_lower_bound(rc, pos);
    if (i < rc.n_exc && (int64_t)rc.exc_pos[i] == pos) return rc.exc_code[i];
  }
  const uint2 b = rc.blk[pos >> 5];
  const uint32_t s = (uint32_t)(pos & 31);
  return 1u << (((b.x >> s) & 1u) | (((b.y >> s) & 1u) << 1));
}

// Mismatch count (capped at 2) of pattern P at start s; positions outside
// [vlo, vhi] count as mismatches.  eq (edge steps, always fixed=TRUE) or a
// fixed pattern: code equality; otherwise IUPAC bit-set AND (fixed=FALSE).
// iupac: fixed=FALSE whatever the pattern (the --use_filter matches).
__device__ __forceinline__ int mism_generic(const ReadCtx& rc, const NtPat& P, bool eq, int64_t s,
                                            int64_t vlo, int64_t vhi, bool iupac = false) {
  eq = eq || (P.fixed && !iupac);
  int nm = 0;
  for (int j = 0; j < P.m && nm < 2; ++j) {
    const int64_t pos = s + j;
    if (pos < vlo || pos > vhi) { ++nm; continue; }
    const uint32_t c = code_at(rc, pos);
    const uint32_t pc = P.code[j];
    if (eq ? (c != pc) : ((c & pc) == 0u)) ++nm;
  }
  return nm;
}

// Re-evaluate every start of the word [base, base+31] whose pattern window
// touches an exception letter.  Biostrings start range for k=1 is [vlo-1,
// vhi-m+2] (m>=2) or [vlo, vhi] (m==1); for k=0 [vlo, vhi-m+1].
__device__ __forceinline__ void patch_exceptions(const ReadCtx& rc, int64_t base, int64_t vlo,
                                              int64_t vhi, const NtPat& P, bool eq, uint32_t& a0,
                                              uint32_t& a1, bool iupac = false) {
  const int m = P.m;
  const int64_t xlo = base > vlo ? base : vlo;
  int64_t xhi = base + 31 + m - 1;
  if (xhi > vhi) xhi = vhi;
  if (xlo > xhi) return;
  uint32_t dirty = 0u;
  for (int32_t i = exc_lower_bound(rc, xlo); i < rc.n_exc && (int64_t)rc.exc_pos[i] <= xhi; ++i) {
    const int64_t x = rc.exc_pos[i];
    dirty |= range_mask(base, x - m + 1, x);
  }
  const int64_t k1lo = m <= 1 ? vlo : vlo - 1, k1hi = m <= 1 ? vhi : vhi - m + 2;
  while (dirty) {
    const int b = __builtin_ctz(dirty);
    dirty &= dirty - 1u;
    const int64_t s = base + b;
    const int nm = mism_generic(rc, P, eq, s, vlo, vhi, iupac);
    const uint32_t bit = 1u << b;
    a0 = (nm == 0 && s >= vlo && s <= vhi - m + 1) ? (a0 | bit) : (a0 & ~bit);
    a1 = (nm <= 1 && s >= k1lo && s <= k1hi) ? (a1 | bit) : (a1 & ~bit);
  }
}

// Hits of pattern P at the 32 starts [base, base+31] against positions
// restricted to [vlo, vhi] (plane data fetched from global memory).
__device__ __forceinline__ void hits_at(const ReadCtx& rc, const NtPat& P, bool eq, int64_t base,
                                        int64_t vlo, int64_t vhi, uint32_t& a0, uint32_t& a1) {
  uint32_t L0, H0, L1, H1;
  plane_at(rc, base, L0, H0);
  plane_at(rc, base + 32, L1, H1);
  const uint32_t V0 = range_mask(base, vlo, vhi), V1 = range_mask(base + 32, vlo, vhi);
  hits32<true>(L0, L1, H0, H1, V0, V1, eq ? P.tm_eq : P.tm_scan, P.m, a0, a1);
  if (P.m <= 1) a1 &= V0;
  if (rc.n_exc) patch_exceptions(rc, base, vlo, vhi, P, eq, a0, a1);
}

// ------------------------------------------------------------ wave helpers

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ int64_t split_window_count(int64_t n, int L) {
  if (n <= 0 || L <= 0) return 0;
  int64_t c = (n - 1) / L + 1;
  const int64_t last_start = 1 + (c - 1) * (int64_t)L;
  if ((double)(n - last_start) < (double)L / 2.0) c -= 1;
  return c;
}

}  // namespace nt
