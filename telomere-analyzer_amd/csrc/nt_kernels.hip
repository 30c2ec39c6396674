// nt_kernels.hip -- NanoTel hot path on MI355X (gfx950 / CDNA4).
//
// One fused kernel, one wave per read (grid-stride over reads):
//
//  scan  (HBM-bound): each lane owns one 32-base word of the read; the wave
//     streams the read's 2-bit planes (coalesced 8-byte loads, a 2-deep
//     prefetch ring), runs the bit-sliced matchPattern of every pattern at
//     the 32 starts of each word (exact and <=1 mismatch in one pass,
//     Biostrings' out-of-bound rule), builds coverage = OR of shifted hit
//     words (trim + IRanges::reduce) and accumulates covered bases per
//     subseq_length window with LDS atomics (analyze_subtelos /
//     get_sub_density, NanoTel.R:717-766, 449-468).  Window counts (uint16)
//     and matchPattern hit counts go to HBM.
//
//  call  (latency-bound, no HBM traffic beyond L2/MALL re-reads): the same
//     wave calls the telomere of every pass from the LDS window counts:
//     telomeric-window bitmask by ballot, find_telo_position / _wraper run
//     scans with fp64 sums in R's order, get_accurate_start/end,
//     find_left/right_telo, search_left/right_patterns (NanoTel.R:973-1155,
//     1692-1764, 843-959, 496-697) and the row densities.  Coverage near the
//     boundaries is recomputed from the planes ("regions").  While a wave
//     calls, the other waves of its CU keep streaming, so the calling latency
//     hides behind the scan.
//
// No MFMA: integer/bit work bound by HBM bandwidth.
#include <hip/hip_runtime.h>

#include "nt_common.h"
#include "nt_device.h"
#include "nt_rng.h"

namespace nt {

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// floor(p / L), 0 <= p < 2^31 (multiply-shift, exact; see nt_compile)
__device__ __forceinline__ int div_l(const NtProgram* prog, int p) {
  if (prog->div32_m == 0u) return p;  // L == 1
  return (int)(__umulhi((uint32_t)p, prog->div32_m) >> prog->div32_s);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ================================================================= scan

// Hits of one pattern at this lane's 32 starts: exact a0, <=1 mismatch a1.
template <bool kValid, int kM = 0>
__device__ __forceinline__ void word_hits(const ReadCtx& rc, const NtPat& P, int base, uint2 b0,
                                          uint2 b1, uint32_t V0, uint32_t V1, uint32_t& a0,
                                          uint32_t& a1) {
  hits32<kValid, kM>(b0.x, b1.x, b0.y, b1.y, V0, V1, P.tm_scan, P.m, a0, a1);
  if (kValid && P.m <= 1) a1 &= V0;
  if (rc.n_exc) patch_exceptions(rc, base, 0, rc.n - 1, P, false, a0, a1);
}

// Add coverage popcounts of this lane's word (positions [p0, p0+31]) to the
// window counters of up to three passes; window k = min(p / L, nw - 1)
// (split_telo's last window absorbs the tail).
__device__ __forceinline__ void windows_add(const NtProgram* prog, uint32_t* cnt, int nw, int np,
                                            int L, int p0, uint32_t c0, uint32_t c1, uint32_t c2) {
  if (!(c0 | c1 | c2)) return;
  const int k0 = min(div_l(prog, p0), nw - 1), k1 = min(div_l(prog, p0 + 31), nw - 1);
  if (L >= 32 || k0 == k1) {
    // at most two windows
    const uint32_t lom = k0 == k1 ? 0xFFFFFFFFu : ((1u << (uint32_t)((k0 + 1) * L - p0)) - 1u);
    const uint32_t cv[3] = {c0, c1, c2};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if (p >= np || !cv[p]) continue;
      const uint32_t lo = __builtin_popcount(cv[p] & lom), hi = __builtin_popcount(cv[p] & ~lom);
      if (lo) atomicAdd(&cnt[p * nw + k0], lo);
      if (hi) atomicAdd(&cnt[p * nw + k1], hi);
    }
    return;
  }
  for (int k = k0; k <= k1; ++k) {
    const int lo = k * L > p0 ? k * L - p0 : 0;
    const int hi = k == k1 ? 31 : (k + 1) * L - 1 - p0;
    const uint32_t m = (hi >= 31 ? 0xFFFFFFFFu : ((1u << (uint32_t)(hi + 1)) - 1u)) &
                       (0xFFFFFFFFu << (uint32_t)lo);
    const uint32_t cv[3] = {c0, c1, c2};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      if (p >= np) continue;
      const uint32_t v = __builtin_popcount(cv[p] & m);
      if (v) atomicAdd(&cnt[p * nw + k], v);
    }
  }
}

// One 63-word wave chunk.  Lane l owns offset word w = c0 + l - 1 (positions
// [32(w-1), 32(w-1)+31]); lane 0 recomputes the word before the chunk so that
// lanes 1..63 get their carry-in hit starts by a lane shift.  b1: this lane's
// block w (prefetched); carry: block c0-2 (lane 62's block of the previous
// chunk) for lane 0.
template <bool kSingle, bool kValid, int kM>
__device__ __forceinline__ void scan_chunk(const NtProgram* __restrict__ prog, const ReadCtx& rc,
                                           int c0, int lane, int np, int nw, uint2 b1, uint2 carry,
                                           uint32_t* cnt, uint32_t* hitacc, uint32_t& acc0,
                                           uint32_t& acc1) {
  const int n = (int)rc.n, L = prog->L;
  const int w = c0 + lane - 1;
  const int base = 32 * (w - 1);
  const bool owned = lane >= 1 && w <= rc.nblk;
  uint2 b0;
  b0.x = __shfl_up(b1.x, 1, kWave);
  b0.y = __shfl_up(b1.y, 1, kWave);
  if (lane == 0) b0 = carry;
  uint32_t V0 = 0xFFFFFFFFu, V1 = 0xFFFFFFFFu;
  if (kValid) {
    V0 = range_mask(base, 0, n - 1);
    V1 = range_mask(base + 32, 0, n - 1);
  }
  uint32_t cv0 = 0u, cv1 = 0u, cv2 = 0u;
  const int n_pat = kSingle ? 1 : prog->n_pat;
  for (int p = 0; p < n_pat; ++p) {
    const NtPat& P = prog->pat[p];
    uint32_t a0, a1;
    word_hits<kValid, kM>(rc, P, base, b0, b1, V0, V1, a0, a1);
    if (kSingle) {
      if (owned) {
        acc0 += __builtin_popcount(a0);
        acc1 += __builtin_popcount(a1);
      }
    } else if (owned) {
      if (a0) atomicAdd(&hitacc[p * kWave + lane], (uint32_t)__builtin_popcount(a0));
      if (a1) atomicAdd(&hitacc[(n_pat + p) * kWave + lane], (uint32_t)__builtin_popcount(a1));
    }
    cv0 |= spread<kM>(a0, __shfl_up(a0, 1, kWave), P.m);
    cv1 |= spread<kM>(a1, __shfl_up(a1, 1, kWave), P.m);
  }
  if (!kSingle && np == 3) {
    cv2 = cv1;
    for (int t = 0; t < prog->n_tvr; ++t) {
      const NtPat& P = prog->tvr[t];
      uint32_t a0, a1;
      word_hits<kValid>(rc, P, base, b0, b1, V0, V1, a0, a1);
      if (owned && a0) atomicAdd(&hitacc[(2 * n_pat + t) * kWave + lane], (uint32_t)__builtin_popcount(a0));
      cv2 |= spread(a0, __shfl_up(a0, 1, kWave), P.m);
    }
  }
  if (owned && w >= 1 && nw > 0) {
    if (kValid) {
      cv0 &= V0;
      cv1 &= V0;
      cv2 &= V0;
    }
    windows_add(prog, cnt, nw, kSingle ? 2 : np, L, base, cv0, cv1, cv2);
  }
}

template <bool kSingle, int kM>
__device__ __forceinline__ void scan_read(const NtProgram* __restrict__ prog, const ReadCtx& rc,
                                          int lane, int np, int nw, uint32_t* cnt,
                                          uint32_t* hitacc, uint32_t& acc0, uint32_t& acc1) {
  const int n = (int)rc.n, nblk = rc.nblk;
  // 2-deep prefetch ring of this lane's block for the next chunks
  uint2 nx1 = load_blk_nc(rc, 0 + lane - 1), nx2 = load_blk_nc(rc, kOwned + lane - 1);
  uint2 carry = make_uint2(0u, 0u);
  for (int c0 = 0; c0 <= nblk; c0 += kOwned) {
    const uint2 b1 = nx1;
    nx1 = nx2;
    nx2 = load_blk_nc(rc, c0 + 2 * kOwned + lane - 1);
    // interior chunk: every lane's positions [base, base+63] inside the read
    if (c0 >= 2 && 32 * c0 + 32 * kWave <= n)
      scan_chunk<kSingle, false, kM>(prog, rc, c0, lane, np, nw, b1, carry, cnt, hitacc, acc0, acc1);
    else
      scan_chunk<kSingle, true, kM>(prog, rc, c0, lane, np, nw, b1, carry, cnt, hitacc, acc0, acc1);
    carry.x = __shfl(b1.x, kOwned - 1, kWave);
    carry.y = __shfl(b1.y, kOwned - 1, kWave);
  }
}

// ================================================================= call

struct Pos {
  int s, e;
};

// A "region": coverage of 63*32 = 2016 consecutive positions [P0, P0+2015]
// recomputed from the planes, one 32-bit word per lane (lanes 1..63).  S/E:
// range-start / range-end marks of the pass's range set (run starts / ends of
// the reduced coverage, or raw view starts / ends for P1 with a single fixed
// pattern, NanoTel.R:349-355).
struct Region {
  int P0;
  uint32_t cov, S, E;
};

constexpr int kRegionSpan = 32 * kOwned;
constexpr int kNoRegion = INT_MIN;

struct CallCtx {
  ReadCtx rc;
  const NtProgram* prog;
  const uint32_t* cnt;  // this pass's window counts
  const uint64_t* tm;   // telomeric window bitmask
  int n, nw, nmw;
  int L;
  int k;         // 0 for P1, 1 for P2/P3
  bool use_tvr;  // P3
  bool raw;      // P1 raw views
  int lane;
  Region R0, R1;  // two-entry region cache
  int lru;
};

__device__ __forceinline__ int wstart(const CallCtx& c, int i) { return 1 + i * c.L; }
__device__ __forceinline__ int wend(const CallCtx& c, int i) { return i == c.nw - 1 ? c.n : wstart(c, i) + c.L - 1; }
__device__ __forceinline__ int wcount(const CallCtx& c, int i) { return uni((int)c.cnt[i]); }
__device__ __forceinline__ double wdens(const CallCtx& c, int i) {
  return (double)wcount(c, i) / (double)(wend(c, i) - wstart(c, i) + 1);
}

// --------------------------------------------------------- window bitmask

__device__ __forceinline__ uint64_t tword(const CallCtx& c, int wi, bool inv) {
  const uint64_t x = c.tm[wi];
  const uint64_t u = ((uint64_t)(uint32_t)uni((int)(uint32_t)(x >> 32)) << 32) | (uint32_t)uni((int)(uint32_t)x);
  return inv ? ~u : u;
}
__device__ __forceinline__ bool tbit(const CallCtx& c, int i) { return (tword(c, i >> 6, false) >> (i & 63)) & 1ull; }

__device__ __forceinline__ int next_set(const CallCtx& c, int pos, bool inv) {
  if (pos >= c.nw) return c.nw;
  int wi = pos >> 6;
  uint64_t x = tword(c, wi, inv) & (~0ull << (pos & 63));
  for (;;) {
    if (x) {
      const int r = (wi << 6) + __builtin_ctzll(x);
      return r < c.nw ? r : c.nw;
    }
    if (++wi >= c.nmw) return c.nw;
    x = tword(c, wi, inv);
  }
}

__device__ __forceinline__ int prev_set(const CallCtx& c, int pos, bool inv) {
  if (pos < 0) return -1;
  if (pos >= c.nw) pos = c.nw - 1;
  int wi = pos >> 6;
  const uint32_t b = (uint32_t)(pos & 63);
  uint64_t x = tword(c, wi, inv) & (b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull));
  for (;;) {
    if (x) return (wi << 6) + 63 - __builtin_clzll(x);
    if (--wi < 0) return -1;
    x = tword(c, wi, inv);
  }
}

// ---------------------------------------------------------------- regions

__device__ __forceinline__ Region make_region(const CallCtx& c, int P0) {
  const ReadCtx& rc = c.rc;
  const int q = P0 + 32 * (c.lane - 1);  // this lane's 32 positions / starts
  const NtProgram* prog = c.prog;
  uint32_t cov = 0u, raw = 0u;
  for (int p = 0; p < prog->n_pat; ++p) {
    const NtPat& P = prog->pat[p];
    uint32_t a0, a1;
    hits_at(rc, P, false, q, 0, rc.n - 1, a0, a1);
    const uint32_t h = c.k ? a1 : a0;
    if (p == 0) raw = a0;
    cov |= spread(h, __shfl_up(h, 1, kWave), P.m);
  }
  if (c.use_tvr) {
    for (int t = 0; t < prog->n_tvr; ++t) {
      const NtPat& P = prog->tvr[t];
      uint32_t a0, a1;
      hits_at(rc, P, false, q, 0, rc.n - 1, a0, a1);
      cov |= spread(a0, __shfl_up(a0, 1, kWave), P.m);
    }
  }
  cov &= range_mask(q, 0, rc.n - 1);
  const uint32_t cprev = __shfl_up(cov, 1, kWave), cnext = __shfl_down(cov, 1, kWave);
  const uint32_t rprev = __shfl_up(raw, 1, kWave);
  Region R;
  R.P0 = P0;
  R.cov = cov;
  if (c.raw) {
    // raw views of pattern 0: starts = hit starts, ends = starts + m - 1
    const int m = prog->pat[0].m;
    R.S = raw;
    R.E = m > 1 ? funnel(raw, rprev, (uint32_t)(33 - m)) : raw;
  } else {
    R.S = cov & ~((cov << 1) | (cprev >> 31));
    R.E = cov & ~((cov >> 1) | (cnext << 31));
  }
  if (c.lane == 0) R.cov = R.S = R.E = 0u;  // helper lane
  return R;
}

// A cached region containing [x, y] (y - x < kRegionSpan - 64).
__device__ __forceinline__ Region region_for(CallCtx& c, int x, int y) {
  if (c.R0.P0 != kNoRegion && x >= c.R0.P0 && y <= c.R0.P0 + kRegionSpan - 1) {
    c.lru = 1;
    return c.R0;
  }
  if (c.R1.P0 != kNoRegion && x >= c.R1.P0 && y <= c.R1.P0 + kRegionSpan - 1) {
    c.lru = 0;
    return c.R1;
  }
  // new region: x sits ~1/4 into it (32-aligned so lanes load whole blocks)
  int P0 = x - (kRegionSpan / 4);
  P0 = (P0 >> 5) << 5;
  if (y > P0 + kRegionSpan - 1) P0 = (x >> 5) << 5;
  const Region R = make_region(c, P0);
  if (c.lru == 0) { c.R0 = R; c.lru = 1; }
  else { c.R1 = R; c.lru = 0; }
  return R;
}

// |coverage ∩ [x, y]| for 0-based positions, any span (region-sized pieces).
__device__ __forceinline__ int region_count(CallCtx& c, int x, int y) {
  int tot = 0;
  while (x <= y) {
    const int y2 = (y - x > kRegionSpan - 128) ? x + kRegionSpan - 129 : y;
    const Region R = region_for(c, x, y2);
    const int q = R.P0 + 32 * (c.lane - 1);
    const uint32_t w = c.lane ? (R.cov & range_mask(q, x, y2)) : 0u;
    tot += (int)wave_sum_u32((uint32_t)__builtin_popcount(w));
    x = y2 + 1;
  }
  return uni(tot);
}

// sum of window counts k in [ka, kb]
__device__ __forceinline__ int count_sum(const CallCtx& c, int ka, int kb) {
  uint32_t acc = 0;
  for (int i = ka + c.lane; i <= kb; i += kWave) acc += c.cnt[i];
  return uni((int)wave_sum_u32(acc));
}

// sum(width(intersect(IRanges(a1, b1), ranges))): window counts for whole
// windows, recomputed coverage for the partial windows at the two ends.
__device__ __forceinline__ int range_count(CallCtx& c, int a1, int b1) {
  const int a = (a1 < 1 ? 1 : a1) - 1, b = (b1 > c.n ? c.n : b1) - 1;
  if (a > b) return 0;
  if (c.nw == 0) return region_count(c, a, b);
  const int L = c.L;
  const int ka = min(div_l(c.prog, a), c.nw - 1), kb = min(div_l(c.prog, b), c.nw - 1);
  const int ws_a = ka * L, we_b = kb == c.nw - 1 ? c.n - 1 : (kb + 1) * L - 1;
  if (ka == kb) {
    if (a == ws_a && b == we_b) return wcount(c, ka);
    return region_count(c, a, b);
  }
  const int we_a = (ka + 1) * L - 1, ws_b = kb * L;
  int tot = a == ws_a ? wcount(c, ka) : region_count(c, a, we_a);
  if (kb > ka + 1) tot += count_sum(c, ka + 1, kb - 1);
  tot += b == we_b ? wcount(c, kb) : region_count(c, ws_b, b);
  return tot;
}

__device__ __forceinline__ double sub_density(CallCtx& c, int s, int e) {
  return (double)range_count(c, s, e) / (double)(e - s + 1);
}

// min(start(ranges)) with start in [a1, b1] (span <= 100); fallback if none.
__device__ __forceinline__ int min_start_in(CallCtx& c, int a1, int b1, int fallback) {
  int a = a1 - 1, b = b1 - 1;
  if (a < 0) a = 0;
  if (b > c.n - 1) b = c.n - 1;
  if (a > b) return fallback;
  const Region R = region_for(c, a, b);
  const int q = R.P0 + 32 * (c.lane - 1);
  const uint32_t w = c.lane ? (R.S & range_mask(q, a, b)) : 0u;
  const uint64_t bal = __ballot(w != 0u);
  if (!bal) return fallback;
  const int l = __builtin_ctzll(bal);
  const uint32_t wl = (uint32_t)uni((int)__shfl(w, l, kWave));
  return R.P0 + 32 * (l - 1) + __builtin_ctz(wl) + 1;
}

// max(end(ranges)) with end in [a1, b1] (span <= 100); fallback if none.
__device__ __forceinline__ int max_end_in(CallCtx& c, int a1, int b1, int fallback) {
  int a = a1 - 1, b = b1 - 1;
  if (a < 0) a = 0;
  if (b > c.n - 1) b = c.n - 1;
  if (a > b) return fallback;
  const Region R = region_for(c, a, b);
  const int q = R.P0 + 32 * (c.lane - 1);
  const uint32_t w = c.lane ? (R.E & range_mask(q, a, b)) : 0u;
  const uint64_t bal = __ballot(w != 0u);
  if (!bal) return fallback;
  const int l = 63 - __builtin_clzll(bal);
  const uint32_t wl = (uint32_t)uni((int)__shfl(w, l, kWave));
  return R.P0 + 32 * (l - 1) + (31 - __builtin_clz(wl)) + 1;
}

// -------------------------------------------------------- A8 / A11

// find_telo_position (NanoTel.R:973-1077) on the window bitmask.
__device__ __forceinline__ Pos find_telo_position(const CallCtx& c, int min_in_a_row, double thr) {
  int pos = 0, found = -1, start = -1;
  for (;;) {
    const int r = next_set(c, pos, false);
    if (r >= c.nw) break;
    const int q = next_set(c, r, true) - 1;  // last window of the telomeric run
    if (q - r + 1 >= min_in_a_row) {
      double score = 0.0;
      for (int j = r; j <= q; ++j) {
        score = score + wdens(c, j);
        if (j - r + 1 >= min_in_a_row && score >= thr) { found = j; break; }
      }
      if (found >= 0) { start = wstart(c, r); break; }
    }
    pos = q + 1;
  }
  if (found < 0) return Pos{-1, -1};
  const int ep = found + 2;  // end_position, 1-based
  int end = -1;
  if (ep >= c.nw - min_in_a_row + 1) {
    if (c.nw > ep) {
      const int j = prev_set(c, c.nw - 1, false);
      end = (j >= ep) ? wend(c, j) : wend(c, ep - 1);
    } else {
      end = wend(c, c.nw - 1);
    }
  } else {
    // for (i in nrow:end_position): windows nw-1 .. ep-1 (0-based)
    const int lo = ep - 1;
    bool hit = false;
    int p2 = c.nw - 1;
    for (;;) {
      const int q = prev_set(c, p2, false);
      if (q < lo) break;
      const int rr = prev_set(c, q, true) + 1;
      const int r = rr > lo ? rr : lo;
      if (q - r + 1 >= min_in_a_row) {
        double score = 0.0;
        for (int j = q; j >= r; --j) {
          score = score + wdens(c, j);
          if (q - j + 1 >= min_in_a_row && score >= thr) { hit = true; break; }
        }
        if (hit) { end = wend(c, q); break; }
      }
      p2 = rr - 1;
    }
    if (!hit) end = tbit(c, lo) ? wend(c, next_set(c, lo, true) - 1) : -1;
  }
  if (start > end) end = start + (wend(c, 0) - wstart(c, 0));
  return Pos{start, end};
}

// find_left_telo (NanoTel.R:906-959)
__device__ __forceinline__ Pos find_left_telo(const CallCtx& c) {
  if (c.nw == 0) return Pos{1, 1};
  const int f = next_set(c, 0, false);
  if (f < c.nw && wstart(c, f) <= 200) return Pos{wstart(c, f), wend(c, next_set(c, f, true) - 1)};
  if (wstart(c, c.nw - 1) > 200) return Pos{-1, -1};
  return Pos{1, 1};
}

// find_right_telo (NanoTel.R:843-899).  err=true on a 0-row table.
__device__ __forceinline__ Pos find_right_telo(const CallCtx& c, bool& err) {
  if (c.nw == 0) { err = true; return Pos{1, 1}; }
  const int g = prev_set(c, c.nw - 1, false);
  if (g >= 0) {
    if (wend(c, g) < c.n - 200) return Pos{-1, -1};
    return Pos{wstart(c, prev_set(c, g, true) + 1), wend(c, g)};
  }
  if (wend(c, 0) < c.n - 200) return Pos{-1, -1};
  return Pos{1, 1};
}

// ------------------------------------------------------------------ A10

// get_accurate_start (NanoTel.R:1726-1764)
__device__ __forceinline__ int accurate_start(CallCtx& c, int s) {
  if (s == -1) return -1;
  const double first_50 = (double)range_count(c, s, s + 49) / 50.0;
  int t = s;
  if (first_50 < 0.3) {
    t = min_start_in(c, s + 48, s + 99, t);
    t = min_start_in(c, s + 33, s + 48, t);
  } else {
    t = min_start_in(c, s, s + 99, t);
    if (first_50 >= 0.72) t = min_start_in(c, s - 36, s - 1, t);
  }
  return t;
}

// get_accurate_end (NanoTel.R:1692-1721)
__device__ __forceinline__ int accurate_end(CallCtx& c, int e) {
  if (e == -1) return -1;
  const int t = max_end_in(c, e - 99, e, e);
  return max_end_in(c, e + 1, e + 50, t);
}

// ------------------------------------------------------------------ A12

// The four steps of search_right_patterns / search_left_patterns
// (NanoTel.R:576-697: width 18, step 10) evaluated in parallel: lane
// 16*step + q matches pattern q (patterns, then TVRs) against step `step`'s
// sub-sequence with fixed=TRUE, out-of-bound positions counted relative to the
// sub-sequence (multi_pattern_step_*, NanoTel.R:496-575); the steps are then
// consumed in order, stopping at the first step without a match.
__device__ __forceinline__ int search_edge(const CallCtx& c, int index, bool right) {
  const NtProgram* prog = c.prog;
  const int npt = prog->n_pat + (c.use_tvr ? prog->n_tvr : 0);
  const bool only_exact = c.use_tvr && c.k == 0;
  const int step = c.lane >> 4, q = c.lane & 15;
  int sa = 1, sb = 1;
  uint32_t more_mask = 0u;
  if (right) {
    int se = index + 18 < c.n ? index + 18 : c.n;
    for (int i = 0; i < 4; ++i) {
      if (i == step) { sa = se - 17 > 1 ? se - 17 : 1; sb = se; }
      const int ne = se + 11 < c.n ? se + 11 : c.n;
      if (ne != se) more_mask |= 1u << i;
      se = ne;
    }
  } else {
    int ss = index - 18 > 1 ? index - 18 : 1;
    for (int i = 0; i < 4; ++i) {
      if (i == step) { sa = ss; sb = ss + 17 < c.n ? ss + 17 : c.n; }
      const int ns = ss - 9 > 1 ? ss - 9 : 1;
      if (ns != ss) more_mask |= 1u << i;
      ss = ns;
    }
  }
  bool found = false;
  int val = right ? INT_MIN : INT_MAX;
  if (q < npt) {
    const bool is_tvr = q >= prog->n_pat;
    const NtPat& P = is_tvr ? prog->tvr[q - prog->n_pat] : prog->pat[q];
    const int k = (is_tvr || only_exact) ? 0 : c.k;
    const int A = sa - 1, Bz = sb - 1, base = A - 1;
    uint32_t a0, a1w;
    hits_at(c.rc, P, true, base, A, Bz, a0, a1w);
    const uint32_t h = k ? a1w : a0;
    if (h) {
      found = true;
      val = right ? base + (31 - __builtin_clz(h)) + P.m : base + __builtin_ctz(h) + 1;
    }
  }
  for (int o = 8; o > 0; o >>= 1) {  // reduce over the patterns of each step
    const int other = __shfl_xor(val, o, 16);
    val = right ? (other > val ? other : val) : (other < val ? other : val);
  }
  const uint64_t fb = __ballot(found);
  int result = index;
  for (int i = 0; i < 4; ++i) {
    if (!((fb >> (16 * i)) & 0xFFFFull)) break;
    result = uni(__shfl(val, 16 * i, kWave));
    if (!((more_mask >> i) & 1u)) break;
  }
  return result;
}

// find_telo_position_wraper (NanoTel.R:1080-1155) + density (NanoTel.R:1840).
__device__ __forceinline__ void call_pass(CallCtx& c, int& out_s, int& out_e, double& out_d,
                                          uint32_t& err) {
  Pos tp = find_telo_position(c, 3, 2.0);
  const double telo_density = sub_density(c, tp.s, tp.e);
  const int num_rows = (tp.e - tp.s + 1) / c.L;
  if (telo_density < 0.85 && num_rows > 5) {
    const int min_rows = num_rows <= 7 ? num_rows - 2 : 7;
    const double min_density = 0.6 * (double)min_rows;
    tp = find_telo_position(c, min_rows, min_density);
  }
  const int s_acc = accurate_start(c, tp.s);
  int e_acc = accurate_end(c, tp.e);
  if (s_acc > e_acc) e_acc = s_acc;
  tp = Pos{s_acc, e_acc};
  if (tp.e - tp.s + 1 < 100) {
    if (c.prog->right_edge) {
      bool e = false;
      tp = find_right_telo(c, e);
      if (e) { err |= NT_FLAG_ERR_RIGHT; out_s = -1; out_e = -1; out_d = 0.0; return; }
    } else {
      tp = find_left_telo(c);
    }
  }
  if (!c.prog->legacy_no_ext) {
    int e2 = tp.e, s2 = tp.s;
    if (tp.e < c.n) e2 = search_edge(c, tp.e + 1, true);
    if (tp.s > 1) s2 = search_edge(c, tp.s - 1, false);
    tp = Pos{s2, e2};
  }
  if (tp.e < tp.s - 1) { err |= NT_FLAG_ERR_WIDTH; out_s = -1; out_e = -1; out_d = 0.0; return; }
  out_s = tp.s;
  out_e = tp.e;
  out_d = sub_density(c, tp.s, tp.e);
}

// ============================================================== the kernel

// Per-wave scratch: [n_hits][64] hit accumulators (generic programs), the
// window counters [pass][window] (uint32) and the telomeric bitmasks
// [pass][nmw] (uint64).  kLds: in LDS; otherwise in a global scratch slice
// (reads too long for the LDS budget).
template <bool kSingle, bool kLds, int kM>
__global__ void __launch_bounds__(kWG)
nt_kernel(const NtProgram* __restrict__ prog, const uint32_t* __restrict__ thr, NtBatch B, NtOut O,
          uint32_t len_lo, uint32_t len_hi, uint32_t wave_words, uint32_t nw_cap,
          uint32_t* __restrict__ gscr) {
  extern __shared__ uint32_t smem[];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * kNWaves + wave, GW = (uint64_t)gridDim.x * kNWaves;
  const int np = prog->n_pass, nh = prog->n_hits, L = prog->L;
  uint32_t* wmem = kLds ? smem + (uint64_t)wave * wave_words : gscr + gw * wave_words;
  uint32_t* hitacc = wmem;
  uint32_t* cnt = wmem + (kSingle ? 0 : nh * kWave);
  uint64_t* tm = reinterpret_cast<uint64_t*>(cnt + ((np * nw_cap + 1) & ~1u));
  const int nmw_cap = (int)((nw_cap + 63) / 64);

  for (uint64_t r = gw; r < B.n_reads; r += GW) {
    const uint32_t n32 = B.len[r];
    if (n32 <= len_lo || n32 > len_hi) continue;
    ReadCtx rc;
    rc.n = n32;
    rc.nblk = (int32_t)((n32 + 31u) >> 5);
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
    const int n = (int)n32;
    const int nw = (int)split_window_count(n, L);
    const int ncnt = nw * np;
    for (int i = lane; i < ncnt; i += kWave) cnt[i] = 0u;
    if (!kSingle)
      for (int cix = 0; cix < nh; ++cix) hitacc[cix * kWave + lane] = 0u;
    wave_sync();

    // ---------------------------------------------------------- scan
    uint32_t acc0 = 0u, acc1 = 0u;
    scan_read<kSingle, kM>(prog, rc, lane, np, nw, cnt, hitacc, acc0, acc1);
    wave_sync();

    uint16_t* wout = O.win_counts + B.win_off[r] * np;
    for (int i = lane; i < ncnt; i += kWave) wout[i] = (uint16_t)cnt[i];
    if (O.hits) {
      if (kSingle) {
        const uint32_t h0 = wave_sum_u32(acc0), h1 = wave_sum_u32(acc1);
        if (lane == 0) {
          O.hits[r * (uint64_t)nh] = h0;
          O.hits[r * (uint64_t)nh + 1] = h1;
        }
      } else {
        for (int cix = 0; cix < nh; ++cix) {
          const uint32_t v = wave_sum_u32(hitacc[cix * kWave + lane]);
          if (lane == 0) O.hits[r * (uint64_t)nh + cix] = v;
        }
      }
    }

    // ---------------------------------------------------------- call
    const int tsz = (int)prog->thr_size;
    const uint32_t thr_full = thr[L < tsz ? L : tsz - 1];
    uint32_t thr_last = thr_full;
    if (nw > 0) {
      const int wl = n - (nw - 1) * L;
      thr_last = thr[wl < tsz ? wl : tsz - 1];
    }
    const int nmw = (nw + 63) >> 6;
    int maxw = INT_MIN;
    uint32_t flags = NT_FLAG_DONE;
    for (int p = 0; p < np; ++p) {
      const uint32_t* pc = cnt + p * nw;
      uint64_t* ptm = tm + p * nmw_cap;
      // class -5 ("telomeric") iff !(count/width < min_density) iff count >= thr[width]
      for (int ch = 0; ch < nmw; ++ch) {
        const int i = ch * 64 + lane;
        const bool t = i < nw && pc[i] >= (i == nw - 1 ? thr_last : thr_full);
        const uint64_t bal = __ballot(t);
        if (lane == 0) ptm[ch] = bal;
      }
      wave_sync();
      CallCtx c;
      c.rc = rc;
      c.prog = prog;
      c.cnt = pc;
      c.tm = ptm;
      c.n = n;
      c.nw = nw;
      c.nmw = nmw;
      c.L = L;
      c.k = p == 0 ? 0 : 1;
      c.use_tvr = p == 2;
      c.raw = p == 0 && prog->raw_p1;
      c.lane = lane;
      c.R0.P0 = kNoRegion;
      c.R1.P0 = kNoRegion;
      c.lru = 0;
      int s, e;
      double d;
      uint32_t err = 0;
#ifndef NT_NO_CALL
      call_pass(c, s, e, d, err);
#else
      s = c.nw; e = c.nmw; d = 0.0; asm volatile("" :: "v"(c.tm), "v"(c.cnt));
#endif
      flags |= err;
      if (s == -1) flags |= 1u << (NT_FLAG_NA_SHIFT + p);
      if (e - s + 1 > maxw) maxw = e - s + 1;
      if (lane == 0) {
        O.start[r * 3 + p] = s;
        O.end[r * 3 + p] = e;
        O.density[r * 3 + p] = d;
      }
    }
    if (lane == 0) {
      for (int p = np; p < 3; ++p) {
        O.start[r * 3 + p] = -1;
        O.end[r * 3 + p] = -1;
        O.density[r * 3 + p] = 0.0;
      }
      if (maxw >= 30) flags |= NT_FLAG_TELOMERIC;
      O.flags[r] = (uint8_t)flags;
    }
    wave_sync();
  }
}

// ============================================================ synthetic reads

// One thread per 32-base block: bases from the counter-based generator of
// nt_rng.h (identical on the host: nt_synth_base()).
__global__ void __launch_bounds__(256)
nt_synth_kernel(NtSynth S, uint32_t* __restrict__ planes, uint64_t n_reads) {
  const uint64_t nblk = (S.read_len + 31) / 32;
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

}  // namespace nt

// ================================================================ launchers

extern "C" {

// per-wave scratch words for a read with nw_cap windows
uint32_t nt_dev_wave_words(int single, int n_hits, int np, uint32_t nw_cap) {
  const uint32_t hit = single ? 0u : (uint32_t)n_hits * 64u;
  const uint32_t cntw = ((uint32_t)np * nw_cap + 1u) & ~1u;
  const uint32_t tmw = 2u * (uint32_t)np * ((nw_cap + 63u) / 64u);
  return hit + cntw + tmw;
}

hipError_t nt_dev_set_lds_limit(uint32_t bytes) {
  const void* fns[3] = {(const void*)nt::nt_kernel<true, true, 6>, (const void*)nt::nt_kernel<true, true, 0>,
                        (const void*)nt::nt_kernel<false, true, 0>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// single: 1 pattern, no TVR; m6: that pattern has 6 letters (compile-time length)
hipError_t nt_dev_launch(const NtProgram* prog, const uint32_t* thr, const NtBatch* B,
                         const NtOut* O, uint32_t len_lo, uint32_t len_hi, int single, int m6,
                         int lds, uint32_t wave_words, uint32_t nw_cap, uint32_t* gscr, int grid,
                         hipStream_t stream) {
  const size_t lds_bytes = lds ? (size_t)wave_words * 4u * nt::kNWaves : 0;
#define NT_LAUNCH(S, G, M)                                                                          \
  hipLaunchKernelGGL((nt::nt_kernel<S, G, M>), dim3(grid), dim3(nt::kWG), lds_bytes, stream, prog, \
                     thr, *B, *O, len_lo, len_hi, wave_words, nw_cap, gscr)
  if (single && lds && m6) NT_LAUNCH(true, true, 6);
  else if (single && lds) NT_LAUNCH(true, true, 0);
  else if (single) NT_LAUNCH(true, false, 0);
  else if (lds) NT_LAUNCH(false, true, 0);
  else NT_LAUNCH(false, false, 0);
#undef NT_LAUNCH
  return hipGetLastError();
}

hipError_t nt_dev_launch_synth(const NtSynth* S, uint32_t* planes, uint64_t n_reads,
                               hipStream_t stream) {
  const uint64_t nblk = (S->read_len + 31) / 32;
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
