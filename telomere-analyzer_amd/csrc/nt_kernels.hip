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
//  nt_call_kernel  -- one LANE per read.  The telomere calling of
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
// The calling kernel is bound by dependent memory round trips (one lane per
// read-pass walks its read), so each step loads what it needs as one batch of
// independent loads: the telomeric-bitmask words up front (reads of <= 512
// windows), the counts of a run four windows at a time, both A10
// neighbourhoods together, both edge-extension plane windows together, and
// the two partial windows of a range count together with its checkpoints.

struct Pos {
  int s, e;
};

// The pass's telomeric-window bitmask (tm[0 .. nmw)) is copied once per lane
// and walked from there: in LDS (default), 16 words (reads up to 1,024
// windows), word-major with a stride of 256 lanes; or in registers (8 words),
// where every access is an 8-way select chain and the state spills -- the
// LDS copy took the 1M x 50 kb call from 0.90 to 0.55 ms (c10k 0.70 -> 0.47).
#ifndef NT_CALL_TM_LDS
#define NT_CALL_TM_LDS 1
#endif
#ifndef NT_CALL_TM_WORDS
#define NT_CALL_TM_WORDS 16
#endif
constexpr int kTmRegs = NT_CALL_TM_LDS ? NT_CALL_TM_WORDS : 8;  // bitmask words held per lane

// Per-lane state of one read-pass.
struct Lane {
  ReadCtx rc;
  const NtProgram* prog;
  const void* cnt;       // this pass's window counts: uint8 when c8, else uint16
  bool c8;
  const uint64_t* tm;    // this pass's telomeric-window bitmask
  const uint32_t* ck;    // this pass's running counts at every 16th window boundary
  int n, nw, nmw, L;
  int k;         // 0 for P1, 1 for P2/P3
  bool use_tvr;  // P3
  bool raw;      // P1 raw views (single fixed pattern, NanoTel.R:349-355)
  uint32_t* pws;  // NT_CALL_PW_LDS: this lane's edge-extension plane words in LDS
  bool tm_reg;   // tmw holds tm[0 .. nmw)
#if NT_CALL_TM_LDS
  uint64_t* tmw;  // this lane's words in LDS, stride 256 (word-major: conflict-free at equal word)
#else
  uint64_t tmw[kTmRegs];
#endif
};

__device__ __forceinline__ int wstart(const Lane& c, int i) { return 1 + i * c.L; }
__device__ __forceinline__ int wend(const Lane& c, int i) { return i == c.nw - 1 ? c.n : wstart(c, i) + c.L - 1; }
__device__ __forceinline__ int wcount(const Lane& c, int i) {
  return c.c8 ? (int)static_cast<const uint8_t*>(c.cnt)[i] : (int)static_cast<const uint16_t*>(c.cnt)[i];
}
__device__ __forceinline__ double wdens_of(const Lane& c, int i, int cnt) {
  return (double)cnt / (double)(wend(c, i) - wstart(c, i) + 1);
}

__device__ __forceinline__ void tm_preload(Lane& c) {
  c.tm_reg = c.nmw > 0 && c.nmw <= kTmRegs;
  if (!c.tm_reg) return;
#if NT_CALL_TM_LDS
  uint64_t v[kTmRegs];
#pragma unroll
  for (int t = 0; t < kTmRegs; ++t) v[t] = t < c.nmw ? c.tm[t] : 0ull;
#pragma unroll
  for (int t = 0; t < kTmRegs; ++t) c.tmw[t * 256] = v[t];
#else
#pragma unroll
  for (int t = 0; t < kTmRegs; ++t) c.tmw[t] = t < c.nmw ? c.tm[t] : 0ull;
#endif
}

__device__ __forceinline__ uint64_t tword(const Lane& c, int wi, bool inv) {
  uint64_t x;
  if (c.tm_reg) {
#if NT_CALL_TM_LDS
    x = c.tmw[(wi < kTmRegs ? wi : 0) * 256];
#else
    x = c.tmw[0];
#pragma unroll
    for (int t = 1; t < kTmRegs; ++t)
      if (wi == t) x = c.tmw[t];
#endif
  } else {
    x = c.tm[wi];
  }
  return inv ? ~x : x;
}
__device__ __forceinline__ bool tbit(const Lane& c, int i) { return (tword(c, i >> 6, false) >> (i & 63)) & 1ull; }

__device__ __forceinline__ int next_set(const Lane& c, int pos, bool inv) {
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

__device__ __forceinline__ int prev_set(const Lane& c, int pos, bool inv) {
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

// ------------------------------------------- boundary neighbourhoods
//
// The calling touches the coverage only near a few positions (the partial
// windows of range_count, the A10 boundary refinements).  A neighbourhood
// computes the pass's coverage words over [q0, q0 + 32K) at once from one
// batch of K+5 block loads (nb_fetch), then the bit-sliced match of every
// pattern at every start with the letter tables hoisted out of the word loop
// (nb_compute).
// cov[i + 1] = coverage of [q0 + 32i, q0 + 32i + 31] for i = -1..K (kMarks: the
// two neighbour words run marks need; else i = 0..K-1 are meaningful);
// rs/re: P1's raw view starts / ends (c.raw) at the same positions.
template <int K, bool kMarks = true>
struct Nb {
  int q0;
  uint32_t cov[K + 2];
  uint32_t rs[kMarks ? K + 2 : 1];
  uint32_t re[kMarks ? K + 2 : 1];
};

template <int K, bool kMarks = true>
struct NbBlocks {
  uint2 b[K + (kMarks ? 2 : 0) + 3];
};

template <int K, bool kMarks>
__device__ __forceinline__ void nb_fetch(const Lane& c, int q0, NbBlocks<K, kMarks>& f) {
  constexpr int E = kMarks ? 1 : 0;
  constexpr int NP = K + 2 * E + 2;
  const int bb = (q0 >> 5) - E - 1;  // arithmetic shift: floor for q0 < 0
#pragma unroll
  for (int t = 0; t <= NP; ++t) {
    const int b = bb + t;
    f.b[t] = (b >= 0 && b < c.rc.nblk) ? c.rc.blk[b] : make_uint2(0u, 0u);
  }
}

template <int K, bool kMarks>
__device__ __forceinline__ void nb_compute(const Lane& c, int q0, const NbBlocks<K, kMarks>& f,
                                           Nb<K, kMarks>& nb) {
  constexpr int E = kMarks ? 1 : 0;  // extra word each side
  constexpr int NC = K + 2 * E;      // coverage words computed, i = -E..K-1+E
  constexpr int NP = NC + 2;         // plane words, positions [q0 + 32i, +31], i = -E-1..K+E
  constexpr int NH = NC + 1;         // hit words, starts [q0 + 32i, +31], i = -E-1..K-1+E
  constexpr int T0 = -E - 1;         // index of plane / hit word 0
  nb.q0 = q0;
  uint32_t Lw[NP], Hw[NP], Vw[NP];
  const uint32_t sh = (uint32_t)(q0 & 31);
#pragma unroll
  for (int t = 0; t < NP; ++t) {
    Lw[t] = funnel(f.b[t + 1].x, f.b[t].x, sh);
    Hw[t] = funnel(f.b[t + 1].y, f.b[t].y, sh);
    Vw[t] = range_mask((int64_t)q0 + 32 * (t + T0), 0, c.n - 1);
  }
#pragma unroll
  for (int i = 0; i < K + 2; ++i) nb.cov[i] = 0u;
  const NtProgram* prog = c.prog;
  const int npt = prog->n_pat + (c.use_tvr ? prog->n_tvr : 0);
  for (int pi = 0; pi < npt; ++pi) {
    const bool is_tvr = pi >= prog->n_pat;
    const NtPat& P = is_tvr ? prog->tvr[pi - prog->n_pat] : prog->pat[pi];
    const int m = P.m;
    uint32_t x0[NH], x1[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) x0[h] = x1[h] = 0xFFFFFFFFu;
    for (int j = 0; j < m; ++j) {
      const uint32_t t0 = P.tm_scan[j][0], t1 = P.tm_scan[j][1], t2 = P.tm_scan[j][2], t3 = P.tm_scan[j][3];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const uint32_t Ls = funnel(Lw[h + 1], Lw[h], (uint32_t)j);
        const uint32_t Hs = funnel(Hw[h + 1], Hw[h], (uint32_t)j);
        const uint32_t q = bfi(Hs, bfi(Ls, t3, t2), bfi(Ls, t1, t0)) & funnel(Vw[h + 1], Vw[h], (uint32_t)j);
        x1[h] = (x1[h] & q) | x0[h];
        x0[h] &= q;
      }
    }
    if (m <= 1) {
#pragma unroll
      for (int h = 0; h < NH; ++h) x1[h] &= Vw[h];
    }
    if (c.rc.n_exc) {
#pragma unroll
      for (int h = 0; h < NH; ++h)
        patch_exceptions(c.rc, (int64_t)q0 + 32 * (h + T0), 0, c.n - 1, P, false, x0[h], x1[h]);
    }
    const bool use_a1 = !is_tvr && c.k;
    // coverage word ci (i = ci - E) from hit words i and i - 1
#pragma unroll
    for (int ci = 0; ci < NC; ++ci)
      nb.cov[ci + 1 - E] |= spread(use_a1 ? x1[ci + 1] : x0[ci + 1], use_a1 ? x1[ci] : x0[ci], m);
    if constexpr (kMarks) {
      if (c.raw && pi == 0) {
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
          nb.rs[ci] = x0[ci + 1];
          nb.re[ci] = m > 1 ? funnel(x0[ci + 1], x0[ci], (uint32_t)(32 - (m - 1))) : x0[ci + 1];
        }
      }
    }
  }
#pragma unroll
  for (int ci = 0; ci < NC; ++ci) nb.cov[ci + 1 - E] &= Vw[ci + 1];
}

// |coverage ∩ [a, b]|, [a, b] within [q0, q0 + 32K)
template <int K, bool kMarks>
__device__ __forceinline__ int nb_count(const Nb<K, kMarks>& nb, int a, int b) {
  int t = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) t += __builtin_popcount(nb.cov[i + 1] & range_mask((int64_t)nb.q0 + 32 * i, a, b));
  return t;
}

// min(start(ranges)) with start in [a1, b1] (1-based), fallback if none;
// run starts of the reduced coverage, or P1's raw view starts
template <int K>
__device__ __forceinline__ int nb_min_start(const Lane& c, const Nb<K>& nb, int a1, int b1, int fallback) {
  const int a = max(a1 - 1, 0), b = min(b1 - 1, c.n - 1);
  int res = fallback;
  bool found = false;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const uint32_t cur = nb.cov[i + 1];
    const uint32_t mk = c.raw ? nb.rs[i + 1] : (cur & ~((cur << 1) | (nb.cov[i] >> 31)));
    const uint32_t m = mk & range_mask((int64_t)nb.q0 + 32 * i, a, b);
    if (!found && m) {
      res = nb.q0 + 32 * i + __builtin_ctz(m) + 1;
      found = true;
    }
  }
  return res;
}

// max(end(ranges)) with end in [a1, b1] (1-based), fallback if none
template <int K>
__device__ __forceinline__ int nb_max_end(const Lane& c, const Nb<K>& nb, int a1, int b1, int fallback) {
  const int a = max(a1 - 1, 0), b = min(b1 - 1, c.n - 1);
  int res = fallback;
  bool found = false;
#pragma unroll
  for (int i = K - 1; i >= 0; --i) {
    const uint32_t cur = nb.cov[i + 1];
    const uint32_t mk = c.raw ? nb.re[i + 1] : (cur & ~((cur >> 1) | (nb.cov[i + 2] << 31)));
    const uint32_t m = mk & range_mask((int64_t)nb.q0 + 32 * i, a, b);
    if (!found && m) {
      res = nb.q0 + 32 * i + (31 - __builtin_clz(m)) + 1;
      found = true;
    }
  }
  return res;
}

// |coverage ∩ [x, y]| (0-based positions), 128 bases per neighbourhood
__device__ __forceinline__ int cov_count(const Lane& c, int x, int y) {
  int tot = 0;
  for (int q = x; q <= y; q += 128) {
    NbBlocks<4, false> f;
    Nb<4, false> nb;
    nb_fetch(c, q, f);
    nb_compute(c, q, f, nb);
    tot += nb_count(nb, q, min(y, q + 127));
  }
  return tot;
}

// |coverage ∩ [x1, y1]| + |coverage ∩ [x2, y2]| (x > y: empty); both fetched
// in one batch when each range spans at most 128 bases
__device__ __forceinline__ int cov_count2(const Lane& c, int x1, int y1, int x2, int y2) {
  if (y1 - x1 >= 128 || y2 - x2 >= 128) return cov_count(c, x1, y1) + cov_count(c, x2, y2);
  NbBlocks<4, false> f1, f2;
  nb_fetch(c, x1, f1);
  nb_fetch(c, x2, f2);
  int t = 0;
  if (x1 <= y1) {
    Nb<4, false> nb;
    nb_compute(c, x1, f1, nb);
    t += nb_count(nb, x1, y1);
  }
  if (x2 <= y2) {
    Nb<4, false> nb;
    nb_compute(c, x2, f2, nb);
    t += nb_count(nb, x2, y2);
  }
  return t;
}

// sum(width(intersect(IRanges(a1, b1), ranges))): window counts for whole
// windows, recomputed coverage for the partial windows at the two ends.
// Covered bases of windows [0, k) (0 <= k <= nw): the scan's checkpoint at
// window 16*(k/16) plus at most 15 window counts (independent loads).
__device__ __forceinline__ int cnt_before(const Lane& c, int k) {
  const int r = k & 15, k0 = k - r;
  int t = (int)c.ck[k >> 4];
#pragma unroll
  for (int i = 0; i < 15; ++i)
    if (i < r) t += wcount(c, k0 + i);
  return t;
}

__device__ __forceinline__ int range_count(const Lane& c, int a1, int b1) {
  const int a = (a1 < 1 ? 1 : a1) - 1, b = (b1 > c.n ? c.n : b1) - 1;
  if (a > b) return 0;
  if (c.nw == 0) return cov_count(c, a, b);
  const int L = c.L;
  const int ka = min(div_l(c.prog, a), c.nw - 1), kb = min(div_l(c.prog, b), c.nw - 1);
  const int ws_a = ka * L, we_b = kb == c.nw - 1 ? c.n - 1 : (kb + 1) * L - 1;
  const bool a_whole = a == ws_a, b_whole = b == we_b;
  if (ka == kb) return (a_whole && b_whole) ? wcount(c, ka) : cov_count(c, a, b);
  // whole windows from the running counts, partial end windows from coverage
  const int whole = cnt_before(c, b_whole ? kb + 1 : kb) - cnt_before(c, a_whole ? ka : ka + 1);
  return whole + cov_count2(c, a_whole ? 0 : a, a_whole ? -1 : (ka + 1) * L - 1, b_whole ? 0 : kb * L,
                            b_whole ? -1 : b);
}

__device__ __forceinline__ double sub_density(const Lane& c, int s, int e) {
  return (double)range_count(c, s, e) / (double)(e - s + 1);
}

// ---------------------------------------------------------------- A8 / A11

// find_telo_position (NanoTel.R:973-1077) on the window bitmask; the scores
// are summed in R's order, the counts of a run fetched four at a time.
__device__ __forceinline__ Pos find_telo_position(const Lane& c, int min_in_a_row, double thr) {
  int pos = 0, found = -1, start = -1;
  for (;;) {
    const int r = next_set(c, pos, false);
    if (r >= c.nw) break;
    const int q = next_set(c, r, true) - 1;  // last window of the telomeric run
    if (q - r + 1 >= min_in_a_row) {
      double score = 0.0;
      for (int j0 = r; j0 <= q && found < 0; j0 += 4) {
        int cn[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) cn[t] = wcount(c, min(j0 + t, q));
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int j = j0 + t;
          if (j <= q && found < 0) {
            score = score + wdens_of(c, j, cn[t]);
            if (j - r + 1 >= min_in_a_row && score >= thr) found = j;
          }
        }
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
        for (int j0 = q; j0 >= r && !hit; j0 -= 4) {
          int cn[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) cn[t] = wcount(c, max(j0 - t, r));
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int j = j0 - t;
            if (j >= r && !hit) {
              score = score + wdens_of(c, j, cn[t]);
              if (q - j + 1 >= min_in_a_row && score >= thr) hit = true;
            }
          }
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
__device__ __forceinline__ Pos find_left_telo(const Lane& c) {
  if (c.nw == 0) return Pos{1, 1};
  const int f = next_set(c, 0, false);
  if (f < c.nw && wstart(c, f) <= 200) return Pos{wstart(c, f), wend(c, next_set(c, f, true) - 1)};
  if (wstart(c, c.nw - 1) > 200) return Pos{-1, -1};
  return Pos{1, 1};
}

// find_right_telo (NanoTel.R:843-899).  err=true on a 0-row table.
__device__ __forceinline__ Pos find_right_telo(const Lane& c, bool& err) {
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

// get_accurate_start (NanoTel.R:1726-1764) reads only ranges in [s-37, s+98]
// and get_accurate_end (NanoTel.R:1692-1721) only ranges in [e-100, e+49]
// (0-based; the offsets are hard-coded in the reference), so each is one
// neighbourhood, [s-42, s+118) and [e-102, e+58); both fetched in one batch.
__device__ __forceinline__ void accurate_fetch(const Lane& c, int s, int e, NbBlocks<5>& fs, NbBlocks<5>& fe) {
  nb_fetch(c, s - 42, fs);
  nb_fetch(c, e - 102, fe);
}

__device__ __forceinline__ void accurate_both(const Lane& c, int s, int e, const NbBlocks<5>& fs,
                                              const NbBlocks<5>& fe, int& s_acc, int& e_acc) {
  s_acc = -1;
  e_acc = -1;
  if (s != -1) {
    Nb<5> nb;
    nb_compute(c, s - 42, fs, nb);
    const int a = max(s, 1) - 1, b = min(s + 49, c.n) - 1;
    const double first_50 = (double)(a > b ? 0 : nb_count(nb, a, b)) / 50.0;
    int t = s;
    if (first_50 < 0.3) {
      t = nb_min_start(c, nb, s + 48, s + 99, t);
      t = nb_min_start(c, nb, s + 33, s + 48, t);
    } else {
      t = nb_min_start(c, nb, s, s + 99, t);
      if (first_50 >= 0.72) t = nb_min_start(c, nb, s - 36, s - 1, t);
    }
    s_acc = t;
  }
  if (e != -1) {
    Nb<5> nb;
    nb_compute(c, e - 102, fe, nb);
    const int t = nb_max_end(c, nb, e - 99, e, e);
    e_acc = nb_max_end(c, nb, e + 1, e + 50, t);
  }
}

// ------------------------------------------------------------------ A12

// Plane words of [q0, q0 + 32K) (q0 a multiple of 32; zero outside the read).
// The four steps of one side of the edge extension match at bases within 33
// (right) / 27 (left) of the lowest one, each over 64 positions, so one batch
// of K = 5 block loads per side from the lowest base serves all of them.
#ifndef NT_CALL_PW_LDS
#define NT_CALL_PW_LDS 0  // measured +-0 (edge-extension words in LDS)
#endif
#ifndef NT_CALL_ACC_EARLY
#define NT_CALL_ACC_EARLY 0  // measured 1 % slower (0.559 vs 0.553 ms at c50k)
#endif
template <int K>
struct Pw {
  int q0;
#if NT_CALL_PW_LDS
  uint32_t* s;  // this lane's 2K words in LDS (L then H), stride 256
#else
  uint32_t L[K], H[K];
#endif
};

template <int K>
__device__ __forceinline__ void pw_load(const Lane& c, int q0, Pw<K>& w) {
  w.q0 = q0;
  const int b0 = q0 >> 5;
#if NT_CALL_PW_LDS
  uint2 x[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int b = b0 + i;
    x[i] = (b >= 0 && b < c.rc.nblk) ? c.rc.blk[b] : make_uint2(0u, 0u);
  }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    w.s[i * 256] = x[i].x;
    w.s[(K + i) * 256] = x[i].y;
  }
#else
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int b = b0 + i;
    const uint2 x = (b >= 0 && b < c.rc.nblk) ? c.rc.blk[b] : make_uint2(0u, 0u);
    w.L[i] = x.x;
    w.H[i] = x.y;
  }
#endif
}

// planes of [p, p + 31] (as plane_at), from the window when it holds them
template <int K>
__device__ __forceinline__ void pw_at(const Lane& c, const Pw<K>& w, int p, uint32_t& L, uint32_t& H) {
  const int d = p - w.q0;
  const int i = d >> 5;
  if (d < 0 || i + 1 >= K) {
    plane_at(c.rc, p, L, H);
    return;
  }
#if NT_CALL_PW_LDS
  const uint32_t l0 = w.s[i * 256], l1 = w.s[(i + 1) * 256];
  const uint32_t h0 = w.s[(K + i) * 256], h1 = w.s[(K + i + 1) * 256];
#else
  uint32_t l0 = w.L[0], h0 = w.H[0], l1 = w.L[1], h1 = w.H[1];
#pragma unroll
  for (int t = 1; t + 1 < K; ++t)
    if (i == t) {
      l0 = w.L[t];
      h0 = w.H[t];
      l1 = w.L[t + 1];
      h1 = w.H[t + 1];
    }
#endif
  const uint32_t sh = (uint32_t)(d & 31);
  L = funnel(l1, l0, sh);
  H = funnel(h1, h0, sh);
}

// hits_at (nt_device.h) with the planes taken from the window
template <int K>
__device__ __forceinline__ void hits_at_w(const Lane& c, const Pw<K>& w, const NtPat& P, bool eq, int base,
                                          int vlo, int vhi, uint32_t& a0, uint32_t& a1) {
  uint32_t L0, H0, L1, H1;
  pw_at(c, w, base, L0, H0);
  pw_at(c, w, base + 32, L1, H1);
  const uint32_t V0 = range_mask(base, vlo, vhi), V1 = range_mask((int64_t)base + 32, vlo, vhi);
  hits32<true>(L0, L1, H0, H1, V0, V1, eq ? P.tm_eq : P.tm_scan, P.m, a0, a1);
  if (P.m <= 1) a1 &= V0;
  if (c.rc.n_exc) patch_exceptions(c.rc, base, vlo, vhi, P, eq, a0, a1);
}

// max end (right) / min start (left) of the fixed=TRUE matches of the pass's
// pattern set in the sub-sequence [a1, b1], out-of-bound relative to the
// sub-sequence (multi_pattern_step_right/left, NanoTel.R:496-575).
template <int K>
__device__ __forceinline__ bool step_extreme(const Lane& c, const Pw<K>& w, int a1, int b1, bool right, int& val) {
  const NtProgram* prog = c.prog;
  const int A = a1 - 1, Bz = b1 - 1, base = A - 1;
  const bool only_exact = c.use_tvr && c.k == 0;
  const int npt = prog->n_pat + (c.use_tvr ? prog->n_tvr : 0);
  bool any = false;
  int best = right ? INT_MIN : INT_MAX;
  for (int i = 0; i < npt; ++i) {
    const bool is_tvr = i >= prog->n_pat;
    const NtPat& P = is_tvr ? prog->tvr[i - prog->n_pat] : prog->pat[i];
    const int k = (is_tvr || only_exact) ? 0 : c.k;
    uint32_t a0, a1w;
    hits_at_w(c, w, P, true, base, A, Bz, a0, a1w);
    const uint32_t h = k ? a1w : a0;
    if (!h) continue;
    any = true;
    if (right) best = max(best, base + (31 - __builtin_clz(h)) + P.m);
    else best = min(best, base + __builtin_ctz(h) + 1);
  }
  if (any) val = best;
  return any;
}

// search_right_patterns (NanoTel.R:635-697): width 18, step 10, 4 steps.
// Match bases from max(min(end_index + 18, n) - 17, 1) - 2, up to +33.
template <int K>
__device__ __forceinline__ int search_right(const Lane& c, const Pw<K>& w, int end_index) {
  int subseq_end = min(end_index + 18, c.n);
  int new_end = end_index;
  for (int it = 0; it < 4; ++it) {
    const int curr_start = max(subseq_end - 17, 1);
    int v;
    if (!step_extreme(c, w, curr_start, subseq_end, true, v)) break;
    new_end = v;
    const int ne = min(subseq_end + 11, c.n);
    if (ne == subseq_end) break;
    subseq_end = ne;
  }
  return new_end;
}

// search_left_patterns (NanoTel.R:576-633).  Match bases from
// max(start_index - 18, 1) - 2 down to max(start_index - 45, 1) - 2.
template <int K>
__device__ __forceinline__ int search_left(const Lane& c, const Pw<K>& w, int start_index) {
  int subseq_start = max(start_index - 18, 1);
  int new_start = start_index;
  for (int it = 0; it < 4; ++it) {
    const int curr_end = min(subseq_start + 17, c.n);
    int v;
    if (!step_extreme(c, w, subseq_start, curr_end, false, v)) break;
    new_start = v;
    const int ns = max(subseq_start - 9, 1);
    if (ns == subseq_start) break;
    subseq_start = ns;
  }
  return new_start;
}

// The last window of a read scanned by the bundle scan (nt_tscan.h): that scan
// does not mask the read ends, so the window holding them -- whose width may
// differ from L, and into which split_telo may have merged a short last block
// (NanoTel.R:199-227) -- is recounted here from the read's own planes (exact
// out-of-bound rule at the end), and its window count, the checkpoint at
// window nw (the read's total, when nw is a multiple of 16) and its bit of the
// telomeric bitmask (threshold of its own width) are rewritten.  Idempotent
// for reads of the per-read scan.
__device__ __forceinline__ void call_fix_last(Lane& c, const uint32_t* __restrict__ thr, uint32_t thr_size) {
  if (c.nw <= 0) return;
  const int last = c.nw - 1, a = last * c.L;
  const int exact = cov_count(c, a, c.n - 1);
  const int old = wcount(c, last);
  if (exact != old) {
    if (c.c8) static_cast<uint8_t*>(const_cast<void*>(c.cnt))[last] = (uint8_t)exact;
    else static_cast<uint16_t*>(const_cast<void*>(c.cnt))[last] = (uint16_t)exact;
    if ((c.nw & 15) == 0) const_cast<uint32_t*>(c.ck)[c.nw >> 4] += (uint32_t)(exact - old);
  }
  const uint32_t w = (uint32_t)(c.n - a);
  const bool tel = (uint32_t)exact >= thr[w < thr_size ? w : thr_size - 1];
  uint64_t* tw = const_cast<uint64_t*>(c.tm) + (last >> 6);
  const uint64_t m = 1ull << (last & 63), x = *tw;
  const uint64_t y = tel ? (x | m) : (x & ~m);
  if (y != x) *tw = y;
}

// find_telo_position_wraper (NanoTel.R:1080-1155) + density (NanoTel.R:1840).
__device__ __forceinline__ void call_pass(Lane& c, int& out_s, int& out_e, double& out_d, uint32_t& err) {
  tm_preload(c);
  Pos tp = find_telo_position(c, 3, 2.0);
#ifndef NT_DBG_NO_ACC
  // get_accurate_* neighbourhoods fetched with the wrapper's density loads
  // (one memory round trip less); refetched if the wrapper re-runs the call
  NbBlocks<5> fs, fe;
  if (NT_CALL_ACC_EARLY) accurate_fetch(c, tp.s, tp.e, fs, fe);
#endif
#ifdef NT_DBG_NO_WRAP
  const double telo_density = 1.0;
#else
  const double telo_density = sub_density(c, tp.s, tp.e);
#endif
  const int num_rows = (tp.e - tp.s + 1) / c.L;
  bool refetch = !NT_CALL_ACC_EARLY;
  if (telo_density < 0.85 && num_rows > 5) {
    const int min_rows = num_rows <= 7 ? num_rows - 2 : 7;
    const double min_density = 0.6 * (double)min_rows;
    tp = find_telo_position(c, min_rows, min_density);
    refetch = true;
  }
#ifdef NT_DBG_NO_ACC  // timing experiments only (wrong results)
  const int s_acc = tp.s;
  int e_acc = tp.e;
#else
  if (refetch) accurate_fetch(c, tp.s, tp.e, fs, fe);
  int s_acc, e_acc;
  accurate_both(c, tp.s, tp.e, fs, fe, s_acc, e_acc);
#endif
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
#ifdef NT_DBG_NO_EXT
  if (false) {
#else
  if (!c.prog->legacy_no_ext) {
#endif
    // both sides' plane windows in one batch, then the step walks in registers
    const int ei = tp.e + 1, si = tp.s - 1;
    Pw<5> wr, wl;
#if NT_CALL_PW_LDS
    wr.s = c.pws;
    wl.s = c.pws + 10 * 256;
#endif
    pw_load(c, (max(min(ei + 18, c.n) - 17, 1) - 2) & ~31, wr);
    pw_load(c, (max(si - 45, 1) - 2) & ~31, wl);
    int e2 = tp.e, s2 = tp.s;
    if (tp.e < c.n) e2 = search_right(c, wr, ei);
    if (tp.s > 1) s2 = search_left(c, wl, si);
    tp = Pos{s2, e2};
  }
  if (tp.e < tp.s - 1) { err |= NT_FLAG_ERR_WIDTH; out_s = -1; out_e = -1; out_d = 0.0; return; }
  out_s = tp.s;
  out_e = tp.e;
#ifdef NT_DBG_NO_FINAL
  out_d = 0.5;
#else
  out_d = sub_density(c, tp.s, tp.e);
#endif
}

// One lane per (read, pass): the passes of a read are independent until the
// row is assembled, so a read's G = 2 (P1, P2) or 4 (P1-P3 and an idle lane)
// lanes call them side by side -- half the dependent memory round trips per
// lane of a one-lane-per-read walk -- and combine flags / the max width over
// the passes with lane shuffles (G divides 64 and the grid stride is a
// multiple of 64, so a read's lanes share a wave).  NT_CALL_WAVES_PER_EU
// trades VGPRs for occupancy: the kernel waits on memory, so 3 waves/SIMD
// (168 VGPRs, a few spills) beat 2 (196, none) and 4 (128, 109 spilled):
// 1M x 50 kb call 1.03 / 0.90 / 0.98 ms at 2 / 3 / 4.
#ifndef NT_CALL_WAVES_PER_EU
#define NT_CALL_WAVES_PER_EU 3
#endif
#define NT_CALL_ATTR __attribute__((amdgpu_waves_per_eu(NT_CALL_WAVES_PER_EU)))
__global__ void __launch_bounds__(256) NT_CALL_ATTR
nt_call_kernel(const NtProgram* __restrict__ prog, NtBatch B, NtOut O,
               const uint64_t* __restrict__ tmask, const uint32_t* __restrict__ thr, uint32_t thr_size,
               int fix_last) {
  const int np = prog->n_pass, L = prog->L;
#if NT_CALL_TM_LDS
  __shared__ uint64_t tm_lds[kTmRegs * 256];
#endif
#if NT_CALL_PW_LDS
  __shared__ uint32_t pw_lds[20 * 256];
#endif
  const int lg = np <= 2 ? 1 : 2;  // log2(G)
  // the reads: B.list[0 .. n_list) when given (~0u entries: none), else all
  const uint64_t total = (B.list ? B.n_list : B.n_reads) << lg;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t base = blockIdx.x * (uint64_t)blockDim.x; base < total; base += stride) {
    const uint64_t idx = base + threadIdx.x;
    const uint64_t r = idx < total ? (B.list ? (uint64_t)B.list[idx >> lg] : idx >> lg) : 0;
    const bool in = idx < total && r != 0xFFFFFFFFull;  // whole waves stay in the loop for the shuffles
    const int p = (int)(idx & ((1u << lg) - 1u));
    int s = -1, e = -1;
    double d = 0.0;
    uint32_t flags = 0u;
    int w = INT_MIN;
    bool align = false;
    if (in) {
      const uint32_t n32 = B.len[r];
      align = (B.blk_off[r] & 1u) != 0;  // the scan skipped this read (layout contract)
      if (!align && p < np) {
        Lane c;
#if NT_CALL_TM_LDS
        c.tmw = tm_lds + threadIdx.x;
#endif
#if NT_CALL_PW_LDS
        c.pws = pw_lds + threadIdx.x;
#endif
        c.rc.n = n32;
        c.rc.nblk = (int32_t)((n32 + 31u) >> 5);
        c.rc.blk = reinterpret_cast<const uint2*>(B.planes) + B.blk_off[r];
        c.rc.n_exc = 0;
        c.rc.exc_pos = nullptr;
        c.rc.exc_code = nullptr;
        if (B.exc_off) {
          const uint32_t e0 = B.exc_off[r], e1 = B.exc_off[r + 1];
          c.rc.n_exc = (int32_t)(e1 - e0);
          c.rc.exc_pos = B.exc_pos + e0;
          c.rc.exc_code = B.exc_code + e0;
        }
        c.prog = prog;
        c.n = (int)n32;
        c.L = L;
        c.nw = (int)split_window_count(c.n, L);
        c.nmw = (c.nw + 63) >> 6;
        const uint64_t woff = B.win_off[r];
        const uint64_t* tmr = tmask + aux_base(woff, r, np);
        const uint32_t* ckr = reinterpret_cast<const uint32_t*>(tmr + np * aux_nmw(c.nw));
        c.c8 = prog->cnt8 != 0;
        c.cnt = static_cast<const uint8_t*>(O.win_counts) +
                (woff * np + (uint64_t)p * NT_WIN_ROWS((uint64_t)c.nw)) * (c.c8 ? 1u : 2u);
        c.tm = tmr + p * c.nmw;
        c.ck = ckr + p * aux_nck(c.nw);
        c.k = p == 0 ? 0 : 1;
        c.use_tvr = p == 2;
        c.raw = p == 0 && prog->raw_p1;
        if (fix_last) call_fix_last(c, thr, thr_size);
        call_pass(c, s, e, d, flags);
        if (s == -1) flags |= 1u << (NT_FLAG_NA_SHIFT + p);
        w = e - s + 1;
      }
    }
    // combine over the read's lanes
    for (int o = 1; o < (1 << lg); o <<= 1) {
      flags |= (uint32_t)__shfl_xor((int)flags, o, kWave);
      w = max(w, __shfl_xor(w, o, kWave));
    }
    if (!in) continue;
    if (align) {
      if (p < 3) {
        O.start[r * 3 + p] = -1;
        O.end[r * 3 + p] = -1;
        O.density[r * 3 + p] = 0.0;
      }
      if (p == 0) {
        if (lg == 1) {
          O.start[r * 3 + 2] = -1;
          O.end[r * 3 + 2] = -1;
          O.density[r * 3 + 2] = 0.0;
        }
        O.flags[r] = (uint8_t)(NT_FLAG_DONE | NT_FLAG_ERR_ALIGN);
      }
      continue;
    }
    if (p < 3) {  // passes >= np: -1 / -1 / 0
      O.start[r * 3 + p] = s;
      O.end[r * 3 + p] = e;
      O.density[r * 3 + p] = d;
    }
    if (p == 0) {
      if (lg == 1) {
        O.start[r * 3 + 2] = -1;
        O.end[r * 3 + 2] = -1;
        O.density[r * 3 + 2] = 0.0;
      }
      if (w >= 30) flags |= NT_FLAG_TELOMERIC;
      O.flags[r] = (uint8_t)(flags | NT_FLAG_DONE);
    }
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

// ================================================================ bundles
//
// The T-layout of the bundle scan (nt_common.h) from the per-read planes: one
// workgroup per bundle, its half stripes in turn (32 blocks = 32 L positions =
// L plane words of each of the bundle's 32 reads).  The half stripe's words
// of the 32 reads come into LDS by coalesced loads; then per step every lane
// takes one {lo, hi} word of its read (lanes 0-31: word w of slot s, lanes
// 32-63: word w + 1; the 4 waves every 4th step), masked past the read end,
// and two 32 x 32 bit transposes inside each half wave turn
// them into the 32-slot columns of 32 positions; these go to an LDS copy of
// the half stripe's T-layout rows (row t: 32 words of 16 bytes, 8-byte halves
// by position parity), written out as whole 512-byte row runs.  Every word of
// every stripe is written (zeros past the reads): no memset first.
constexpr int kBndRowWords = 132;  // LDS row stride (words): 128 + 4 spreads the banks

__global__ void __launch_bounds__(256)
nt_bundle_kernel(NtBatch B, uint32_t* __restrict__ tp, int L, uint32_t div_m, uint32_t div_s) {
  extern __shared__ uint32_t lds[];
  const int T = (L + 1) / 2;
  const int R = 2 * L + 2;                // words per read in the input copy (bank spread)
  uint32_t* in = lds;                     // [32][R]: the half stripe's plane words of each read
  uint32_t* rows = lds + NT_BUNDLE * R;   // [T][kBndRowWords]: its T-layout rows
  uint32_t* meta = rows + T * kBndRowWords;  // [32][4]: len, block offset lo / hi of each slot
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x >> 6;
  const int s = lane & 31, hh = lane >> 5;
  const BitTr bt(lane);
  for (uint64_t b = blockIdx.x; b < B.n_bundles; b += gridDim.x) {
    const uint32_t r = B.bnd_read[b * NT_BUNDLE + s];
    const int64_t len = r != 0xFFFFFFFFu ? (int64_t)B.len[r] : 0;
    const uint64_t g0 = uniform_u64(B.bnd_stripe[b]), g1 = uniform_u64(B.bnd_stripe[b + 1]);
    if (threadIdx.x < NT_BUNDLE) {
      const uint64_t bo = r != 0xFFFFFFFFu ? B.blk_off[r] : 0ull;
      *reinterpret_cast<uint4*>(meta + 4 * s) = make_uint4((uint32_t)len, (uint32_t)bo, (uint32_t)(bo >> 32), 0u);
    }
    __syncthreads();
    // 1. a half stripe's words [w0, w0 + L) of the 32 reads, coalesced (8
    // bytes a thread), into registers -- the next half stripe's while this
    // one is transposed -- then into LDS
    constexpr int kMaxE = (NT_BUNDLE * 170 + 255) / 256;  // L <= 170 (nt_tscan_eligible)
    uint2 v[kMaxE];
    auto fetch = [&](uint64_t uu) {
      const uint64_t wu = (uint64_t)L * uu;
#pragma unroll
      for (int k = 0; k < kMaxE; ++k) {
        const uint32_t e = threadIdx.x + 256u * k;
        v[k] = make_uint2(0u, 0u);
        if (e < (uint32_t)(NT_BUNDLE * L)) {
          const uint32_t rs = __umulhi(e, div_m) >> div_s, wd = e - rs * (uint32_t)L;
          const uint4 m = *reinterpret_cast<const uint4*>(meta + 4 * rs);
          if (32 * (int64_t)(wu + wd) < (int64_t)m.x)  // (empty slots have len 0)
            v[k] = reinterpret_cast<const uint2*>(B.planes)[(((uint64_t)m.z << 32) | m.y) + wu + wd];
        }
      }
    };
    const uint64_t nu = 2 * (g1 - g0);  // half stripes of the bundle
    fetch(0);
    for (uint64_t u = 0; u < nu; ++u) {
      const uint64_t G = g0 + (u >> 1);
      const int h = (int)(u & 1);
      const uint64_t w0 = (uint64_t)L * u;  // first plane word of the half stripe
#pragma unroll
      for (int k = 0; k < kMaxE; ++k) {
        const uint32_t e = threadIdx.x + 256u * k;
        if (e < (uint32_t)(NT_BUNDLE * L)) {
          const uint32_t rs = __umulhi(e, div_m) >> div_s, wd = e - rs * (uint32_t)L;
          *reinterpret_cast<uint2*>(in + rs * R + 2 * wd) = v[k];
        }
      }
      if ((L & 1) && threadIdx.x < 32)  // odd L: the last row's second half holds no position
        *reinterpret_cast<uint2*>(rows + (T - 1) * kBndRowWords + 4 * s + 2) = make_uint2(0u, 0u);
      __syncthreads();
      if (u + 1 < nu) fetch(u + 1);  // in flight during the transposes and the stores
      // 2. wave wv takes the steps wv, wv + 4, ... (step = 2 words: lanes 0-31
      // the first, 32-63 the second): lane 32 hh + i gets the 32-read columns
      // of position 32 wl + i
      for (int w = 2 * wv; w < L; w += 8) {
        const int wl = w + hh;
        uint2 v = make_uint2(0u, 0u);
        if (wl < L) {
          v = *reinterpret_cast<const uint2*>(in + s * R + 2 * wl);
          const int64_t nb = len - 32 * (int64_t)(w0 + wl);  // valid bases of the word
          const uint32_t m = nb >= 32 ? ~0u : nb <= 0 ? 0u : ((1u << nb) - 1u);
          v.x &= m;
          v.y &= m;
        }
        const uint32_t cl = half_bit_transpose(v.x, lane, bt), ch = half_bit_transpose(v.y, lane, bt);
        if (wl < L) {
          const uint32_t p = 32u * (uint32_t)wl + (uint32_t)s;  // position in the half stripe
          const uint32_t l = __umulhi(p, div_m) >> div_s, o = p - l * (uint32_t)L;
          *reinterpret_cast<uint2*>(rows + (o >> 1) * kBndRowWords + 4 * l + 2 * (o & 1)) = make_uint2(cl, ch);
        }
      }
      __syncthreads();
      // 3. rows t: 32 words of 16 bytes at word (G T + t) 64 + 32 h + l
      uint4* out = reinterpret_cast<uint4*>(tp) + G * (uint64_t)T * kWave + 32 * h;
      for (int t = threadIdx.x >> 5; t < T; t += 8)
        out[(uint64_t)t * kWave + s] = *reinterpret_cast<const uint4*>(rows + t * kBndRowWords + 4 * s);
      __syncthreads();
    }
    __syncthreads();  // meta is rewritten for the next bundle
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

hipError_t nt_dev_launch_call(const NtProgram* prog, const NtBatch* B, const NtOut* O,
                              const uint64_t* tmask, const uint32_t* thr, uint32_t thr_size, int fix_last,
                              int call_grid, hipStream_t stream);

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
                         int grid, int call_grid, hipStream_t stream) {
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
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || call_grid <= 0) return e;
  return nt_dev_launch_call(prog, B, O, tmask, thr, 0, 0, call_grid, stream);
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
                              int call_grid, hipStream_t stream) {
  hipLaunchKernelGGL(nt::nt_call_kernel, dim3(call_grid), dim3(256), 0, stream, prog, *B, *O, tmask, thr,
                     thr_size, fix_last);
  return hipGetLastError();
}

hipError_t nt_dev_launch_bundle(const NtBatch* B, uint64_t n_stripes, uint32_t* tp, int L, uint32_t div_m,
                                uint32_t div_s, hipStream_t stream, int cu_count) {
  // one workgroup per bundle (its half stripes in turn), a grid-stride loop over them
  uint64_t grid = n_stripes ? B->n_bundles : 0;
  if (grid > (uint64_t)cu_count * 16) grid = (uint64_t)cu_count * 16;
  if (grid == 0) return hipSuccess;
  const size_t lds = ((size_t)((L + 1) / 2) * nt::kBndRowWords + (size_t)NT_BUNDLE * (2 * L + 2) + 4 * NT_BUNDLE) * 4;
  hipLaunchKernelGGL(nt::nt_bundle_kernel, dim3((uint32_t)grid), dim3(256), lds, stream, *B, tp, L, div_m, div_s);
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
