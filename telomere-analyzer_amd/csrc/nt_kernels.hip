// nt_kernels.hip -- NanoTel hot path on MI355X (gfx950 / CDNA4).
//
// One workgroup (4 waves) owns one read at a time (grid-stride over reads):
//   1. scan   : bit-sliced matchPattern of every pattern at 32 starts per lane
//               (exact and <=1 mismatch in the same pass, Biostrings OOB rule),
//               coverage = OR of shifted hit words (trim + IRanges::reduce),
//               coverage words of every pass kept in LDS.
//   2. windows: per-window covered-base counts (get_sub_density numerators,
//               analyze_subtelos NanoTel.R:717-766) -> LDS + HBM (uint16).
//   3. call   : wave p runs pass p's telomere calling (A8-A12:
//               find_telo_position, _wraper, get_accurate_*, find_left/right,
//               search_left/right_patterns) with ballot bitmasks over windows
//               and LDS coverage range queries; fp64 sums in R's order.
//   4. row    : analyze_read row fields (NanoTel.R:1840-1974).
// No MFMA: this is integer/bit work bound by HBM.
#include <hip/hip_runtime.h>

#include "nt_common.h"
#include "nt_device.h"
#include "nt_rng.h"

namespace nt {

struct Pos {
  int64_t s, e;
};

// Per-pass calling context (uniform across the calling wave).
struct PassCtx {
  ReadCtx rc;  // by value: taking the address of a local would force it to scratch
  const NtProgram* prog;
  const uint32_t* cov;  // coverage words, position space: word i = positions [32i, 32i+31]
  const uint16_t* cnt;  // window counts
  const uint64_t* tm;   // telomeric-window bitmask
  int64_t n, nw, nmw;
  int32_t nblk;
  int L;
  int k;        // 0 for P1, 1 for P2/P3
  bool use_tvr; // P3
  bool raw;     // P1 with raw views (single fixed pattern)
  int lane;
};

__device__ __forceinline__ int64_t wstart(const PassCtx& c, int64_t i) { return 1 + i * (int64_t)c.L; }
__device__ __forceinline__ int64_t wend(const PassCtx& c, int64_t i) {
  return i == c.nw - 1 ? c.n : wstart(c, i) + c.L - 1;
}
__device__ __forceinline__ double wdens(const PassCtx& c, int64_t i) {
  return (double)c.cnt[i] / (double)(wend(c, i) - wstart(c, i) + 1);
}

// ---------------------------------------------------------- window bitmask

__device__ __forceinline__ bool tbit(const PassCtx& c, int64_t i) {
  return (c.tm[i >> 6] >> (i & 63)) & 1ull;
}
__device__ __forceinline__ int64_t next_set(const PassCtx& c, int64_t pos, bool inv) {
  if (pos >= c.nw) return c.nw;
  int64_t wi = pos >> 6;
  uint64_t x = (inv ? ~c.tm[wi] : c.tm[wi]) & (~0ull << (pos & 63));
  for (;;) {
    if (x) {
      const int64_t r = (wi << 6) + __builtin_ctzll(x);
      return r < c.nw ? r : c.nw;
    }
    if (++wi >= c.nmw) return c.nw;
    x = inv ? ~c.tm[wi] : c.tm[wi];
  }
}
__device__ __forceinline__ int64_t prev_set(const PassCtx& c, int64_t pos, bool inv) {
  if (pos < 0) return -1;
  if (pos >= c.nw) pos = c.nw - 1;
  int64_t wi = pos >> 6;
  const uint32_t b = (uint32_t)(pos & 63);
  uint64_t x = (inv ? ~c.tm[wi] : c.tm[wi]) & (b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull));
  for (;;) {
    if (x) return (wi << 6) + 63 - __builtin_clzll(x);
    if (--wi < 0) return -1;
    x = inv ? ~c.tm[wi] : c.tm[wi];
  }
}

// ------------------------------------------------------ coverage queries

// 32 coverage bits of positions [p, p+31] (0 outside the read).
__device__ __forceinline__ uint32_t cov_at(const PassCtx& c, int64_t p) {
  const int64_t b = p >> 5;
  const uint32_t off = (uint32_t)(p & 31);
  const uint32_t x = (b >= 0 && b < c.nblk) ? c.cov[b] : 0u;
  const uint32_t y = (b + 1 >= 0 && b + 1 < c.nblk) ? c.cov[b + 1] : 0u;
  return funnel(y, x, off);
}

// sum(width(intersect(IRanges(a1, b1), ranges))) -- wave-parallel popcount.
__device__ __forceinline__ int64_t range_count(const PassCtx& c, int64_t a1, int64_t b1) {
  int64_t a = (a1 < 1 ? 1 : a1) - 1, b = (b1 > c.n ? c.n : b1) - 1;
  if (a > b) return 0;
  const int64_t ia = a >> 5, ib = b >> 5;
  uint32_t acc = 0;
  for (int64_t i = ia + c.lane; i <= ib; i += kWave) {
    uint32_t w = c.cov[i];
    if (i == ia) w &= 0xFFFFFFFFu << (uint32_t)(a & 31);
    if (i == ib) w &= 0xFFFFFFFFu >> (uint32_t)(31 - (b & 31));
    acc += __builtin_popcount(w);
  }
  return (int64_t)wave_sum_u32(acc);
}

__device__ __forceinline__ double sub_density(const PassCtx& c, int64_t s, int64_t e) {
  return (double)range_count(c, s, e) / (double)(e - s + 1);
}

// Run-start / run-end / raw-hit bits for positions [p, p+31] of this pass's
// range set (IRanges starts/ends).  kind: 0 = starts, 1 = ends.
__device__ __forceinline__ uint32_t range_marks(const PassCtx& c, int64_t p, int kind) {
  if (c.raw) {
    // raw views of the single fixed pattern: starts = hit starts; ends =
    // starts + m - 1 (bit for position e-1 set when a view ends at e).
    const NtPat& P = c.prog->pat[0];
    const int64_t base = kind == 0 ? p : p - (P.m - 1);
    uint32_t a0, a1;
    hits_at(c.rc, P, false, base, 0, c.n - 1, a0, a1);
    return a0;
  }
  const uint32_t cw = cov_at(c, p);
  return kind == 0 ? (cw & ~cov_at(c, p - 1)) : (cw & ~cov_at(c, p + 1));
}

// min(start(ranges)) with start in [a1, b1] (1-based); returns fallback if none.
__device__ __forceinline__ int64_t min_start_in(const PassCtx& c, int64_t a1, int64_t b1, int64_t fallback) {
  int64_t a = a1 - 1, b = b1 - 1;  // 0-based position of the start
  if (a < 0) a = 0;
  if (b > c.n - 1) b = c.n - 1;
  if (a > b) return fallback;
  const int64_t nchunk = ((b - a) >> 5) + 1;  // <= 4 for the A10 spans
  int64_t best = INT64_MAX;
  for (int64_t c0 = 0; c0 < nchunk; c0 += kWave) {
    const int64_t ch = c0 + c.lane;
    uint32_t w = 0u;
    if (ch < nchunk) {
      const int64_t p = a + 32 * ch;
      w = range_marks(c, p, 0) & range_mask(p, a, b);
    }
    const uint64_t bal = __ballot(w != 0u);
    if (bal) {
      const int l = __builtin_ctzll(bal);
      const uint32_t wl = __shfl(w, l, kWave);
      best = a + 32 * (c0 + l) + __builtin_ctz(wl);
      break;
    }
  }
  return best == INT64_MAX ? fallback : best + 1;
}

// max(end(ranges)) with end in [a1, b1]; returns fallback if none.
__device__ __forceinline__ int64_t max_end_in(const PassCtx& c, int64_t a1, int64_t b1, int64_t fallback) {
  int64_t a = a1 - 1, b = b1 - 1;  // 0-based position of the last base
  if (a < 0) a = 0;
  if (b > c.n - 1) b = c.n - 1;
  if (a > b) return fallback;
  const int64_t nchunk = ((b - a) >> 5) + 1;
  int64_t best = -1;
  const int64_t top = ((nchunk + kWave - 1) / kWave) * kWave;
  for (int64_t c0 = top - kWave; c0 >= 0; c0 -= kWave) {
    const int64_t ch = c0 + c.lane;
    uint32_t w = 0u;
    if (ch < nchunk) {
      const int64_t p = a + 32 * ch;
      w = range_marks(c, p, 1) & range_mask(p, a, b);
    }
    const uint64_t bal = __ballot(w != 0u);
    if (bal) {
      const int l = 63 - __builtin_clzll(bal);
      const uint32_t wl = __shfl(w, l, kWave);
      best = a + 32 * (c0 + l) + 31 - __builtin_clz(wl);
      break;
    }
  }
  return best < 0 ? fallback : best + 1;
}

// ----------------------------------------------------------- A8 / A9 / A11

// find_telo_position (NanoTel.R:973-1077) on the window bitmask.
__device__ __forceinline__ Pos find_telo_position(const PassCtx& c, int64_t min_in_a_row, double thr) {
  int64_t pos = 0, found = -1, start = -1;
  for (;;) {
    const int64_t r = next_set(c, pos, false);
    if (r >= c.nw) break;
    const int64_t q = next_set(c, r, true) - 1;  // end of the run of telomeric windows
    if (q - r + 1 >= min_in_a_row) {
      double score = 0.0;
      for (int64_t j = r; j <= q; ++j) {
        score = score + wdens(c, j);
        if (j - r + 1 >= min_in_a_row && score >= thr) { found = j; break; }
      }
      if (found >= 0) { start = wstart(c, r); break; }
    }
    pos = q + 1;
  }
  if (found < 0) return Pos{-1, -1};
  const int64_t ep = found + 2;  // end_position, 1-based
  int64_t end = -1;
  if (ep >= c.nw - min_in_a_row + 1) {
    if (c.nw > ep) {
      const int64_t j = prev_set(c, c.nw - 1, false);
      end = (j >= ep) ? wend(c, j) : wend(c, ep - 1);
    } else {
      end = wend(c, c.nw - 1);
    }
  } else {
    // for (i in nrow:end_position): windows nw-1 .. ep-1 (0-based), reset/accumulate
    const int64_t lo = ep - 1;
    bool hit = false;
    int64_t p2 = c.nw - 1;
    for (;;) {
      const int64_t q = prev_set(c, p2, false);
      if (q < lo) break;
      const int64_t rr = prev_set(c, q, true) + 1;  // bottom of the run
      const int64_t r = rr > lo ? rr : lo;
      if (q - r + 1 >= min_in_a_row) {
        double score = 0.0;
        for (int64_t j = q; j >= r; --j) {
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
__device__ __forceinline__ Pos find_left_telo(const PassCtx& c) {
  if (c.nw == 0) return Pos{1, 1};
  const int64_t f = next_set(c, 0, false);
  if (f < c.nw && wstart(c, f) <= 200) {
    const int64_t e = next_set(c, f, true) - 1;
    return Pos{wstart(c, f), wend(c, e)};
  }
  if (wstart(c, c.nw - 1) > 200) return Pos{-1, -1};
  return Pos{1, 1};
}

// find_right_telo (NanoTel.R:843-899).  err=true on a 0-row table.
__device__ __forceinline__ Pos find_right_telo(const PassCtx& c, bool& err) {
  if (c.nw == 0) { err = true; return Pos{1, 1}; }
  const int64_t g = prev_set(c, c.nw - 1, false);
  if (g >= 0) {
    if (wend(c, g) < c.n - 200) return Pos{-1, -1};
    const int64_t r = prev_set(c, g, true) + 1;
    return Pos{wstart(c, r), wend(c, g)};
  }
  if (wend(c, 0) < c.n - 200) return Pos{-1, -1};
  return Pos{1, 1};
}

// ----------------------------------------------------------------- A10

// get_accurate_start (NanoTel.R:1726-1764)
__device__ __forceinline__ int64_t accurate_start(const PassCtx& c, int64_t s) {
  if (s == -1) return -1;
  const double first_50 = (double)range_count(c, s, s + 49) / 50.0;
  int64_t t = s;
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
__device__ __forceinline__ int64_t accurate_end(const PassCtx& c, int64_t e) {
  if (e == -1) return -1;
  int64_t t = max_end_in(c, e - 99, e, e);
  t = max_end_in(c, e + 1, e + 50, t);
  return t;
}

// ----------------------------------------------------------------- A12

// max end / min start of fixed=TRUE matches of the pass's pattern set in the
// sub-sequence [a1, b1] (multi_pattern_step_right/left NanoTel.R:496-575;
// out-of-bound relative to the sub-sequence, no trim).
__device__ __forceinline__ bool step_extreme(const PassCtx& c, int64_t a1, int64_t b1, bool want_end, int64_t& val) {
  const int64_t A = a1 - 1, B = b1 - 1;
  const int64_t base = A - 1;
  const bool only_exact = c.use_tvr && c.k == 0;
  bool any = false;
  int64_t best = want_end ? INT64_MIN : INT64_MAX;
  const int npat = c.prog->n_pat + (c.use_tvr ? c.prog->n_tvr : 0);
  for (int q = 0; q < npat; ++q) {
    const bool is_tvr = q >= c.prog->n_pat;
    const NtPat& P = is_tvr ? c.prog->tvr[q - c.prog->n_pat] : c.prog->pat[q];
    const int k = (is_tvr || only_exact) ? 0 : c.k;
    uint32_t a0, a1;
    hits_at(c.rc, P, true, base, A, B, a0, a1);
    const uint32_t h = k ? a1 : a0;
    if (!h) continue;
    any = true;
    if (want_end) {
      const int64_t e1 = base + (31 - __builtin_clz(h)) + P.m;
      if (e1 > best) best = e1;
    } else {
      const int64_t s1 = base + __builtin_ctz(h) + 1;
      if (s1 < best) best = s1;
    }
  }
  if (any) val = best;
  return any;
}

// search_right_patterns (NanoTel.R:635-697): width 18, step 10, 4 steps
__device__ __forceinline__ int64_t search_right(const PassCtx& c, int64_t end_index) {
  int64_t subseq_end = end_index + 18 < c.n ? end_index + 18 : c.n;
  int64_t new_end = end_index;
  for (int it = 0; it < 4; ++it) {
    const int64_t curr_start = subseq_end - 17 > 1 ? subseq_end - 17 : 1;
    int64_t v;
    if (!step_extreme(c, curr_start, subseq_end, true, v)) break;
    new_end = v;
    const int64_t ne = subseq_end + 11 < c.n ? subseq_end + 11 : c.n;
    if (ne == subseq_end) break;
    subseq_end = ne;
  }
  return new_end;
}

// search_left_patterns (NanoTel.R:576-633)
__device__ __forceinline__ int64_t search_left(const PassCtx& c, int64_t start_index) {
  int64_t subseq_start = start_index - 18 > 1 ? start_index - 18 : 1;
  int64_t new_start = start_index;
  for (int it = 0; it < 4; ++it) {
    const int64_t curr_end = subseq_start + 17 < c.n ? subseq_start + 17 : c.n;
    int64_t v;
    if (!step_extreme(c, subseq_start, curr_end, false, v)) break;
    new_start = v;
    const int64_t ns = subseq_start - 9 > 1 ? subseq_start - 9 : 1;
    if (ns == subseq_start) break;
    subseq_start = ns;
  }
  return new_start;
}

// find_telo_position_wraper (NanoTel.R:1080-1155) + density (NanoTel.R:1840).
__device__ __forceinline__ void call_pass(const PassCtx& c, int64_t& out_s, int64_t& out_e, double& out_d,
                          uint32_t& err) {
  Pos tp = find_telo_position(c, 3, 2.0);
  const double telo_density = sub_density(c, tp.s, tp.e);
  const int64_t num_rows = (tp.e - tp.s + 1) / c.L;
  if (telo_density < 0.85 && num_rows > 5) {
    const int64_t min_rows = num_rows <= 7 ? num_rows - 2 : 7;
    const double min_density = 0.6 * (double)min_rows;
    tp = find_telo_position(c, min_rows, min_density);
  }
  const int64_t s_acc = accurate_start(c, tp.s);
  int64_t e_acc = accurate_end(c, tp.e);
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
    int64_t e2 = tp.e, s2 = tp.s;
    if (tp.e < c.n) e2 = search_right(c, tp.e + 1);
    if (tp.s > 1) s2 = search_left(c, tp.s - 1);
    tp = Pos{s2, e2};
  }
  if (tp.e < tp.s - 1) { err |= NT_FLAG_ERR_WIDTH; out_s = -1; out_e = -1; out_d = 0.0; return; }
  out_s = tp.s;
  out_e = tp.e;
  out_d = sub_density(c, tp.s, tp.e);
}

// --------------------------------------------------------------- the kernel

struct LdsLayout {
  uint32_t cov_words;  // per pass
  uint32_t cnt_words;  // per pass (uint16 pairs)
  uint32_t tm_words;   // per pass (uint32 words of the uint64 mask; even)
  uint32_t total;      // words for all passes
};

__host__ __device__ inline LdsLayout lds_layout(int64_t n, int L, int np) {
  LdsLayout l;
  const int64_t nblk = (n + 31) / 32;
  int64_t nw = 0;
  if (n > 0 && L > 0) {
    nw = (n - 1) / L + 1;
    const int64_t last_start = 1 + (nw - 1) * (int64_t)L;
    if ((double)(n - last_start) < (double)L / 2.0) nw -= 1;
  }
  l.cov_words = (uint32_t)((nblk + 1) & ~1ll);
  l.cnt_words = (uint32_t)((((nw + 1) / 2) + 1) & ~1ll);
  l.tm_words = (uint32_t)(((nw + 63) / 64) * 2);
  l.total = (uint32_t)np * (l.cov_words + l.cnt_words + l.tm_words);
  return l;
}

template <bool kGlobal>
__global__ void __launch_bounds__(kWG)
nt_scan_call_kernel(const NtProgram* __restrict__ prog, NtBatch B, NtOut O, uint32_t len_lo,
                    uint32_t len_hi, uint32_t* __restrict__ gscratch, uint64_t scratch_words) {
  extern __shared__ uint32_t smem[];
  __shared__ uint32_t s_hits[3 * NT_MAX_PAT];
  __shared__ int64_t s_res_s[NT_MAX_PASS], s_res_e[NT_MAX_PASS];
  __shared__ double s_res_d[NT_MAX_PASS];
  __shared__ uint32_t s_err;

  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
  const int np = prog->n_pass, L = prog->L;
  const int n_pat = prog->n_pat, n_tvr = prog->n_tvr;
  const double min_density = prog->min_density;
  uint32_t* store = kGlobal ? gscratch + (uint64_t)blockIdx.x * scratch_words : smem;

  for (uint64_t r = blockIdx.x; r < B.n_reads; r += gridDim.x) {
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
    const int64_t n = rc.n;
    const int32_t nblk = rc.nblk;
    const int64_t nw = split_window_count(n, L);
    const LdsLayout lay = lds_layout(n, L, np);
    uint32_t* cov = store;
    uint16_t* cnt = reinterpret_cast<uint16_t*>(store + np * lay.cov_words);
    uint64_t* tm = reinterpret_cast<uint64_t*>(store + np * (lay.cov_words + lay.cnt_words));

    if (tid < 3 * NT_MAX_PAT) s_hits[tid] = 0u;
    if (tid == 0) s_err = 0u;
    __syncthreads();

    // ---------------------------------------------------------------- scan
    // Offset-space word w covers positions [32(w-1), 32(w-1)+31]; words
    // 0..nblk hold hit starts (start -1 lives in word 0), coverage is kept for
    // words 1..nblk.  Lane 0 of every wave-chunk recomputes the word before
    // the chunk so that lanes 1..63 get their carry-in starts by a shuffle.
    for (int64_t c0 = (int64_t)wave * kOwned; c0 <= nblk; c0 += (int64_t)kOwned * kNWaves) {
      const int64_t w = c0 + lane - 1;
      const int64_t base = 32 * (w - 1);
      const bool owned = lane >= 1 && w <= nblk;
      const uint2 b0 = load_blk(rc, w - 1), b1 = load_blk(rc, w);
      const uint32_t V0 = range_mask(base, 0, n - 1), V1 = range_mask(base + 32, 0, n - 1);
      uint32_t cv0 = 0u, cv1 = 0u, cv2 = 0u;
      for (int p = 0; p < n_pat; ++p) {
        const NtPat& P = prog->pat[p];
        uint32_t a0, a1;
        hits32(b0.x, b1.x, b0.y, b1.y, V0, V1, P.tt_scan, P.m, a0, a1);
        if (P.m <= 1) a1 &= V0;
        if (rc.n_exc) patch_exceptions(rc, base, 0, n - 1, P, false, a0, a1);
        const uint32_t h0 = wave_sum_u32(owned ? (uint32_t)__builtin_popcount(a0) : 0u);
        const uint32_t h1 = wave_sum_u32(owned ? (uint32_t)__builtin_popcount(a1) : 0u);
        if (lane == 0) {
          atomicAdd(&s_hits[p], h0);
          atomicAdd(&s_hits[n_pat + p], h1);
        }
        const uint32_t p0 = __shfl_up(a0, 1, kWave), p1 = __shfl_up(a1, 1, kWave);
        cv0 |= spread(a0, p0, P.m);
        cv1 |= spread(a1, p1, P.m);
      }
      if (np == 3) {
        cv2 = cv1;
        for (int t = 0; t < n_tvr; ++t) {
          const NtPat& P = prog->tvr[t];
          uint32_t a0, a1;
          hits32(b0.x, b1.x, b0.y, b1.y, V0, V1, P.tt_scan, P.m, a0, a1);
          if (rc.n_exc) patch_exceptions(rc, base, 0, n - 1, P, false, a0, a1);
          const uint32_t h0 = wave_sum_u32(owned ? (uint32_t)__builtin_popcount(a0) : 0u);
          if (lane == 0) atomicAdd(&s_hits[2 * n_pat + t], h0);
          const uint32_t p0 = __shfl_up(a0, 1, kWave);
          cv2 |= spread(a0, p0, P.m);
        }
      }
      if (owned && w >= 1) {
        cov[w - 1] = cv0 & V0;
        cov[lay.cov_words + w - 1] = cv1 & V0;
        if (np == 3) cov[2 * lay.cov_words + w - 1] = cv2 & V0;
      }
    }
    __syncthreads();

    // ------------------------------------------------------- window counts
    for (int64_t i = tid; i < nw; i += kWG) {
      const int64_t ws = i * (int64_t)L;
      const int64_t we = (i == nw - 1) ? n - 1 : ws + L - 1;
      for (int p = 0; p < np; ++p) {
        const uint32_t* cp = cov + p * lay.cov_words;
        uint32_t acc = 0;
        for (int64_t wi = ws >> 5; wi <= (we >> 5); ++wi) {
          uint32_t x = cp[wi];
          if (wi == (ws >> 5)) x &= 0xFFFFFFFFu << (uint32_t)(ws & 31);
          if (wi == (we >> 5)) x &= 0xFFFFFFFFu >> (uint32_t)(31 - (we & 31));
          acc += __builtin_popcount(x);
        }
        cnt[p * (2 * lay.cnt_words) + i] = (uint16_t)acc;
        if (O.win_counts) O.win_counts[B.win_off[r] * np + (uint64_t)p * nw + i] = (uint16_t)acc;
      }
    }
    __syncthreads();

    // ------------------------------------------------------------- calling
    if (wave < np) {
      const int p = wave;
      PassCtx c;
      c.rc = rc;
      c.prog = prog;
      c.cov = cov + p * lay.cov_words;
      c.cnt = cnt + p * (2 * lay.cnt_words);
      uint64_t* tmp = tm + p * (lay.tm_words / 2);
      c.tm = tmp;
      c.n = n;
      c.nw = nw;
      c.nmw = (nw + 63) >> 6;
      c.nblk = nblk;
      c.L = L;
      c.k = p == 0 ? 0 : 1;
      c.use_tvr = p == 2;
      c.raw = p == 0 && prog->raw_p1;
      c.lane = lane;
      // telomeric-window bitmask: class -5 iff !(density < min_density)
      for (int64_t ch = 0; ch < c.nmw; ++ch) {
        const int64_t i = ch * 64 + lane;
        bool t = false;
        if (i < nw) t = !(wdens(c, i) < min_density);
        const uint64_t bal = __ballot(t);
        if (lane == 0) tmp[ch] = bal;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      int64_t s, e;
      double d;
      uint32_t err = 0;
      call_pass(c, s, e, d, err);
      if (lane == 0) {
        s_res_s[p] = s;
        s_res_e[p] = e;
        s_res_d[p] = d;
        if (err) atomicOr(&s_err, err);
      }
    }
    __syncthreads();

    // ----------------------------------------------------------------- row
    if (tid == 0) {
      int64_t maxw = INT64_MIN;
      uint32_t flags = NT_FLAG_DONE | s_err;
      for (int p = 0; p < np; ++p) {
        const int64_t wdt = s_res_e[p] - s_res_s[p] + 1;
        if (wdt > maxw) maxw = wdt;
        if (s_res_s[p] == -1) flags |= 1u << (NT_FLAG_NA_SHIFT + p);
        O.start[r * 3 + p] = (int32_t)s_res_s[p];
        O.end[r * 3 + p] = (int32_t)s_res_e[p];
        O.density[r * 3 + p] = s_res_d[p];
      }
      for (int p = np; p < 3; ++p) {
        O.start[r * 3 + p] = -1;
        O.end[r * 3 + p] = -1;
        O.density[r * 3 + p] = 0.0;
      }
      if (maxw >= 30) flags |= NT_FLAG_TELOMERIC;
      O.flags[r] = (uint8_t)flags;
    }
    if (O.hits && tid < prog->n_hits) O.hits[r * (uint64_t)prog->n_hits + tid] = s_hits[tid];
    __syncthreads();
  }
}

// ------------------------------------------------------------ synthetic reads

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

// ------------------------------------------------------------- launchers

extern "C" {

uint32_t nt_dev_lds_words(int64_t n, int L, int np) { return nt::lds_layout(n, L, np).total; }

hipError_t nt_dev_launch_scan_call(const NtProgram* prog_dev, const NtBatch* B, const NtOut* O,
                                   uint32_t len_lo, uint32_t len_hi, int global_scratch,
                                   uint32_t* gscratch, uint64_t scratch_words, uint32_t lds_words,
                                   int grid, hipStream_t stream) {
  if (global_scratch) {
    hipLaunchKernelGGL(nt::nt_scan_call_kernel<true>, dim3(grid), dim3(nt::kWG), 0, stream,
                       prog_dev, *B, *O, len_lo, len_hi, gscratch, scratch_words);
  } else {
    hipLaunchKernelGGL(nt::nt_scan_call_kernel<false>, dim3(grid), dim3(nt::kWG),
                       (size_t)lds_words * 4u, stream, prog_dev, *B, *O, len_lo, len_hi,
                       (uint32_t*)nullptr, (uint64_t)0);
  }
  return hipGetLastError();
}

hipError_t nt_dev_set_lds_limit(uint32_t bytes) {
  return hipFuncSetAttribute((const void*)nt::nt_scan_call_kernel<false>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
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
