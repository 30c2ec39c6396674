// nt_call.h -- the telomere calling kernel (find_telo_position_wraper and
// callees, NanoTel.R:973-1155, 1692-1764, 843-959, 496-697; analyze_read's
// row, NanoTel.R:1840-1974) from the scan's window counts and bitmasks.
//
// The calling kernel is bound by dependent memory round trips (one lane per
// read-pass walks its read), so each step loads what it needs as one batch of
// independent loads: the telomeric-bitmask words up front (reads of <= 512
// windows), the counts of a run four windows at a time, both A10
// neighbourhoods together, both edge-extension plane windows together, and
// the two partial windows of a range count together with its checkpoints.
//
// Compiled twice: ahead of time with run-time pattern lists (RtCall,
// nt_kernels.hip), and by hiprtc with the program's patterns as types
// (CtCall, nt_jit.cpp), where every letter test is a constant truth table
// (one v_bitop3 with the validity mask, shared across letters and patterns)
// and the m letters of a pattern combine three at a time -- the boundary
// neighbourhoods recompute coverage of every pattern at every start, which
// is most of the kernel's VALU work with several patterns.
#pragma once
#include "nt_scan.h"

namespace nt {

// The two-range recounts (cov_count2, accurate_both) are written as 2-trip
// loops: NT_CALL_ROLLED=1 keeps them rolled,
// one coverage-computation site each (a smaller kernel, hiprtc builds ~2x
// faster), 0 unrolls them into two copies.  Unrolled measured faster (fewer
// live registers across the sites: 118 VGPRs, 4 waves/SIMD, against 162-168
// and spills rolled; calling at c10k 0.51 vs 0.58 ms, c4 3.57 vs 3.84 ms;
// the ahead-of-time kernel 1.30 ms rolled with 111 spilled VGPRs).
#ifndef NT_CALL_ROLLED
#define NT_CALL_ROLLED 0
#endif
#if NT_CALL_ROLLED
#define NT_CALL_SITE_LOOP _Pragma("unroll 1")
#else
#define NT_CALL_SITE_LOOP _Pragma("unroll")
#endif

constexpr int kIntMin = -2147483647 - 1;
constexpr int kIntMax = 2147483647;

// Run-time IUPAC letters, code-equality semantics (fixed=TRUE: the edge steps).
template <int M>
struct RtTableEq {
  static constexpr int kM = M;
  const NtPat* P;
  __device__ __forceinline__ int m() const { return M > 0 ? M : P->m; }
  __device__ __forceinline__ uint32_t E(int j, uint32_t L, uint32_t H) const {
    const uint32_t* t = P->tm_eq[j];
    return bfi(H, bfi(L, t[3], t[2]), bfi(L, t[1], t[0]));
  }
};

// Pattern-set policies of the calling kernel: for_pat / for_tvr visit (index,
// descriptor) with the scan letter semantics (coverage, get_density_iranges),
// for_pat_eq / for_tvr_eq with code equality (the edge steps).  kNTvr: TVRs
// known at compile time (-1: read the program).
struct RtCall {
  static constexpr int kNTvr = -1;
  static constexpr bool kMayRaw = true;  // P1 raw views possible (program's raw_p1)
  static constexpr bool kLong = false;   // TVRs of 33..64 letters (wider neighbourhoods)
  template <class F>
  __device__ __forceinline__ static void for_pat(const NtProgram* prog, F&& f) {
    for (int p = 0; p < prog->n_pat; ++p) f(p, RtTable<0>{&prog->pat[p]});
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr(const NtProgram* prog, F&& f) {
    for (int t = 0; t < prog->n_tvr; ++t) f(t, RtTable<0>{&prog->tvr[t]});
  }
  template <class F>
  __device__ __forceinline__ static void for_pat_eq(const NtProgram* prog, F&& f) {
    for (int p = 0; p < prog->n_pat; ++p) f(p, RtTableEq<0>{&prog->pat[p]});
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr_eq(const NtProgram* prog, F&& f) {
    for (int t = 0; t < prog->n_tvr; ++t) f(t, RtTableEq<0>{&prog->tvr[t]});
  }
};
// The same for programs with a TVR of more than 32 letters (host dispatch).
struct RtCallLong : RtCall {
  static constexpr bool kLong = true;
};

// Compile-time lists (hiprtc): CtList<CtPat<m, tt...>...> of the scan truth
// tables and of the code-equality ones, for the patterns and the TVRs.
template <class Pats, class Tvrs, class PatsEq, class TvrsEq, bool kRaw>
struct CtCall {
  static constexpr int kNTvr = Tvrs::kN;
  // raw_p1 (single fixed pattern) known: without it the raw-view marks and
  // their registers are compiled out
  static constexpr bool kMayRaw = kRaw;
  static constexpr bool kLong = CtMaxM<Tvrs>::value > 32;
  template <class F>
  __device__ __forceinline__ static void for_pat(const NtProgram* prog, F&& f) {
    CtVisit<Pats>::run(prog->pat, f);
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr(const NtProgram* prog, F&& f) {
    CtVisit<Tvrs>::run(prog->tvr, f);
  }
  template <class F>
  __device__ __forceinline__ static void for_pat_eq(const NtProgram* prog, F&& f) {
    CtVisit<PatsEq>::run(prog->pat, f);
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr_eq(const NtProgram* prog, F&& f) {
    CtVisit<TvrsEq>::run(prog->tvr, f);
  }
};

// Hits of descriptor d at the 32 starts of each hit word h in [0, NH), from
// the plane words Lw/Hw and validity Vw of positions [32h, 32h + 63] (words h,
// h + 1; with kX = 1, TVRs of 33..64 letters, [32h, 32h + 95]: words h .. h + 2):
// x0 exact, x1 <= 1 mismatch (invalid positions are mismatches).  Letter tests
// are made on the unshifted words and shifted by j.
// kExact: x0 only (a P1 kernel of the per-pass split; x1 is left undefined).
template <int NH, int kX, class D, bool kExact = false>
__device__ __forceinline__ void words_hits(const D& d, const uint32_t* Lw, const uint32_t* Hw,
                                           const uint32_t* Vw, uint32_t* x0, uint32_t* x1) {
  constexpr int kM = D::kM;
  if constexpr (kM > 0) {
    static_assert(kM <= 32 * (kX + 1), "pattern longer than the neighbourhood's plane words");
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      uint32_t q[kM];
#pragma unroll
      for (int j = 0; j < kM; ++j) {
        const int w = h + (j >> 5);
        const uint32_t e0 = d.E(j, Lw[w], Hw[w]) & Vw[w], e1 = d.E(j, Lw[w + 1], Hw[w + 1]) & Vw[w + 1];
        q[j] = funnel(e1, e0, (uint32_t)(j & 31));
      }
      combine<kM, kExact>(q, x0[h], x1[h]);
      if (kM <= 1) x1[h] &= Vw[h];
    }
  } else {
    const int m = d.m();
    const int m0 = m < 32 ? m : 32;
#pragma unroll
    for (int h = 0; h < NH; ++h) x0[h] = x1[h] = 0xFFFFFFFFu;
    for (int j = 0; j < m0; ++j) {
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const uint32_t Ls = funnel(Lw[h + 1], Lw[h], (uint32_t)j);
        const uint32_t Hs = funnel(Hw[h + 1], Hw[h], (uint32_t)j);
        const uint32_t q = d.E(j, Ls, Hs) & funnel(Vw[h + 1], Vw[h], (uint32_t)j);
        if (!kExact) x1[h] = (x1[h] & q) | x0[h];
        x0[h] &= q;
      }
    }
    if constexpr (kX > 0) {
      for (int j = 32; j < m; ++j) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          const uint32_t Ls = funnel(Lw[h + 2], Lw[h + 1], (uint32_t)(j - 32));
          const uint32_t Hs = funnel(Hw[h + 2], Hw[h + 1], (uint32_t)(j - 32));
          const uint32_t q = d.E(j, Ls, Hs) & funnel(Vw[h + 2], Vw[h + 1], (uint32_t)(j - 32));
          if (!kExact) x1[h] = (x1[h] & q) | x0[h];
          x0[h] &= q;
        }
      }
    }
    if (m <= 1) {
#pragma unroll
      for (int h = 0; h < NH; ++h) x1[h] &= Vw[h];
    }
  }
}

// A copy of the n words the compiler cannot prove equal to the originals
// (an empty asm per word): letter tests made from it are not common
// subexpressions of another pattern's, so they are recomputed (one op each)
// instead of held live across all the patterns (NT_CALL_LAUNDER).
#ifndef NT_CALL_LAUNDER
#define NT_CALL_LAUNDER 1
#endif
template <int N>
__device__ __forceinline__ void launder_words(const uint32_t* in, uint32_t* out) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    out[i] = in[i];
    if (NT_CALL_LAUNDER) asm volatile("" : "+v"(out[i]));
  }
}

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

constexpr int kExcLocal = 4;

// Per-lane state of one read-pass.
struct Lane {
  ReadCtx rc;
  uint32_t exc_lo, exc_hi;        // the read's first / last exception position (n_exc > 0)
  uint32_t xpos[kExcLocal];       // its exception positions when n_exc <= kExcLocal
  uint32_t xcode;                 // and their codes, 8 bits each
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

// A neighbourhood's hit words with the read's non-ACGT letters applied,
// patch_exceptions' result (nt_device.h; scan semantics: fixed = code
// equality, else IUPAC bit-set AND; positions outside the read mismatch) for
// every start of [hb, hb + 32 NH).  Bit-parallel over a touched word's 32
// starts: its hits are recomputed from the plane words in registers (Lw / Hw
// / Vw: positions [hb + 32 t, + 31], t < NP) with every exception letter
// counted as a match, then each exception letter's mismatches are added (a
// 2-bit saturating count, one exception letter per start and exception).  A
// read of at most kExcLocal letters has them in the lane's registers
// (Lane::xpos / xcode): no memory access.  (patch_exceptions per hit word
// looked every letter of every touched start up in memory; per start in
// registers it still made the calling kernel, latency-bound, the pipeline's
// bottleneck at c10k with 10 % of the reads carrying an N.)  One copy per
// pattern site: the touched words are selected by index.
template <int NH, int NP>
__device__ __forceinline__ void patch_words(const Lane& c, int64_t hb, const uint32_t* Lw, const uint32_t* Hw,
                                            const uint32_t* Vw, const NtPat& P, uint32_t* x0, uint32_t* x1) {
  const ReadCtx& rc = c.rc;
  const int m = P.m;
  const int64_t n = rc.n;
  const int64_t shi = hb + 32 * NH - 1;  // the last start
  const int64_t xlo = hb > 0 ? hb : 0;
  int64_t xhi = shi + m - 1;
  if (xhi > n - 1) xhi = n - 1;
  if (xlo > xhi || xhi < (int64_t)c.exc_lo || xlo > (int64_t)c.exc_hi) return;
  const bool cached = rc.n_exc <= kExcLocal;
  auto exc_at = [&](int32_t i) -> int64_t {  // position of exception i
    uint32_t xi = 0u;
#pragma unroll
    for (int k = 0; k < kExcLocal; ++k) xi = k == i ? c.xpos[k] : xi;
    return cached ? (int64_t)xi : (int64_t)rc.exc_pos[i];
  };
  auto code_of = [&](int32_t i) -> uint32_t {
    return cached ? ((c.xcode >> (8 * (i & 3))) & 255u) : (uint32_t)rc.exc_code[i];
  };
  const int32_t i0 = cached ? 0 : exc_lower_bound(rc, xlo);
  const bool eqx = P.fixed != 0;
  int hdone = -1;  // words <= hdone recomputed
  for (int32_t i = i0; i < rc.n_exc; ++i) {
    const int64_t x = exc_at(i);
    if (x > xhi) break;
    if (x < xlo) continue;
    int h0 = (int)((x - m + 1 - hb) >> 5), h1 = (int)((x - hb) >> 5);  // (arithmetic shifts: floor)
    if (h0 <= hdone) h0 = hdone + 1;
    if (h0 < 0) h0 = 0;
    if (h1 > NH - 1) h1 = NH - 1;
    for (int h = h0; h <= h1; ++h) {
      const int64_t base = hb + 32 * h;
      // the exception letters of [base, base + 95] as bits (the starts' letters reach base + 31 + m - 1)
      const int32_t kb = cached ? 0 : exc_lower_bound(rc, base);
      uint32_t e0 = 0u, e1 = 0u, e2 = 0u;
      for (int32_t k = kb; k < rc.n_exc; ++k) {
        const int64_t y = exc_at(k) - base;
        if (y > 95) break;
        if (y < 0) continue;
        const uint32_t bit = 1u << (uint32_t)(y & 31);
        e0 |= y < 32 ? bit : 0u;
        e1 |= (y >= 32 && y < 64) ? bit : 0u;
        e2 |= y >= 64 ? bit : 0u;
      }
      uint32_t L0 = 0u, L1 = 0u, L2 = 0u, H0 = 0u, H1 = 0u, H2 = 0u, V0 = 0u, V1 = 0u, V2 = 0u;
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        L0 = u == h ? Lw[u] : L0;
        H0 = u == h ? Hw[u] : H0;
        V0 = u == h ? Vw[u] : V0;
        L1 = u == h + 1 ? Lw[u] : L1;
        H1 = u == h + 1 ? Hw[u] : H1;
        V1 = u == h + 1 ? Vw[u] : V1;
        L2 = u == h + 2 ? Lw[u] : L2;
        H2 = u == h + 2 ? Hw[u] : H2;
        V2 = u == h + 2 ? Vw[u] : V2;
      }
      uint32_t a0 = 0xFFFFFFFFu, a1 = 0xFFFFFFFFu;
      for (int j = 0; j < m; ++j) {  // the letters j of the 32 starts, exception letters as matches
        const bool lo = j < 32;
        const uint32_t sj = (uint32_t)(j & 31);
        const uint32_t Ls = lo ? funnel(L1, L0, sj) : funnel(L2, L1, sj);
        const uint32_t Hs = lo ? funnel(H1, H0, sj) : funnel(H2, H1, sj);
        const uint32_t Vs = lo ? funnel(V1, V0, sj) : funnel(V2, V1, sj);
        const uint32_t Es = lo ? funnel(e1, e0, sj) : funnel(e2, e1, sj);
        const uint32_t* t = P.tm_scan[j];
        const uint32_t q = (bfi(Hs, bfi(Ls, t[3], t[2]), bfi(Ls, t[1], t[0])) & Vs) | Es;
        a1 = (a1 & q) | a0;
        a0 &= q;
      }
      if (m <= 1) a1 &= V0;
      // each exception letter's mismatches (one letter per start and exception)
      for (int32_t k = kb; k < rc.n_exc; ++k) {
        const int64_t y = exc_at(k) - base;
        if (y > 31 + m - 1) break;
        if (y < 0) continue;
        const uint32_t cd = code_of(k);
        uint32_t M = 0u;
        for (int j = 0; j < m; ++j) {
          const int64_t sb = y - j;  // the start whose letter j is y
          const uint32_t pc = P.code[j];
          const bool mm = eqx ? (cd != pc) : ((cd & pc) == 0u);
          M |= (mm && sb >= 0 && sb < 32) ? (1u << (uint32_t)sb) : 0u;
        }
        a1 = (a1 & ~M) | (a0 & M);
        a0 &= ~M;
      }
#pragma unroll
      for (int u = 0; u < NH; ++u) {
        x0[u] = u == h ? a0 : x0[u];
        x1[u] = u == h ? a1 : x1[u];
      }
    }
    if (h1 > hdone) hdone = h1;
  }
}


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

// kX = 1 (TVRs of 33..64 letters): one more plane word each side.
template <int K, bool kMarks = true, int kX = 0>
struct NbBlocks {
  uint2 b[K + (kMarks ? 2 : 0) + 3 + 2 * kX];
};

template <int K, bool kMarks, int kX>
__device__ __forceinline__ void nb_fetch(const Lane& c, int q0, NbBlocks<K, kMarks, kX>& f) {
  constexpr int E = kMarks ? 1 : 0;
  constexpr int NP = K + 2 * E + 2 + 2 * kX;
  const int bb = (q0 >> 5) - E - 1 - kX;  // arithmetic shift: floor for q0 < 0
#pragma unroll
  for (int t = 0; t <= NP; ++t) {
    const int b = bb + t;
    f.b[t] = (b >= 0 && b < c.rc.nblk) ? c.rc.blk[b] : make_uint2(0u, 0u);
  }
}

// kPass: -1 = every pass of a read on lanes of one wave (run); 0, 1, 2 = one
// pass, a lane per read (run_pass: the per-pass split, where the pass's
// mismatch rule, TVR use and P1's raw views are compile-time).
template <class CS, int kPass = -1>
struct Call {
static constexpr int kX = CS::kLong ? 1 : 0;  // extra plane / hit word for TVRs of 33..64 letters
static __device__ __forceinline__ int pk(const Lane& c) { return kPass >= 0 ? (kPass ? 1 : 0) : c.k; }
static __device__ __forceinline__ bool ptvr(const Lane& c) { return kPass >= 0 ? kPass == 2 : c.use_tvr; }
static __device__ __forceinline__ bool praw(const Lane& c) { return CS::kMayRaw && kPass <= 0 && c.raw; }
static constexpr bool kTvrCode = CS::kNTvr != 0 && (kPass < 0 || kPass == 2);
using NbB4 = NbBlocks<4, false, kX>;
using NbB5 = NbBlocks<5, true, kX>;

template <int K, bool kMarks>
static __device__ __forceinline__ void nb_compute(const Lane& c, int q0, const NbBlocks<K, kMarks, kX>& f,
                                           Nb<K, kMarks>& nb) {
  constexpr int E = kMarks ? 1 : 0;  // extra word each side
  constexpr int NC = K + 2 * E;      // coverage words computed, i = -E..K-1+E
  constexpr int NP = NC + 2 + 2 * kX;  // plane words, positions [q0 + 32i, +31], i = -E-1-kX..K+E+kX
  constexpr int NH = NC + 1 + kX;    // hit words, starts [q0 + 32i, +31], i = -E-1-kX..K-1+E
  constexpr int T0 = -E - 1 - kX;    // index of plane / hit word 0
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
  // every pattern (P1 exact, P2/P3 <= 1 mismatch), then the TVRs (exact, P3
  // only): the lanes of a wave hold different passes, so all of them compute
  // the hits and each keeps its pass's
  CS::for_pat(prog, [&](int pi, auto d) {
    constexpr int kM = decltype(d)::kM;
    const int m = d.m();
    uint32_t x0[NH], x1[NH];
    uint32_t Lp[NP], Hp[NP], Vp[NP];
    launder_words<NP>(Lw, Lp);
    launder_words<NP>(Hw, Hp);
    launder_words<NP>(Vw, Vp);
    words_hits<NH, kX, decltype(d), kPass == 0>(d, Lp, Hp, Vp, x0, x1);
    if (c.rc.n_exc) patch_words<NH, NP>(c, (int64_t)q0 + 32 * T0, Lw, Hw, Vw, *d.P, x0, x1);
    // coverage word ci (i = ci - E) from hit words i and i - 1 (patterns <= 18 letters)
    const bool k1 = pk(c) != 0;
#pragma unroll
    for (int ci = 0; ci < NC; ++ci)
      nb.cov[ci + 1 - E] |= spread<kM>(k1 ? x1[ci + 1 + kX] : x0[ci + 1 + kX], k1 ? x1[ci + kX] : x0[ci + kX], m);
    if constexpr (kMarks) {
      if (praw(c) && pi == 0) {
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
          nb.rs[ci] = x0[ci + 1 + kX];
          nb.re[ci] = m > 1 ? funnel(x0[ci + 1 + kX], x0[ci + kX], (uint32_t)(32 - (m - 1))) : x0[ci + 1 + kX];
        }
      }
    }
  });
  if (kTvrCode && prog->n_tvr > 0) {
    CS::for_tvr(prog, [&](int, auto d) {
      constexpr int kM = decltype(d)::kM;
      uint32_t x0[NH], x1[NH];
      uint32_t Lp[NP], Hp[NP], Vp[NP];
      launder_words<NP>(Lw, Lp);
      launder_words<NP>(Hw, Hp);
      launder_words<NP>(Vw, Vp);
      words_hits<NH, kX>(d, Lp, Hp, Vp, x0, x1);
      if (c.rc.n_exc) patch_words<NH, NP>(c, (int64_t)q0 + 32 * T0, Lw, Hw, Vw, *d.P, x0, x1);
      if (ptvr(c)) {
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
          if constexpr (kX > 0)
            nb.cov[ci + 1 - E] |= spread_long<kM>(x0[ci + 2], x0[ci + 1], x0[ci], d.m());
          else
            nb.cov[ci + 1 - E] |= spread<kM>(x0[ci + 1], x0[ci], d.m());
        }
      }
    });
  }
#pragma unroll
  for (int ci = 0; ci < NC; ++ci) nb.cov[ci + 1 - E] &= Vw[ci + 1 + kX];
}

// |coverage ∩ [a, b]|, [a, b] within [q0, q0 + 32K)
template <int K, bool kMarks>
static __device__ __forceinline__ int nb_count(const Nb<K, kMarks>& nb, int a, int b) {
  int t = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) t += __builtin_popcount(nb.cov[i + 1] & range_mask((int64_t)nb.q0 + 32 * i, a, b));
  return t;
}

// min(start(ranges)) with start in [a1, b1] (1-based), fallback if none;
// run starts of the reduced coverage, or P1's raw view starts
template <int K>
static __device__ __forceinline__ int nb_min_start(const Lane& c, const Nb<K>& nb, int a1, int b1, int fallback) {
  const int a = max(a1 - 1, 0), b = min(b1 - 1, c.n - 1);
  int res = fallback;
  bool found = false;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const uint32_t cur = nb.cov[i + 1];
    const uint32_t mk = praw(c) ? nb.rs[i + 1] : (cur & ~((cur << 1) | (nb.cov[i] >> 31)));
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
static __device__ __forceinline__ int nb_max_end(const Lane& c, const Nb<K>& nb, int a1, int b1, int fallback) {
  const int a = max(a1 - 1, 0), b = min(b1 - 1, c.n - 1);
  int res = fallback;
  bool found = false;
#pragma unroll
  for (int i = K - 1; i >= 0; --i) {
    const uint32_t cur = nb.cov[i + 1];
    const uint32_t mk = praw(c) ? nb.re[i + 1] : (cur & ~((cur >> 1) | (nb.cov[i + 2] << 31)));
    const uint32_t m = mk & range_mask((int64_t)nb.q0 + 32 * i, a, b);
    if (!found && m) {
      res = nb.q0 + 32 * i + (31 - __builtin_clz(m)) + 1;
      found = true;
    }
  }
  return res;
}

// |coverage ∩ [x1, y1]| + |coverage ∩ [x2, y2]| (0-based positions; x > y:
// empty), 128 bases of each range per round: both ranges' blocks fetched in
// one batch, then ONE neighbourhood computation site in a rolled loop over the
// two (the pattern code is the bulk of the kernel: every inlined copy costs
// instruction cache and, specialised, hiprtc build time).
static __device__ __forceinline__ int cov_count2(const Lane& c, int x1, int y1, int x2, int y2) {
  int t = 0;
  while (x1 <= y1 || x2 <= y2) {
    NbB4 f1, f2;
    nb_fetch(c, x1, f1);
    nb_fetch(c, x2, f2);
NT_CALL_SITE_LOOP
    for (int i = 0; i < 2; ++i) {
      const int x = i ? x2 : x1, y = i ? y2 : y1;
      if (x <= y) {
        Nb<4, false> nb;
        nb_compute(c, x, f1, nb);
        t += nb_count(nb, x, min(y, x + 127));
      }
      f1 = f2;  // (the second range's blocks take the first's registers)
    }
    x1 += 128;
    x2 += 128;
  }
  return t;
}

static __device__ __forceinline__ int cov_count(const Lane& c, int x, int y) { return cov_count2(c, x, y, 0, -1); }

// sum(width(intersect(IRanges(a1, b1), ranges))): window counts for whole
// windows, recomputed coverage for the partial windows at the two ends.
// Covered bases of windows [0, k) (0 <= k <= nw): the scan's checkpoint at
// window 16*(k/16) plus at most 15 window counts (independent loads).
// 8-bit counts: the 16 counts of a checkpoint group are one aligned 16-byte
// load (rows start on 64-window boundaries), summed under a byte mask with
// v_dot4_u32_u8 -- one load instead of up to 15 (c10k: the two densities of
// a call 0.20 -> see DESIGN §4.2).
static __device__ __forceinline__ int cnt_before(const Lane& c, int k) {
  const int r = k & 15, k0 = k - r;
  int t = (int)c.ck[k >> 4];
  if (c.c8) {
    if (r > 0) {  // (r == 0: the group may lie past the row's allocation)
      const uint4 v = reinterpret_cast<const uint4*>(c.cnt)[k >> 4];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t acc = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nb = min(max(r - 4 * i, 0), 4);  // bytes of word i before window k
        const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        acc = __builtin_amdgcn_udot4(w[i] & m, 0x01010101u, acc, false);
      }
      t += (int)acc;
    }
    return t;
  }
#pragma unroll
  for (int i = 0; i < 15; ++i)
    if (i < r) t += wcount(c, k0 + i);
  return t;
}

static __device__ __forceinline__ int range_count(const Lane& c, int a1, int b1) {
  const int a = (a1 < 1 ? 1 : a1) - 1, b = (b1 > c.n ? c.n : b1) - 1;
  if (a > b) return 0;
  // coverage recounted over [x1, y1] and [x2, y2] (one cov_count2 site)
  int whole = 0, x1 = a, y1 = b, x2 = 0, y2 = -1;
  if (c.nw > 0) {
    const int L = c.L;
    const int ka = min(div_l(c.prog, a), c.nw - 1), kb = min(div_l(c.prog, b), c.nw - 1);
    const int ws_a = ka * L, we_b = kb == c.nw - 1 ? c.n - 1 : (kb + 1) * L - 1;
    const bool a_whole = a == ws_a, b_whole = b == we_b;
    if (ka == kb) {
      if (a_whole && b_whole) return wcount(c, ka);
    } else {
      // whole windows from the running counts, partial end windows from coverage
      whole = cnt_before(c, b_whole ? kb + 1 : kb) - cnt_before(c, a_whole ? ka : ka + 1);
      y1 = a_whole ? -1 : (ka + 1) * L - 1;
      x2 = kb * L;
      y2 = b_whole ? -1 : b;
    }
  }
  return whole + cov_count2(c, x1, y1, x2, y2);
}

static __device__ __forceinline__ double sub_density(const Lane& c, int s, int e) {
  return (double)range_count(c, s, e) / (double)(e - s + 1);
}

// ---------------------------------------------------------------- A8 / A11

// find_telo_position (NanoTel.R:973-1077) on the window bitmask; the scores
// are summed in R's order, the counts of a run fetched four at a time.
static __device__ __forceinline__ Pos find_telo_position(const Lane& c, int min_in_a_row, double thr) {
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
static __device__ __forceinline__ Pos find_left_telo(const Lane& c) {
  if (c.nw == 0) return Pos{1, 1};
  const int f = next_set(c, 0, false);
  if (f < c.nw && wstart(c, f) <= 200) return Pos{wstart(c, f), wend(c, next_set(c, f, true) - 1)};
  if (wstart(c, c.nw - 1) > 200) return Pos{-1, -1};
  return Pos{1, 1};
}

// find_right_telo (NanoTel.R:843-899).  err=true on a 0-row table.
static __device__ __forceinline__ Pos find_right_telo(const Lane& c, bool& err) {
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
static __device__ __forceinline__ void accurate_fetch(const Lane& c, int s, int e, NbB5& fs, NbB5& fe) {
  nb_fetch(c, s - 42, fs);
  nb_fetch(c, e - 102, fe);
}

static __device__ __forceinline__ void accurate_both(const Lane& c, int s, int e, const NbB5& fs,
                                                     const NbB5& fe, int& s_acc, int& e_acc) {
  s_acc = -1;
  e_acc = -1;
  // one neighbourhood computation site, start side then end side
  NbB5 f = fs;
NT_CALL_SITE_LOOP
  for (int i = 0; i < 2; ++i, f = fe) {
    if ((i ? e : s) == -1) continue;
    Nb<5> nb;
    nb_compute(c, i ? e - 102 : s - 42, f, nb);
    if (i == 0) {
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
    } else {
      const int t = nb_max_end(c, nb, e - 99, e, e);
      e_acc = nb_max_end(c, nb, e + 1, e + 50, t);
    }
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
static __device__ __forceinline__ void pw_load(const Lane& c, int q0, Pw<K>& w) {
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
static __device__ __forceinline__ void pw_at(const Lane& c, const Pw<K>& w, int p, uint32_t& L, uint32_t& H) {
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

// hits_at (nt_device.h) with the planes taken from the window, code-equality
// letters (descriptor d of for_pat_eq / for_tvr_eq)
template <int K, class D>
static __device__ __forceinline__ void hits_at_w(const Lane& c, const Pw<K>& w, const D& d, int base, int vlo,
                                                 int vhi, uint32_t& a0, uint32_t& a1) {
  // A TVR of more than 32 letters (exact only) never matches inside the
  // <= 18-base sub-sequence of a step: no hits.
  if constexpr (D::kM > 32) {
    a0 = a1 = 0u;
  } else {
    if (d.m() > 32) {
      a0 = a1 = 0u;
      return;
    }
    uint32_t Lw[2], Hw[2], Vw[2];
    pw_at(c, w, base, Lw[0], Hw[0]);
    pw_at(c, w, base + 32, Lw[1], Hw[1]);
    Vw[0] = range_mask(base, vlo, vhi);
    Vw[1] = range_mask((int64_t)base + 32, vlo, vhi);
    words_hits<1, 0>(d, Lw, Hw, Vw, &a0, &a1);
    if (c.rc.n_exc && (int64_t)base + 31 + d.m() - 1 >= c.exc_lo && (int64_t)base <= c.exc_hi)
      patch_exceptions(c.rc, base, vlo, vhi, *d.P, true, a0, a1);
  }
}

// max end (right) / min start (left) of the fixed=TRUE matches of the pass's
// pattern set in the sub-sequence [a1, b1], out-of-bound relative to the
// sub-sequence (multi_pattern_step_right/left, NanoTel.R:496-575).
template <int K>
static __device__ __forceinline__ bool step_extreme(const Lane& c, const Pw<K>& w, int a1, int b1, bool right, int& val) {
  const NtProgram* prog = c.prog;
  const int A = a1 - 1, Bz = b1 - 1, base = A - 1;
  const bool only_exact = ptvr(c) && pk(c) == 0;
  bool any = false;
  int best = right ? kIntMin : kIntMax;
  auto visit = [&](bool is_tvr, const auto& d) {
    const int k = (is_tvr || only_exact) ? 0 : pk(c);
    uint32_t a0, a1w;
    hits_at_w(c, w, d, base, A, Bz, a0, a1w);
    uint32_t h = k ? a1w : a0;
    if (is_tvr && !ptvr(c)) h = 0u;  // TVRs extend P3 only
    if (!h) return;
    any = true;
    if (right) best = max(best, base + (31 - __builtin_clz(h)) + d.m());
    else best = min(best, base + __builtin_ctz(h) + 1);
  };
  CS::for_pat_eq(prog, [&](int, auto d) { visit(false, d); });
  if (kTvrCode && prog->n_tvr > 0) CS::for_tvr_eq(prog, [&](int, auto d) { visit(true, d); });
  if (any) val = best;
  return any;
}

// search_right_patterns (NanoTel.R:635-697): width 18, step 10, 4 steps.
// Match bases from max(min(end_index + 18, n) - 17, 1) - 2, up to +33.
template <int K>
static __device__ __forceinline__ int search_right(const Lane& c, const Pw<K>& w, int end_index) {
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
static __device__ __forceinline__ int search_left(const Lane& c, const Pw<K>& w, int start_index) {
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

// exc_windows (nt_common.h, the rule nt_exc_marks applies on the host) over
// the lane's exceptions: from its registers when the read has at most
// kExcLocal, else from memory.
template <class F>
static __device__ __forceinline__ int lane_exc_windows(const Lane& c, int cap, F&& f) {
  const int mm = c.prog->m_max, L = c.L, nw = c.nw, n = c.n;
  int cnt = 0, next = 0;
  for (int32_t i = 0; i < c.rc.n_exc && next < nw - 1; ++i) {
    uint32_t xi = 0u;
#pragma unroll
    for (int k = 0; k < kExcLocal; ++k) xi = k == i ? c.xpos[k] : xi;
    const int p = c.rc.n_exc <= kExcLocal ? (int)xi : (int)c.rc.exc_pos[i];
    const int a = p - (mm - 1) < 0 ? 0 : p - (mm - 1);
    const int b = p + (mm - 1) > n - 1 ? n - 1 : p + (mm - 1);
    int w0 = a / L, w1 = b / L;
    if (w1 > nw - 2) w1 = nw - 2;
    if (w0 < next) w0 = next;
    for (int w = w0; w <= w1; ++w) {
      if (cnt == cap) return cap + 1;
      ++cnt;
      f(w);
    }
    if (w1 + 1 > next) next = w1 + 1;
  }
  return cnt;
}

// The last window of a read scanned by the bundle scan (nt_tscan.h): that scan
// does not mask the read ends, so the window holding them -- whose width may
// differ from L, and into which split_telo may have merged a short last block
// (NanoTel.R:199-227) -- is recounted here from the read's own planes (exact
// out-of-bound rule at the end), and its window count, the checkpoint at
// window nw (the read's total, when nw is a multiple of 16) and its bit of the
// telomeric bitmask (threshold of its own width) are rewritten.  Idempotent
// for reads of the per-read scan.
//
// A read with non-ACGT letters scanned in a bundle (nt_common.h, exc_windows)
// has the windows near its exceptions recounted the same way first, each
// checkpoint after them moved by the difference.  A read whose exceptions
// reach more than NT_EXC_WINDOWS windows was left on the per-read scan: its
// counts are exact and only its last window is recounted.  One coverage site
// for all of them (the windows in a rolled loop).
static __device__ __forceinline__ void call_fix_windows(Lane& c, const uint32_t* __restrict__ thr, uint32_t thr_size) {
  if (c.nw <= 0) return;
  int ne = 0;
  if (c.rc.n_exc) {
    ne = lane_exc_windows(c, NT_EXC_WINDOWS, [](int) {});
    if (ne > NT_EXC_WINDOWS) ne = 0;
  }
  for (int k = 0; k <= ne; ++k) {
    int w = c.nw - 1;  // the last window after the exception windows
    if (k < ne) {
      int i = 0;
      lane_exc_windows(c, k + 1, [&](int x) {
        if (i++ == k) w = x;
      });
    }
    const int a = w * c.L, b = w == c.nw - 1 ? c.n - 1 : a + c.L - 1;
    const int exact = cov_count(c, a, b);
    const int old = wcount(c, w);
    if (exact != old) {
      if (c.c8) static_cast<uint8_t*>(const_cast<void*>(c.cnt))[w] = (uint8_t)exact;
      else static_cast<uint16_t*>(const_cast<void*>(c.cnt))[w] = (uint16_t)exact;
      // the checkpoints after window w (covered bases before window 16 j)
      for (int j = (w >> 4) + 1; j <= (c.nw >> 4); ++j) const_cast<uint32_t*>(c.ck)[j] += (uint32_t)(exact - old);
    }
    const uint32_t wd = (uint32_t)(b - a + 1);
    const bool tel = (uint32_t)exact >= thr[wd < thr_size ? wd : thr_size - 1];
    uint64_t* tw = const_cast<uint64_t*>(c.tm) + (w >> 6);
    const uint64_t m = 1ull << (w & 63), x = *tw;
    const uint64_t y = tel ? (x | m) : (x & ~m);
    if (y != x) *tw = y;
  }
}

// find_telo_position_wraper (NanoTel.R:1080-1155) + density (NanoTel.R:1840).
static __device__ __forceinline__ void call_pass(Lane& c, int& out_s, int& out_e, double& out_d, uint32_t& err) {
  tm_preload(c);
  Pos tp = find_telo_position(c, 3, 2.0);
  // get_accurate_* neighbourhoods fetched with the wrapper's density loads
  // (one memory round trip less); refetched if the wrapper re-runs the call
  NbB5 fs, fe;
  if (NT_CALL_ACC_EARLY) accurate_fetch(c, tp.s, tp.e, fs, fe);
  const double telo_density = sub_density(c, tp.s, tp.e);
  const int num_rows = (tp.e - tp.s + 1) / c.L;
  bool refetch = !NT_CALL_ACC_EARLY;
  if (telo_density < 0.85 && num_rows > 5) {
    const int min_rows = num_rows <= 7 ? num_rows - 2 : 7;
    const double min_density = 0.6 * (double)min_rows;
    tp = find_telo_position(c, min_rows, min_density);
    refetch = true;
  }
  if (refetch) accurate_fetch(c, tp.s, tp.e, fs, fe);
  int s_acc, e_acc;
  accurate_both(c, tp.s, tp.e, fs, fe, s_acc, e_acc);
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
  out_d = sub_density(c, tp.s, tp.e);
}

// The lane of read r, pass p.
static __device__ __forceinline__ void init_lane(Lane& c, const NtProgram* __restrict__ prog, const NtBatch& B,
                                                 const NtOut& O, const uint64_t* __restrict__ tmask, uint64_t r,
                                                 int p, uint64_t* tm_lds, uint32_t* pw_lds) {
  const int np = prog->n_pass, L = prog->L;
  const uint32_t n32 = B.len[r];
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
    if (e1 > e0) {
      c.exc_lo = B.exc_pos[e0];
      c.exc_hi = B.exc_pos[e1 - 1];
      c.xcode = 0u;
#pragma unroll
      for (int k = 0; k < kExcLocal; ++k) {
        const bool ok = e0 + (uint32_t)k < e1;
        c.xpos[k] = ok ? B.exc_pos[e0 + k] : 0xFFFFFFFFu;
        c.xcode |= (ok ? (uint32_t)B.exc_code[e0 + k] : 0u) << (8 * k);
      }
    }
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
}

// A bundled read the bundle scan did not scan: its bundle's planes span more
// than 2 GiB (nt_tscan.h kTsSpanError in its first checkpoint, which is
// otherwise 0).  Reported as a layout-contract error, as an odd blk_off is.
static __device__ __forceinline__ bool bundle_span_error(const NtProgram* __restrict__ prog, const NtBatch& B,
                                                         const uint64_t* __restrict__ tmask, uint64_t r) {
  const int np = prog->n_pass;
  const int nw = (int)split_window_count((int)B.len[r], prog->L);
  if (nw == 0) return false;  // nothing to call from the scan's outputs (its ck[0] is written anyway)
  const uint32_t* ck = reinterpret_cast<const uint32_t*>(tmask + aux_base(B.win_off[r], r, np) + (uint64_t)np * aux_nmw(nw));
  return ck[0] == 0xFFFFFFFFu;
}

// The per-pass split (kPass >= 0): a lane per read, this pass's start / end /
// density; an error is left in end (-2: find_right_telo on a 0-row table, -3:
// a negative width) and the flags are made by nt_call_combine_kernel after
// every pass's launch.  Reads the scan skipped (odd blk_off) are left to it.
static __device__ __forceinline__ void run_pass(const NtProgram* __restrict__ prog, NtBatch B, NtOut O,
                                                const uint64_t* __restrict__ tmask, const uint32_t* __restrict__ thr,
                                                uint32_t thr_size, int fix_last, uint64_t* tm_lds, uint32_t* pw_lds) {
  static_assert(kPass >= 0 && kPass < 3, "run_pass: one pass");
  const uint64_t total = B.list ? B.n_list : B.n_reads;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total; idx += stride) {
    const uint64_t r = B.list ? (uint64_t)B.list[idx] : idx;
    if (r == 0xFFFFFFFFull || (B.blk_off[r] & 1u)) continue;
    if (fix_last && bundle_span_error(prog, B, tmask, r)) {  // left to nt_call_combine_kernel (end -4)
      O.start[r * 3 + kPass] = -1;
      O.end[r * 3 + kPass] = -4;
      O.density[r * 3 + kPass] = 0.0;
      continue;
    }
    Lane c;
    init_lane(c, prog, B, O, tmask, r, kPass, tm_lds, pw_lds);
    if (fix_last) call_fix_windows(c, thr, thr_size);
    int s = -1, e = -1;
    double d = 0.0;
    uint32_t flags = 0u;
    call_pass(c, s, e, d, flags);
    if (flags & NT_FLAG_ERR_RIGHT) e = -2;
    else if (flags & NT_FLAG_ERR_WIDTH) e = -3;
    O.start[r * 3 + kPass] = s;
    O.end[r * 3 + kPass] = e;
    O.density[r * 3 + kPass] = d;
  }
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
static __device__ __forceinline__ void run(const NtProgram* __restrict__ prog, NtBatch B, NtOut O,
                                           const uint64_t* __restrict__ tmask, const uint32_t* __restrict__ thr,
                                           uint32_t thr_size, int fix_last, uint64_t* tm_lds, uint32_t* pw_lds) {
  const int np = prog->n_pass;
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
    int w = kIntMin;
    bool align = false;
    if (in) {
      align = (B.blk_off[r] & 1u) != 0;  // the scan skipped this read (layout contract)
      if (!align && fix_last) align = bundle_span_error(prog, B, tmask, r);
      if (!align && p < np) {
        Lane c;
        init_lane(c, prog, B, O, tmask, r, p, tm_lds, pw_lds);
        if (fix_last) call_fix_windows(c, thr, thr_size);
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
};  // struct Call


}  // namespace nt

// NT_CALL_WAVES_PER_EU trades VGPRs for occupancy (see Call::run).
#ifndef NT_CALL_WAVES_PER_EU
#define NT_CALL_WAVES_PER_EU 3
#endif
#define NT_CALL_ATTR __attribute__((amdgpu_waves_per_eu(NT_CALL_WAVES_PER_EU)))
#if NT_CALL_TM_LDS
#define NT_CALL_TM_DECL __shared__ uint64_t tm_lds[nt::kTmRegs * 256];
#define NT_CALL_TM_ARG tm_lds
#else
#define NT_CALL_TM_DECL
#define NT_CALL_TM_ARG nullptr
#endif
#if NT_CALL_PW_LDS
#define NT_CALL_PW_DECL __shared__ uint32_t pw_lds[20 * 256];
#define NT_CALL_PW_ARG pw_lds
#else
#define NT_CALL_PW_DECL
#define NT_CALL_PW_ARG nullptr
#endif
// The calling kernel NAME for pattern-set policy CS (256 threads a block);
// NT_CALL_KERNEL_PASS: the pass-P kernel of the per-pass split.
#define NT_CALL_KERNEL(NAME, CS)                                                                             \
  extern "C" __global__ void __launch_bounds__(256) NT_CALL_ATTR                                             \
  NAME(const NtProgram* __restrict__ prog, NtBatch B, NtOut O, const uint64_t* __restrict__ tmask,           \
       const uint32_t* __restrict__ thr, uint32_t thr_size, int fix_last) {                                  \
    NT_CALL_TM_DECL                                                                                          \
    NT_CALL_PW_DECL                                                                                          \
    nt::Call<CS>::run(prog, B, O, tmask, thr, thr_size, fix_last, NT_CALL_TM_ARG, NT_CALL_PW_ARG);          \
  }
#define NT_CALL_KERNEL_PASS(NAME, CS, P)                                                                     \
  extern "C" __global__ void __launch_bounds__(256) NT_CALL_ATTR                                             \
  NAME(const NtProgram* __restrict__ prog, NtBatch B, NtOut O, const uint64_t* __restrict__ tmask,           \
       const uint32_t* __restrict__ thr, uint32_t thr_size, int fix_last) {                                  \
    NT_CALL_TM_DECL                                                                                          \
    NT_CALL_PW_DECL                                                                                          \
    nt::Call<CS, P>::run_pass(prog, B, O, tmask, thr, thr_size, fix_last, NT_CALL_TM_ARG, NT_CALL_PW_ARG);  \
  }
