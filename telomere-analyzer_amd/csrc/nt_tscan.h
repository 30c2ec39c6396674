// nt_tscan.h -- the bundle scan of the NanoTel hot path on gfx950.
//
// The same outputs as scan_reads (nt_scan.h): per read and pass the covered
// bases of every subseq_length window (analyze_subtelos / get_density_iranges
// / get_sub_density, NanoTel.R:717-766, 308-397, 449-468), the telomeric-window
// bitmask (class -5, NanoTel.R:749-758) and the running-count checkpoints the
// calling kernel sums with.  Reads are grouped 32 to a BUNDLE (nt_bundle_plan)
// and scanned from their own 2-bit planes -- the one copy of the reads in HBM
// -- transposed on the fly in registers, so that every word of the walk holds
// ONE position of all 32 reads (bit s = slot s).  A shift by one position is
// then a register rename, and the whole walk -- the letter tests of
// matchPattern, the 3-letter majority combine (<= 1 mismatch, Biostrings'
// out-of-bound rule), the coverage spread (trim + IRanges::reduce) and the
// per-window counts (bit-sliced carry-save adders) -- is plain 3-input bit
// logic, which gfx950 issues at full rate (v_bitop3 / v_and / v_or / v_xor),
// where the per-read layout spends its instructions on funnel shifts, DPP
// neighbour moves and popcounts (tools/valu_issue_bench.hip).
//
// Work split.  A wave claims a bundle from the per-XCD queues and walks its
// HALF STRIPES (32 windows of every read) in turn.  The half stripe's plane
// words of the 32 reads are loaded straight into a per-wave LDS buffer (one
// 16-byte buffer load per read and lane); lane (l, h) walks half h of window
// 32 hs + l -- L0 = ceil(L / 2) positions plus kLam of halo on each side
// (kLam = longest pattern - 1: the left halo feeds the coverage of the half's
// first bases, the right halo the letter tests of its last starts) -- in
// RANGES of 32 positions: the 32-position piece of every read at the lane's
// bit offset (ds_read_b64 of two plane words, v_alignbit) and two 32 x 32 bit
// transposes in the lane's own registers (v_perm for the byte stages, shift +
// v_bfi for the bit stages) give the 32 position words of the range, walked
// fully unrolled (L and the patterns are baked into the hiprtc build) into 8
// bit planes of counts per pass (acc[b] bit s = bit b of read s's count;
// counts <= L <= 170).  The halves' counts are added across the wave's halves
// (v_permlane32_swap); two half stripes make one output stripe of 64 windows.
//
// Output, lane = window, per stripe and pass: the telomeric bits (count >=
// thr[L]) by a bit-sliced compare and a 32 x 32 bit transpose inside each
// half wave; the counts (uint8: L <= 170) by an 8 x 8 bit transpose within
// every byte, a 4 x 4 byte transpose inside every quad of lanes and an LDS
// row per read, stored from LDS as whole 128-byte lines every second stripe
// (non-temporal); the checkpoints every 16 windows from v_dot4 sums of the
// same rows.  Bitmask words and checkpoints wait in LDS and go out as runs of
// a read's row (TsAux).  The read ends are not masked (a lane reads on past a
// short read, into the planes that follow it), so the LAST window of every
// read -- whose width may differ from L, and into which split_telo may have
// merged a short last block (NanoTel.R:220) -- is recounted exactly by the
// calling kernel from the per-read planes (call_fix_windows, nt_call.h).
#pragma once
#include "nt_scan.h"

namespace nt {

// 3-input logic as v_bitop3 (full rate; hipcc picks the half-rate v_or3_b32
// for a | b | c)
__device__ __forceinline__ uint32_t or3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xFE);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t and3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
}
__device__ __forceinline__ uint32_t mj3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// ----------------------------------------------------- compile-time lists

constexpr int cmax() { return 0; }
template <class... T>
constexpr int cmax(int a, T... r) {
  return a > cmax(r...) ? a : cmax(r...);
}
constexpr int cmin() { return 1 << 30; }
template <class... T>
constexpr int cmin(int a, T... r) {
  return a < cmin(r...) ? a : cmin(r...);
}

template <class List>
struct LInfo;
template <class... P>
struct LInfo<CtList<P...>> {
  static constexpr int kN = sizeof...(P);
  static constexpr int kMax = cmax(P::kM...);
  static constexpr int kMin = cmin(P::kM...);
};
template <class List, int I>
struct LAt;
template <int I, class... P>
struct LAt<CtList<P...>, I> {
  using type = typename CtAt<I, P...>::type;
};

// Exact (a0) and <= 1 mismatch (a1) of one start from its kM letter words:
// letters in groups of three, each group (all three, at least two) by one
// v_bitop3 apiece, the groups chained with x1 = two & x1 & (all | x0) (= the
// (x1 & all) | (x0 & two) of combine(), as x0 <= x1 and all <= two).
template <int kM, bool kExact>
__device__ __forceinline__ void tcombine(const uint32_t* q, uint32_t& a0, uint32_t& a1) {
  if constexpr (kExact) {
    uint32_t x = q[0];
    int j = 1;
    for (; j + 2 <= kM; j += 2) x = and3(x, q[j], q[j + 1]);
    if (j < kM) x &= q[j];
    a0 = x;
    a1 = 0u;
  } else {
    uint32_t x0 = 0u, x1 = 0u;
#pragma unroll
    for (int g = 0; g < kM; g += 3) {
      const int n = kM - g < 3 ? kM - g : 3;
      uint32_t all, two;
      if (n == 3) {
        all = and3(q[g], q[g + 1], q[g + 2]);
        two = mj3(q[g], q[g + 1], q[g + 2]);
      } else if (n == 2) {
        all = q[g] & q[g + 1];
        two = q[g] | q[g + 1];
      } else {
        all = q[g];
        two = 0xFFFFFFFFu;
      }
      if (g == 0) {
        x0 = all;
        x1 = two;
      } else {
        x1 = (n == 1) ? (x1 & (all | x0)) : and3(two, x1, all | x0);
        x0 &= all;
      }
    }
    a0 = x0;
    a1 = x1;
  }
}

// ------------------------------------------------------ the bundle program

// Pats / Tvrs: CtList<CtPat<m, tt...>...> (every pattern of a list the same
// length: the host routes other programs to scan_reads); kL: subseq_length.
template <class Pats, class Tvrs, int kL_>
struct TProg {
  static constexpr int kL = kL_;
  static constexpr int kNPat = LInfo<Pats>::kN, kNTvr = LInfo<Tvrs>::kN;
  static constexpr int kMP = LInfo<Pats>::kMax, kMT = kNTvr ? LInfo<Tvrs>::kMax : 0;
  static constexpr int kNP = kNTvr ? 3 : 2;
  static constexpr int kM = kMP > kMT ? kMP : kMT;
  static constexpr int kH = kM - 1;               // halo on each side
  static constexpr int kLam = kH;                 // counting lag = the halo (a walk: 2 kLam prologue steps)
};

// Widths of the sliding-OR stages of the coverage spread for pattern length
// m: w_0 = 1, each stage at most triples the width (one v_bitop3 per position
// and stage; TTAGGG: 1 -> 3 -> 6).
template <int kM>
struct Spread {
  static constexpr int width(int s) {
    int w = 1;
    for (int t = 0; t < s; ++t) w = 3 * w <= kM ? 3 * w : kM;
    return w;
  }
  static constexpr int stages() {
    int s = 0;
    while (width(s) < kM) ++s;
    return s;
  }
  static constexpr int kS = stages();
};

// Bit-sliced counter of 1-bit words (one per position; bit s = slot s):
// acc[b] bit s = bit b of slot s's count.  Levels 0..3 add their words in
// carry-save pairs with the level's accumulator (xor3 / majority: one
// v_bitop3 each), the pair's carry is a word of the next level; level 4 and
// up add by ripple (one word per 16 positions).  Push indices are per run.
struct BitCount {
  uint32_t acc[8];
  uint32_t pend[4];
  // keep the counters computed where they are: the scheduler otherwise sinks
  // the count chains of a whole walk to its end (their only use) and spills
  // everything they read
  __device__ __forceinline__ void pin() {
#pragma unroll
    for (int l = 0; l < 8; ++l) asm volatile("" : "+v"(acc[l]));
  }
  template <int Lvl>
  __device__ __forceinline__ void ripple(uint32_t x) {
#pragma unroll
    for (int l = Lvl; l < 8; ++l) {
      const uint32_t c = acc[l] & x;
      acc[l] ^= x;
      x = c;
    }
  }
  template <int Lvl, int Idx>
  __device__ __forceinline__ void push(uint32_t x) {
    if constexpr (Lvl >= 4) {
      ripple<Lvl>(x);
    } else if constexpr (Idx % 2 == 0) {
      pend[Lvl] = x;
    } else {
      const uint32_t a = pend[Lvl], c = acc[Lvl];
      acc[Lvl] = xor3(a, x, c);
      push<Lvl + 1, Idx / 2>(mj3(a, x, c));
    }
  }
  // the run pushed Cnt words at level Lvl: fold a pending one upward
  template <int Lvl, int Cnt>
  __device__ __forceinline__ void flush() {
    if constexpr (Lvl < 4) {
      if constexpr (Cnt % 2 == 1) {
        const uint32_t p = pend[Lvl];
        const uint32_t c = acc[Lvl] & p;
        acc[Lvl] ^= p;
        push<Lvl + 1, Cnt / 2>(c);
        flush<Lvl + 1, Cnt / 2 + 1>();
      } else {
        flush<Lvl + 1, Cnt / 2>();
      }
    }
  }
};

// The letter truth tables a program tests (bit tt of the mask: some letter of
// some pattern or TVR has truth table tt); each is one word per position.
template <class List>
struct LTests;
template <class... P>
struct LTests<CtList<P...>> {
  template <class D>
  static constexpr uint32_t one() {
    uint32_t m = 0;
    for (int j = 0; j < D::kM; ++j) m |= 1u << (D::kTT[j] & 15);
    return m;
  }
  static constexpr uint32_t kMask = (0u | ... | one<P>());
};

// Exact matches of a list of TVRs of one length (NanoTel.R:360-393: P3 adds
// the TVRs' exact matches) with the letters every TVR shares factored out:
// hit = AND(shared letters) & OR_t AND(t's other letters).  TGAGGG + TTGGGG
// share T....GGG: 4 bitwise ops a position instead of 7 (two and-chains of
// six letters and an OR).  Pure bitwise: the same hits as OR_t AND_j.
template <class List>
struct TvrShared;
template <class... P>
struct TvrShared<CtList<P...>> {
  template <class D>
  static constexpr int tt(int j) { return D::kTT[j] & 15; }
  // bit j: every TVR has the same truth table at letter j
  static constexpr uint64_t mask() {
    using D0 = typename CtAt<0, P...>::type;
    uint64_t m = 0;
    for (int j = 0; j < D0::kM; ++j)  // (a fold, not a braced list: hiprtc has no <initializer_list>)
      if (((tt<P>(j) == tt<D0>(j)) && ...)) m |= 1ull << j;
    return m;
  }
  static constexpr uint64_t kMask = mask();
};

// AND of n words, three at a time (v_bitop3 and3), times an extra word x
template <int N>
__device__ __forceinline__ uint32_t and_all(const uint32_t (&q)[N], int n, uint32_t x) {
  uint32_t r = x;
  int j = 0;
  for (; j + 2 <= n; j += 2) r = and3(r, q[j], q[j + 1]);
  if (j < n) r &= q[j];
  return r;
}

// The per-lane pipeline of the walk: position by position, the letter tests
// (one word per distinct truth table), the hits of the starts whose last
// letter is the position (exact, <= 1 mismatch; TVRs exact), the sliding-OR
// stages of the coverage spread and the count of the position kH back, whose
// every covering start is then known.  Runs of N positions are unrolled; the
// last HD values of every per-position array carry over to the next run
// (entries no later step reads are dead).  The history holds TEST words, so
// the out-of-bound mask of the first block exists in the prologue only.
template <class TP, class Pats, class Tvrs>
struct TPipe {
  static constexpr int kM = TP::kM, kMP = TP::kMP, kMT = TP::kMT > 0 ? TP::kMT : 1;
  static constexpr int kNTvr = TP::kNTvr, kNPat = TP::kNPat;
  static constexpr int HD = 2 * kM;
  static constexpr uint32_t kTests = LTests<Pats>::kMask | LTests<Tvrs>::kMask;
  using SP = Spread<kMP>;
  using ST = Spread<kMT>;
  static constexpr int kSP = SP::kS, kST = ST::kS;
  uint32_t hT[16][HD];
  uint32_t h0[kSP + 1][HD], h1[kSP + 1][HD], ht[kST + 1][HD];
  BitCount bc[3];

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int t = 0; t < HD; ++t) {
#pragma unroll
      for (int c = 0; c < 16; ++c) hT[c][t] = 0u;
#pragma unroll
      for (int s = 0; s <= kSP; ++s) h0[s][t] = h1[s][t] = 0u;
#pragma unroll
      for (int s = 0; s <= kST; ++s) ht[s][t] = 0u;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int b = 0; b < 8; ++b) bc[p].acc[b] = 0u;
  }

  // sliding-OR stage s at index x of a stage array (earlier entries are final)
  template <class Sp, int s, int X, int NN>
  __device__ __forceinline__ static uint32_t stage(const uint32_t (&w)[NN]) {
    constexpr int a = Sp::width(s - 1), b = Sp::width(s);
    if constexpr (3 * a <= b) return or3(w[X], w[X - a], w[X - 2 * a]);
    else if constexpr (2 * a >= b) return w[X] | w[X - (b - a)];
    else return or3(w[X], w[X - a], w[X - (b - a)]);
  }

  // one run of N positions; kCount: count position P - kH of every step
  // (a run of 16 completes its carry-save pairs); kVarV: Vr masks positions
  // get(ui) -> uint3 {lo, hi, valid mask} of position u, read at step u (after
  // the hooks of the earlier steps: the ring slot may have been refilled)
  template <int N, bool kCount, bool kVarV, int kMaskStep = -1, class Get, class Hook>
  __device__ __forceinline__ void run(Get&& get, Hook&& hook) {
    constexpr int NN = HD + N;
    uint32_t Ts[16][NN];
    uint32_t a0[kSP + 1][NN], a1[kSP + 1][NN], at[kST + 1][NN];
#pragma unroll
    for (int t = 0; t < HD; ++t) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if ((kTests >> c) & 1u) Ts[c][t] = hT[c][t];
#pragma unroll
      for (int s = 0; s <= kSP; ++s) {
        a0[s][t] = h0[s][t];
        a1[s][t] = h1[s][t];
      }
#pragma unroll
      for (int s = 0; s <= kST; ++s) at[s][t] = ht[s][t];
    }
    static_for<0, N>([&](auto ui) {
      constexpr int u = decltype(ui)::value, x = HD + u;
      const uint3 pl = get(ui);
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if ((kTests >> c) & 1u) Ts[c][x] = kVarV ? (tt_test(c, pl.x, pl.y) & pl.z) : tt_test(c, pl.x, pl.y);
      hook(ui);  // the planes of position u are dead: e.g. refill its ring slot
      {  // patterns: the start x - (kMP - 1)
        constexpr int j0 = x - (kMP - 1);
        uint32_t e0 = 0u, e1 = 0u;
        static_for<0, kNPat>([&](auto pi) {
          using D = typename LAt<Pats, decltype(pi)::value>::type;
          uint32_t q[kMP];
#pragma unroll
          for (int j = 0; j < kMP; ++j) q[j] = Ts[D::kTT[j] & 15][j0 + j];
          uint32_t b0, b1;
          tcombine<kMP, false>(q, b0, b1);
          e0 |= b0;
          e1 |= b1;
        });
        a0[0][x] = e0;
        a1[0][x] = e1;
        static_for<1, kSP + 1>([&](auto si) {
          constexpr int s = decltype(si)::value;
          a0[s][x] = stage<SP, s, x>(a0[s - 1]);
          a1[s][x] = stage<SP, s, x>(a1[s - 1]);
        });
      }
      if constexpr (kNTvr > 0) {  // TVRs (exact): the start x - (kMT - 1)
        constexpr int j0 = x - (kMT - 1);
        constexpr uint64_t sh = TvrShared<Tvrs>::kMask;  // letters every TVR shares
        uint32_t e = 0u;
        static_for<0, kNTvr>([&](auto ti) {
          using D = typename LAt<Tvrs, decltype(ti)::value>::type;
          uint32_t q[kMT];
          int nq = 0;
#pragma unroll
          for (int j = 0; j < kMT; ++j)
            if (!((sh >> j) & 1u)) q[nq++] = Ts[D::kTT[j] & 15][j0 + j];
          if (nq == 0) {
            e = 0xFFFFFFFFu;  // (a TVR made of shared letters only: the shared AND is its hit)
          } else {
            uint32_t r = q[0];
            int j = 1;
            for (; j + 2 <= nq; j += 2) r = and3(r, q[j], q[j + 1]);
            if (j < nq) e = __builtin_amdgcn_bitop3_b32(r, q[j], e, 0xEA);  // (r & q) | e
            else e |= r;
          }
        });
        {
          using D0 = typename LAt<Tvrs, 0>::type;
          uint32_t q[kMT];
          int nq = 0;
#pragma unroll
          for (int j = 0; j < kMT; ++j)
            if ((sh >> j) & 1u) q[nq++] = Ts[D0::kTT[j] & 15][j0 + j];
          e = and_all(q, nq, e);
        }
        at[0][x] = e;
        static_for<1, kST + 1>([&](auto si) {
          constexpr int s = decltype(si)::value;
          at[s][x] = stage<ST, s, x>(at[s - 1]);
        });
      }
      if constexpr (kCount) {  // the coverage of position P - kLam
        constexpr int kLam = TP::kLam;
        constexpr int y0 = x - (kLam + 1 - kMP);
        // kMaskStep: this step's count ANDed with pl.z (a walk whose last
        // counted position may lie past its window)
        const uint32_t cm = u == kMaskStep ? pl.z : 0xFFFFFFFFu;
        const uint32_t c1 = a1[kSP][y0] & cm;
        bc[0].template push<0, u>(a0[kSP][y0] & cm);
        bc[1].template push<0, u>(c1);
        if constexpr (kNTvr > 0) {
          constexpr int yt = x - (kLam + 1 - kMT);
          bc[2].template push<0, u>(c1 | (at[kST][yt] & cm));
        }
      }
    });
    if constexpr (kCount) {
      bc[0].template flush<0, N>();
      bc[1].template flush<0, N>();
      if constexpr (kNTvr > 0) bc[2].template flush<0, N>();
    }
#pragma unroll
    for (int t = 0; t < HD; ++t) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if ((kTests >> c) & 1u) hT[c][t] = Ts[c][N + t];
#pragma unroll
      for (int s = 0; s <= kSP; ++s) {
        h0[s][t] = a0[s][N + t];
        h1[s][t] = a1[s][N + t];
      }
#pragma unroll
      for (int s = 0; s <= kST; ++s) ht[s][t] = at[s][N + t];
    }
  }
};

// Distinct pattern lengths of a list (ascending): mixed-length lists (e.g.
// "TTAGGG TTAGG"; the reference takes any list, NanoTel.R:2322-2334, 360-393)
// run one group of patterns per length.
constexpr int kTsMaxGroups = 4;
template <class List>
struct LLens;
template <class... P>
struct LLens<CtList<P...>> {
  static constexpr bool has(int m) { return ((P::kM == m) || ... || false); }
  static constexpr int count() {
    int c = 0;
    for (int m = 1; m <= 64; ++m) c += has(m) ? 1 : 0;
    return c;
  }
  static constexpr int kN = count();
  static constexpr int at(int i) {  // the i-th distinct length
    for (int m = 1; m <= 64; ++m)
      if (has(m) && i-- == 0) return m;
    return 1;
  }
};

// The walk pipeline of a program whose patterns (or TVRs) differ in length:
// TPipe's steps, one group per distinct length m -- the hits of the starts
// x - (m - 1) whose last letter is the position x, that group's sliding-OR
// spread (width m), and the coverage of the counted position x - kLam as the
// OR over the groups of spread_g[x - kLam + m_g - 1] (kLam >= every m_g - 1).
// Single-length programs keep TPipe (same code as before).
template <class TP, class Pats, class Tvrs>
struct TPipeMixed {
  static constexpr int kM = TP::kM;
  static constexpr int kNTvr = TP::kNTvr, kNPat = TP::kNPat;
  static constexpr int HD = 2 * kM;
  static constexpr uint32_t kTests = LTests<Pats>::kMask | LTests<Tvrs>::kMask;
  using LP = LLens<Pats>;
  static constexpr int GP = LP::kN;
  static constexpr int GT = kNTvr > 0 ? LLens<Tvrs>::kN : 1;
  static_assert(GP <= kTsMaxGroups && GT <= kTsMaxGroups, "pattern lengths per list (nt_tscan_eligible)");
  template <int g>
  static constexpr int mp() { return LP::at(g); }
  template <int g>
  static constexpr int mt() {
    if constexpr (kNTvr > 0) return LLens<Tvrs>::at(g);
    else return 1;
  }
  static constexpr int smax() {
    int s = 0;
    for (int g = 0; g < GP; ++g) {
      int w = 1, k = 0, m = LP::at(g);
      while (w < m) { w = 3 * w <= m ? 3 * w : m; ++k; }
      s = k > s ? k : s;
    }
    if (kNTvr > 0)
      for (int g = 0; g < GT; ++g) {
        int w = 1, k = 0, m = LLens<Tvrs>::at(g);
        while (w < m) { w = 3 * w <= m ? 3 * w : m; ++k; }
        s = k > s ? k : s;
      }
    return s;
  }
  static constexpr int kS = smax();
  uint32_t hT[16][HD];
  uint32_t h0[GP][kS + 1][HD], h1[GP][kS + 1][HD], ht[GT][kS + 1][HD];
  BitCount bc[3];

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int t = 0; t < HD; ++t) {
#pragma unroll
      for (int c = 0; c < 16; ++c) hT[c][t] = 0u;
#pragma unroll
      for (int s = 0; s <= kS; ++s) {
#pragma unroll
        for (int g = 0; g < GP; ++g) h0[g][s][t] = h1[g][s][t] = 0u;
#pragma unroll
        for (int g = 0; g < GT; ++g) ht[g][s][t] = 0u;
      }
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int b = 0; b < 8; ++b) bc[p].acc[b] = 0u;
  }

  template <class Sp, int s, int X, int NN>
  __device__ __forceinline__ static uint32_t stage(const uint32_t (&w)[NN]) {
    constexpr int a = Sp::width(s - 1), b = Sp::width(s);
    if constexpr (3 * a <= b) return or3(w[X], w[X - a], w[X - 2 * a]);
    else if constexpr (2 * a >= b) return w[X] | w[X - (b - a)];
    else return or3(w[X], w[X - a], w[X - (b - a)]);
  }

  template <int N, bool kCount, bool kVarV, int kMaskStep = -1, class Get, class Hook>
  __device__ __forceinline__ void run(Get&& get, Hook&& hook) {
    constexpr int NN = HD + N;
    uint32_t Ts[16][NN];
    uint32_t a0[GP][kS + 1][NN], a1[GP][kS + 1][NN], at[GT][kS + 1][NN];
#pragma unroll
    for (int t = 0; t < HD; ++t) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if ((kTests >> c) & 1u) Ts[c][t] = hT[c][t];
#pragma unroll
      for (int s = 0; s <= kS; ++s) {
#pragma unroll
        for (int g = 0; g < GP; ++g) {
          a0[g][s][t] = h0[g][s][t];
          a1[g][s][t] = h1[g][s][t];
        }
#pragma unroll
        for (int g = 0; g < GT; ++g) at[g][s][t] = ht[g][s][t];
      }
    }
    static_for<0, N>([&](auto ui) {
      constexpr int u = decltype(ui)::value, x = HD + u;
      const uint3 pl = get(ui);
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if ((kTests >> c) & 1u) Ts[c][x] = kVarV ? (tt_test(c, pl.x, pl.y) & pl.z) : tt_test(c, pl.x, pl.y);
      hook(ui);
      static_for<0, GP>([&](auto gi) {  // patterns of length m: the start x - (m - 1)
        constexpr int g = decltype(gi)::value, m = mp<g>();
        constexpr int j0 = x - (m - 1);
        uint32_t e0 = 0u, e1 = 0u;
        static_for<0, kNPat>([&](auto pi) {
          using D = typename LAt<Pats, decltype(pi)::value>::type;
          if constexpr (D::kM == m) {
            uint32_t q[m];
#pragma unroll
            for (int j = 0; j < m; ++j) q[j] = Ts[D::kTT[j] & 15][j0 + j];
            uint32_t b0, b1;
            tcombine<m, false>(q, b0, b1);
            e0 |= b0;
            e1 |= b1;
          }
        });
        a0[g][0][x] = e0;
        a1[g][0][x] = e1;
        static_for<1, Spread<m>::kS + 1>([&](auto si) {
          constexpr int s = decltype(si)::value;
          a0[g][s][x] = stage<Spread<m>, s, x>(a0[g][s - 1]);
          a1[g][s][x] = stage<Spread<m>, s, x>(a1[g][s - 1]);
        });
      });
      if constexpr (kNTvr > 0) {
        static_for<0, GT>([&](auto gi) {  // TVRs (exact)
          constexpr int g = decltype(gi)::value, m = mt<g>();
          constexpr int j0 = x - (m - 1);
          uint32_t e = 0u;
          static_for<0, kNTvr>([&](auto ti) {
            using D = typename LAt<Tvrs, decltype(ti)::value>::type;
            if constexpr (D::kM == m) {
              uint32_t q[m];
#pragma unroll
              for (int j = 0; j < m; ++j) q[j] = Ts[D::kTT[j] & 15][j0 + j];
              uint32_t b0, b1;
              tcombine<m, true>(q, b0, b1);
              e |= b0;
            }
          });
          at[g][0][x] = e;
          static_for<1, Spread<m>::kS + 1>([&](auto si) {
            constexpr int s = decltype(si)::value;
            at[g][s][x] = stage<Spread<m>, s, x>(at[g][s - 1]);
          });
        });
      }
      if constexpr (kCount) {  // the coverage of position x - kLam: OR over the groups
        constexpr int kLam = TP::kLam;
        uint32_t c0 = 0u, c1 = 0u, ct = 0u;
        static_for<0, GP>([&](auto gi) {
          constexpr int g = decltype(gi)::value, m = mp<g>();
          constexpr int y = x - (kLam + 1 - m);
          c0 |= a0[g][Spread<m>::kS][y];
          c1 |= a1[g][Spread<m>::kS][y];
        });
        const uint32_t cm = u == kMaskStep ? pl.z : 0xFFFFFFFFu;  // see TPipe
        bc[0].template push<0, u>(c0 & cm);
        bc[1].template push<0, u>(c1 & cm);
        if constexpr (kNTvr > 0) {
          static_for<0, GT>([&](auto gi) {
            constexpr int g = decltype(gi)::value, m = mt<g>();
            constexpr int y = x - (kLam + 1 - m);
            ct |= at[g][Spread<m>::kS][y];
          });
          bc[2].template push<0, u>((c1 | ct) & cm);
        }
      }
    });
    if constexpr (kCount) {
      bc[0].template flush<0, N>();
      bc[1].template flush<0, N>();
      if constexpr (kNTvr > 0) bc[2].template flush<0, N>();
    }
#pragma unroll
    for (int t = 0; t < HD; ++t) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if ((kTests >> c) & 1u) hT[c][t] = Ts[c][N + t];
#pragma unroll
      for (int s = 0; s <= kS; ++s) {
#pragma unroll
        for (int g = 0; g < GP; ++g) {
          h0[g][s][t] = a0[g][s][N + t];
          h1[g][s][t] = a1[g][s][N + t];
        }
#pragma unroll
        for (int g = 0; g < GT; ++g) ht[g][s][t] = at[g][s][N + t];
      }
    }
  }
};

// TPipe for single-length lists, TPipeMixed otherwise
template <class TP, class Pats, class Tvrs, bool kMixed = (LLens<Pats>::kN > 1) || (LLens<Tvrs>::kN > 1)>
struct TPipeSel {
  using type = TPipe<TP, Pats, Tvrs>;
};
template <class TP, class Pats, class Tvrs>
struct TPipeSel<TP, Pats, Tvrs, true> {
  using type = TPipeMixed<TP, Pats, Tvrs>;
};

// a[k] bit p = M[k][p]  ->  a[p] bit k = M[k][p]: a 32 x 32 bit transpose in
// one lane's registers.  Stage j exchanges bit j of the word index with bit
// j of the bit index; the byte stages (j = 16, 8) are one v_perm a word, the
// bit stages (4, 2, 1) a shift and a v_bitop3 a word.
__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t x = a[k], y = a[k + 16];
    a[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);       // lo16(x) | lo16(y) << 16
    a[k + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);  // hi16(x) | hi16(y) << 16
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & 8) continue;
    const uint32_t x = a[k], y = a[k + 8];
    a[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);      // bytes x0 y0 x2 y2
    a[k + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);  // bytes x1 y1 x3 y3
  }
  static_for<0, 3>([&](auto ji) {
    constexpr int j = 4 >> decltype(ji)::value;
    constexpr uint32_t m = j == 4 ? 0x0F0F0F0Fu : j == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (k & j) continue;
      const uint32_t x = a[k], y = a[k + j];
      a[k] = (x & m) | ((y << j) & ~m);
      a[k + j] = ((x >> j) & m) | (y & ~m);
    }
  });
}

// The half-stripe buffer: the planes of a bundle's 32 reads over a half
// stripe (32 windows = 32 L positions = L plane words a read) plus a margin
// of plane words on each side (the walks' halos and the 32-position ranges'
// overhang), staged in LDS: slot s's words are row s, kRow words of 8 bytes.
// Row word j of half stripe hs is plane word hs L - 2 - (hs L & 1) + j of the
// read (even, so that the 16-byte loads that fill it are aligned).  A row is
// filled by kLoads 16-byte buffer loads straight into LDS (lane u = unit u of
// the row's 64-unit piece c; the LDS address is the load's base + 16 lane).
template <int kL>
struct TsStage {
  static constexpr int kRow = 2 * ((kL + 7) / 2);         // plane words a row (>= L + 6, even)
  static constexpr int kRowUnits = kRow / 2;              // 16-byte units a row
  static constexpr int kLoads = (kRowUnits + kWave - 1) / kWave;  // loads a row
  static constexpr int kWords = NT_BUNDLE * kRow * 2;     // uint32 words of LDS
  __device__ __forceinline__ static int first_word(int hs) { return (hs * kL - 2) & ~1; }
};

// LDS banks of the cuts.  Every lane reads its pieces from all 32 rows, one
// ds_read_b64 a row; in slot order the 32 lanes of a half wave read ONE row
// at their own words (lane l: word (l L + h L0 - kLam) / 32 + c), ~3.1 L / 32
// words apart, whose bank words (mod 32) collide pairwise: 2-way conflicts,
// twice the LDS cycles of every cut read (SQ_LDS_BANK_CONFLICT at c5: 2.75
// extra cycles a LDS instruction, profiles/r06).  So lane l reads the rows in
// its own rotated order, row (s + rot_l) mod 32 at read s: its bank word
// moves by rot_l kRow (mod 32), and rot_l in 0..kMaxRot is chosen per lane
// and half (a bipartite matching of lanes to the 32 bank words, at compile
// time) so that every read of a half wave hits 32 distinct bank words.  The
// walk is bitwise in the slots, so bit s of every word then belongs to slot
// (s + rot_l) mod 32: the lane's counters are rotated back before the halves
// are added (one v_alignbit a counter word).
constexpr int kTsMaxRot = 3;
template <int kL, int kLam, int kRow>
struct TsRot {
  struct Tab {
    int rot[64];
  };
  // lane l of half h: its first word mod 32, and the bank word of rotation r
  static constexpr int word(int l, int h) { return (l * kL + h * ((kL + 1) / 2) - kLam) >> 5; }
  static constexpr int bank(int l, int h, int r) { return (((word(l, h) + r * kRow) % 32) + 32) % 32; }
  struct Match {
    int owner[32];  // bank word -> lane (or -1)
    int rot[32];
  };
  // Kuhn's augmenting path from lane l (visited: bank words seen this round)
  static constexpr bool augment(Match& m, int l, int h, bool (&seen)[32]) {
    for (int r = 0; r <= kTsMaxRot; ++r) {
      const int b = bank(l, h, r);
      if (seen[b]) continue;
      seen[b] = true;
      if (m.owner[b] < 0 || augment(m, m.owner[b], h, seen)) {
        m.owner[b] = l;
        m.rot[l] = r;
        return true;
      }
    }
    return false;
  }
  static constexpr Tab make() {
    Tab t{};
    for (int h = 0; h < 2; ++h) {
      Match m{};
      for (int b = 0; b < 32; ++b) m.owner[b] = -1;
      for (int l = 0; l < 32; ++l) m.rot[l] = 0;
      for (int l = 0; l < 32; ++l) {
        bool seen[32] = {};
        augment(m, l, h, seen);  // (an unmatched lane keeps rotation 0: a conflict, not an error)
      }
      for (int l = 0; l < 32; ++l) t.rot[32 * h + l] = m.rot[l];
    }
    return t;
  }
  static constexpr Tab kTab = make();
  static constexpr uint64_t mask(int bit) {
    uint64_t x = 0;
    for (int l = 0; l < 64; ++l) x |= (uint64_t)((kTab.rot[l] >> bit) & 1) << l;
    return x;
  }
  static constexpr uint64_t kBit0 = mask(0), kBit1 = mask(1);
  static_assert(kTsMaxRot <= 3, "two mask bits");
  // this lane's rotation
  __device__ __forceinline__ static int of_lane(int lane) {
    return (int)((kBit0 >> lane) & 1u) | ((int)((kBit1 >> lane) & 1u) << 1);
  }
};

// The walk of one half stripe per lane, from the LDS buffer.  Lane (l, h) =
// (lane & 31, lane >> 5) walks window 32 hs + l's positions [h L0, h L0 + L0)
// -- L0 = ceil(L / 2); the second half is L0 - 1 long when L is odd, its last
// step's count masked -- plus kLam positions of halo each side: walk index i
// = 0 .. kN - 1 is position (32 hs + l) L + h L0 - kLam + i.  Per range of 32
// positions: the pieces at the lane's bit offset of plane words (q, q + 1) of
// every slot (LDS reads, v_alignbit), two 32 x 32 bit transposes in the
// lane's registers, and the range's steps of the pipe.  The pieces of range
// r + 1 are cut before range r is walked, so that the buffer is free once the
// last range's are: issue() then starts the next half stripe's loads into it,
// which land while the lane walks (for L <= 116, kNR = 2: the whole walk).
// Position -1 of the first window (Biostrings' out-of-bound start) is masked
// in the prologue; the read ends are not (the calling kernel recounts every
// read's last window, see the header).
// Lane conditions as mask words (v_and / v_bitop3) instead of selects
// (v_cndmask: on a non-VCC SGPR pair ~0.8-1.5 issue slots more than other VALU
// at one wave a SIMD, on VCC a quarter of the rate in a chain of selects:
// profiles/r06/valu_issue_1w/) in the walk's prologue, the halves' add and the
// checkpoints: same box, c5 / c50k +2 %, c10k +1.7 % -- but c4 (3 passes)
// -1.5 % with the halves' add and checkpoints masked, so those are 2-pass
// programs only; the prologue's mask is every program's (c4 +0.6 %;
// profiles/r06/ab_masks/)
template <class TP>
constexpr bool ts_mask_selects() { return TP::kNP == 2; }

template <class TP, class Pats, class Tvrs>
struct TWalkerL {
  static constexpr int kL = TP::kL, kLam = TP::kLam;
  static constexpr int kL0 = (kL + 1) / 2;
  static constexpr int kN = kL0 + 2 * kLam;        // steps of a half-window walk
  static constexpr int kNR = (kN + 31) / 32;       // ranges of 32 positions
  static constexpr int kPro = 2 * kLam;            // prologue steps (no counts)
  static constexpr int kIssueAt = kNR >= 2 ? kNR - 2 : 0;  // the range walked after the buffer's last read
  using St = TsStage<kL>;
  typename TPipeSel<TP, Pats, Tvrs>::type pp;

  typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64;
  // the row of read s in this lane's rotated order (TsRot): row (s + rot) mod
  // 32; the reads that wrap (s >= 32 - kTsMaxRot) pick their base per lane
  template <int s>
  __device__ __forceinline__ static lds_u64* rrow(lds_u64* a, int rot) {
    if constexpr (s + kTsMaxRot < NT_BUNDLE) return a + s * St::kRow;
    else return a + s * St::kRow - (s + rot >= NT_BUNDLE ? NT_BUNDLE * St::kRow : 0);
  }

  // range r's pieces of every slot: rows from the lane's word w (LDS), read
  // s = slot (s + rot) mod 32
  template <int r>
  __device__ __forceinline__ static void cut(const uint2* row, uint32_t sh, int rot, uint32_t (&lo)[32],
                                             uint32_t (&hi)[32]) {
    // (volatile: one ds_read_b64 a word -- two accesses of 32 lanes, 256 B a
    // clock -- where the compiler would pair a word with its neighbour into a
    // ds_read2_b64, which the LDS serves at half that rate)
    lds_u64* a = (lds_u64*)(row) + rot * St::kRow;
    static_for<0, NT_BUNDLE>([&](auto si) {
      constexpr int s = decltype(si)::value;
      lds_u64* vr = rrow<s>(a, rot);
      const uint64_t x = vr[r], y = vr[r + 1];
      lo[s] = __builtin_amdgcn_alignbit((uint32_t)y, (uint32_t)x, sh);
      hi[s] = __builtin_amdgcn_alignbit((uint32_t)(y >> 32), (uint32_t)(x >> 32), sh);
    });
  }

  // both ranges' pieces of every slot (kNR = 2): plane words w, w + 1, w + 2
  __device__ __forceinline__ static void cut2(const uint2* row, uint32_t sh, int rot, uint32_t (&lo)[kNR][32],
                                              uint32_t (&hi)[kNR][32]) {
    lds_u64* a = (lds_u64*)(row) + rot * St::kRow;
    static_for<0, NT_BUNDLE>([&](auto si) {
      constexpr int s = decltype(si)::value;
      lds_u64* vr = rrow<s>(a, rot);
      const uint64_t x = vr[0], y = vr[1], z = vr[2];
      lo[0][s] = __builtin_amdgcn_alignbit((uint32_t)y, (uint32_t)x, sh);
      hi[0][s] = __builtin_amdgcn_alignbit((uint32_t)(y >> 32), (uint32_t)(x >> 32), sh);
      lo[1][s] = __builtin_amdgcn_alignbit((uint32_t)z, (uint32_t)y, sh);
      hi[1][s] = __builtin_amdgcn_alignbit((uint32_t)(z >> 32), (uint32_t)(y >> 32), sh);
    });
  }

  // the first run (of the at most 4 a range's steps split into: prologue /
  // counted, 16 steps at most) of range r that has steps
  template <int r>
  static constexpr int first_run() {
    const int a = 32 * r, b = 32 * r + 32 < kN ? 32 * r + 32 : kN;
    for (int q = 0; q < 4; ++q) {
      const int m0 = a + 16 * (q >> 1), m1 = a + 16 * (q >> 1) + 16 < b ? a + 16 * (q >> 1) + 16 : b;
      const bool pro = !(q & 1);
      const int u0 = pro ? m0 : (m0 > kPro ? m0 : kPro);
      const int u1 = pro ? (m1 < kPro ? m1 : kPro) : m1;
      if (u1 > u0) return q;
    }
    return 0;
  }

  // one half stripe: the counts of the lane's half window into acc.  buf: the
  // staged rows; w: the lane's first plane word, relative to the row start;
  // sh: its bit offset; first: the lane walks position -1 of the read;
  // cmask: 0 when the lane's last counted step is past its window (odd L, h = 1);
  // rot: the lane's row rotation (TsRot; acc comes back in slot order);
  // issue(): called once the buffer has been read
  template <class Issue>
  __device__ __forceinline__ void walk(const uint2* buf, int w, uint32_t sh, bool first, uint32_t cmask, int rot,
                                       uint32_t (&acc)[3][8], Issue&& issue) {
    pp.init();
    // position -1 of the read masked by a mask word (an AND), not a select
    uint32_t fmask = first ? 0u : 0xFFFFFFFFu;
    asm volatile("" : "+v"(fmask));
    const uint2* row = buf + w;
    uint32_t plo[kNR][32], phi[kNR][32];
    if constexpr (kNR == 2) {
      cut2(row, sh, rot, plo, phi);  // (both ranges from the 3 words they span: a quarter fewer reads)
    } else {
      cut<0>(row, sh, rot, plo[0], phi[0]);
    }
    static_for<0, kNR>([&](auto ri) {
      constexpr int r = decltype(ri)::value;
      if constexpr (kNR != 2 && r + 1 < kNR) cut<r + 1>(row, sh, rot, plo[r + 1], phi[r + 1]);
      uint32_t (&lo)[32] = plo[r];
      uint32_t (&hi)[32] = phi[r];
      transpose32(lo);
      transpose32(hi);
      // the range's steps in runs of at most 16 (the prologue's apart)
      constexpr int a = 32 * r, b = 32 * r + 32 < kN ? 32 * r + 32 : kN;
      static_for<0, 4>([&](auto qi) {
        constexpr int q = decltype(qi)::value;
        constexpr int m0 = a + 16 * (q >> 1), m1 = a + 16 * (q >> 1) + 16 < b ? a + 16 * (q >> 1) + 16 : b;
        constexpr bool pro = !(q & 1);
        constexpr int u0 = pro ? m0 : (m0 > kPro ? m0 : kPro);
        constexpr int u1 = pro ? (m1 < kPro ? m1 : kPro) : m1;
        if constexpr (u1 > u0) {
          // odd L: the count of the walk's last step is masked for h = 1
          constexpr int ms = (!pro && (kL & 1) && u1 == kN) ? kN - 1 - u0 : -1;
          pp.template run<u1 - u0, !pro, pro, ms>(
              [&](auto ui) {
                constexpr int i = u0 + decltype(ui)::value, j = i - 32 * r;
                if constexpr (pro) return make_uint3(lo[j], hi[j], i < kLam ? fmask : 0xFFFFFFFFu);
                else return make_uint3(lo[j], hi[j], cmask);
              },
              [](auto) {});
          pp.bc[0].pin();
          pp.bc[1].pin();
          if constexpr (TP::kNP == 3) pp.bc[2].pin();
          __builtin_amdgcn_sched_barrier(0);
          // the buffer's last reads returned under this run: start the next
          // half stripe's loads into it
          if constexpr (q == first_run<r>() && r == kIssueAt) issue();
        }
      });
    });
    // bit s of the counters is slot (s + rot) mod 32: rotate them back
    const uint32_t rsh = (uint32_t)(32 - rot) & 31u;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int b = 0; b < 8; ++b)
        acc[p][b] = p < TP::kNP ? __builtin_amdgcn_alignbit(pp.bc[p].acc[b], pp.bc[p].acc[b], rsh) : 0u;
  }
};

// acc += x, 8-bit counts bit-sliced over the 32 slots (a ripple adder per slot)
__device__ __forceinline__ void bitsliced_add(uint32_t (&acc)[8], const uint32_t (&x)[8]) {
  uint32_t c = 0u;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint32_t a = acc[b], y = x[b];
    acc[b] = xor3(a, y, c);
    c = mj3(a, y, c);
  }
}

// 8x8 bit transpose inside every byte of 8 words: afterwards byte g of word j
// holds bit b (of word b before) = bit b of the count of slot 8 g + j.
__device__ __forceinline__ void transpose8(uint32_t (&a)[8]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t t = ((a[r] >> 4) ^ a[r + 4]) & 0x0F0F0F0Fu;
    a[r + 4] ^= t;
    a[r] ^= t << 4;
  }
#pragma unroll
  for (int r = 0; r < 8; r += (r & 1) ? 3 : 1) {  // 0, 1, 4, 5
    const uint32_t t = ((a[r] >> 2) ^ a[r + 2]) & 0x33333333u;
    a[r + 2] ^= t;
    a[r] ^= t << 2;
  }
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    const uint32_t t = ((a[r] >> 1) ^ a[r + 1]) & 0x55555555u;
    a[r + 1] ^= t;
    a[r] ^= t << 1;
  }
}

// Per-slot metadata of the bundle being scanned (per-wave LDS, written once
// per bundle): not held in registers across the walk.  {nw, wb} first: one
// ds_read_b128 gives a slot's count row.
struct TSlot {
  uint32_t nw;            // windows (0: empty slot)
  uint32_t wb_lo, wb_hi;  // index of pass 0's window counts (win_off * np)
  uint32_t len;
  uint32_t ab_lo, ab_hi;  // aux_base(win_off, r, np): telomeric bitmasks, then checkpoints
  uint32_t r, occ;
  uint32_t run[3];        // covered bases of the windows before this stripe, per pass
  uint32_t pad;
};
constexpr int kTsSlotWords = 12;

// per-wave LDS of the bundle scan (uint32 words): the slots; the count rows
// of kRS stripes per pass (row s = slot s, 16 kRS words = 64 kRS windows, 4 to a
// word: byte b = window 4 q + b of word q -- the uint8 counts, stored as whole
// 128-byte lines every second stripe for 2 passes; a 3-pass program stores
// 64-byte halves every stripe, which keeps its LDS under the 40 KB of four
// waves per CU); and the telomeric bitmask words / checkpoints of kF stripes,
// written out together (whole runs of a read's row instead of 4-byte pieces: a
// partly written line costs a read-modify-write in the memory system).
constexpr int kTsFlush2 = 2;  // stripes per flush of a 2-pass program (even; LDS: the half-stripe buffer)
constexpr int kTsFlush3 = 2;  // ... of a 3-pass program
template <int kNP>
struct TsAux {
  static constexpr int kF = kNP == 3 ? kTsFlush3 : kTsFlush2;  // stripes per flush (even)
  static_assert(kF >= 2 && kF % 2 == 0, "flush depth");
  static constexpr int kRS = kNP == 3 ? 1 : 2;                 // stripes of count rows
  static constexpr int kRow = 16 * kRS;                         // words of a count row
  static constexpr int kCtWords = kNP * NT_BUNDLE * kRow;      // [p][s][kRS stripes x 16 words]
  static constexpr int kTmWords = kNP * NT_BUNDLE * kF * 2;   // [p][s][stripe] u64
  static constexpr int kCkWords = kNP * NT_BUNDLE * 4 * kF;   // [p][s][4 stripe + g] u32
  static constexpr int kWords = kCtWords + kTmWords + kCkWords;
};
// per-wave LDS words of a kNP-pass program's bundle scan
template <int kNP, int kL>
constexpr int ts_lds_words() {
  return NT_BUNDLE * kTsSlotWords + TsAux<kNP>::kWords + TsStage<kL>::kWords;
}

// 4x4 byte transpose inside every quad of lanes: lane i of the quad gets byte
// i of the quad's four words (byte i' from lane i') -- two DPP exchanges
__device__ __forceinline__ uint32_t quad_byte_transpose(uint32_t x, uint32_t sel2, uint32_t sel1) {
  const uint32_t p2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);  // lane ^ 2
  x = __builtin_amdgcn_perm(p2, x, sel2);
  const uint32_t p1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);  // lane ^ 1
  return __builtin_amdgcn_perm(p1, x, sel1);
}

__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// A bundle whose slots' planes do not lie within 2 GiB of each other (a
// device-resident batch planned without its blk_off, nt_bundle_plan) is not
// scanned: its reads' first checkpoint -- the covered bases before window 0,
// always 0 -- is set to this, and the calling kernel reports them as a layout
// error (NT_FLAG_ERR_ALIGN) instead of calling them.
constexpr uint32_t kTsSpanError = 0xFFFFFFFFu;
constexpr uint64_t kTsMaxSpan = 0x7FFFFFF0ull;  // bytes

// x of lane ^ 32: one v_permlane32_swap (a VALU op: the two halves of x
// trade places) where __shfl_xor is a ds_bpermute through the LDS
__device__ __forceinline__ uint32_t xor32(uint32_t x, bool lower) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return lower ? r[1] : r[0];
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
  return ((uint64_t)hi << 32) | lo;
}

// The bundle scan: every bundle of the batch, one wave per bundle (claimed
// from 8 per-XCD queues), its half stripes in turn.  Per half stripe: the
// staged planes go from registers into the LDS buffer, the next half stripe's
// planes are loaded into those registers (16-byte loads, a read's span whole
// lines: the walk runs meanwhile), the lanes walk their half windows, and the
// two halves of every window are added (lane l + 32 h holds window 32 hs + l
// of the output stripe hs / 2 for h = hs & 1); every second half stripe (and
// the last) goes through the output stage as one stripe of 64 windows.
template <class TP, class Pats, class Tvrs>
__device__ __forceinline__ void tscan_bundles(const NtBatch& B, const NtOut& O, uint64_t* __restrict__ tmask,
                                              unsigned long long* __restrict__ queue,
                                              uint32_t thr_full, uint32_t* wlds) {
  constexpr int kL = TP::kL, kNP = TP::kNP, kLam = TP::kLam;
  static_assert(kL <= 170, "8-bit counts (nt_tscan_eligible)");
  using St = TsStage<kL>;
  using Wk = TWalkerL<TP, Pats, Tvrs>;
  // The calling kernel of the previous bundle range runs beside this one
  // (nt_host.cpp: a second stream) on the same SIMDs: the scan, VALU-bound at
  // one wave per SIMD, takes the issue arbitration first (priority, then age),
  // the latency-bound calling fills the cycles it leaves
  __builtin_amdgcn_s_setprio(2);
  const int lane = threadIdx.x & (kWave - 1);
  TSlot* sl = reinterpret_cast<TSlot*>(wlds);
  uint32_t* ct = wlds + NT_BUNDLE * kTsSlotWords;  // the count rows
  using Aux = TsAux<kNP>;
  uint32_t* tmb = ct + Aux::kCtWords;  // bitmask words of the flush
  uint32_t* ckb = tmb + Aux::kTmWords;  // checkpoints of the flush
  uint2* stage = reinterpret_cast<uint2*>(ckb + Aux::kCkWords);  // the half-stripe buffer
  // quad_byte_transpose selectors (v_perm: bytes 0-3 from x, 4-7 from the partner)
  const uint32_t sel2 = (lane & 2) ? 0x03020706u : 0x05040100u;
  const uint32_t sel1 = (lane & 1) ? 0x03070105u : 0x06020400u;
  const int ms = lane & (NT_BUNDLE - 1), mh = lane >> 5;  // output lane = slot ms, windows 32 mh..
  // this lane's half window: position (32 hs + ms) L + mh L0 - kLam starts the
  // walk, plane word 32 hs L / 32 = hs L exactly, so the word offset within the
  // half stripe and the bit offset are the same in every half stripe
  const int p0 = ms * kL + mh * Wk::kL0 - kLam;  // >= -kLam
  const int wq = p0 >> 5;                        // (arithmetic: -1 for lane 0)
  const uint32_t sh = (uint32_t)(p0 & 31);
  const uint32_t cmask = (mh && (kL & 1)) ? 0u : 0xFFFFFFFFu;
  const int rot = TsRot<kL, kLam, St::kRow>::of_lane(lane);  // this lane's row order in the cuts
  const uint64_t nb = B.n_bundles;
  uint32_t qi = blockIdx.x % NT_QUEUES, qtried = 0;
  auto claim = [&]() -> uint64_t {
    while (qtried < NT_QUEUES) {
      const uint64_t q0 = nb * qi / NT_QUEUES, q1 = nb * (qi + 1) / NT_QUEUES;
      unsigned long long v = 0;
      if (lane == 0) v = atomicAdd(queue + qi * NT_QUEUE_STRIDE, 1ull);
      const uint64_t o = uniform_u64(v);
      if (o < q1 - q0) return q0 + o;
      qi = qi + 1 == NT_QUEUES ? 0 : qi + 1;
      ++qtried;
    }
    return nb;
  };
  for (uint64_t b = claim(); b < nb; b = claim()) {
    // ---- slot metadata into LDS (lanes 0..31 = slots; 32..63 the same)
    uint32_t n_max;
    bool span_ok;
    uint64_t base, top;
    {
      const uint32_t r = B.bnd_read[b * NT_BUNDLE + (lane & 31)];
      const bool o = r != 0xFFFFFFFFu;
      const uint32_t len = o ? B.len[r] : 0u;
      const uint64_t wo = o ? B.win_off[r] : 0ull;
      const uint64_t bo = o ? B.blk_off[r] : ~0ull;  // first plane word (8 bytes) of the read
      // the bundle's planes: from its lowest slot's first word to its highest
      // slot's last one
      uint64_t lo = bo, hi = o ? bo + 2ull * ((len + 63u) >> 6) : 0ull;
#pragma unroll
      for (int x = 1; x < NT_BUNDLE; x <<= 1) {
        const uint64_t l2 = shfl_xor_u64(lo, x), h2 = shfl_xor_u64(hi, x);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
      }
      base = uniform_u64(lo);
      top = uniform_u64(hi);
      span_ok = (top - base) * 8ull <= kTsMaxSpan;
      if (lane < NT_BUNDLE) {
        TSlot t;
        t.len = len;
        t.nw = o ? (uint32_t)split_window_count(len, kL) : 0u;
        t.r = r;
        t.occ = o ? 1u : 0u;
        const uint64_t wb = wo * kNP, ab = aux_base(wo, r, kNP);
        t.wb_lo = (uint32_t)wb;
        t.wb_hi = (uint32_t)(wb >> 32);
        t.ab_lo = (uint32_t)ab;
        t.ab_hi = (uint32_t)(ab >> 32);
        t.run[0] = t.run[1] = t.run[2] = 0u;
        t.pad = o && span_ok ? (uint32_t)((bo - base) * 8ull) : 0u;  // the slot's planes, bytes from base
        sl[lane] = t;
        // the first checkpoint (the calling kernel's span check reads it for
        // every bundled read): the flush writes it for a read with windows; a
        // read of none (<= L/2 bases) or an unscanned bundle gets it here
        if (o && (!span_ok || t.nw == 0u))  // see kTsSpanError
          reinterpret_cast<uint32_t*>(tmask + ab + (uint64_t)kNP * aux_nmw((int)t.nw))[0] =
              span_ok ? 0u : kTsSpanError;
      }
      n_max = (uint32_t)__builtin_amdgcn_readfirstlane((int)len);  // slot 0 = the longest
    }
    wave_sync();
    if (!span_ok) continue;
    const int nwin = ((int)n_max + kL - 1) / kL;  // windows of the longest read (blocks of L)
    const int nhs = (nwin + 31) / 32;             // half stripes
    const int nst = (nhs + 1) / 2;                // output stripes of 64 windows
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(B.planes) + base * 2ull, (short)0, (int)(uint32_t)((top - base) * 8ull), 0x00020000);
    // the buffer's loads: row s piece c <- 16-byte units 64 c + lane of slot s
    // (lanes past the row's end idle), voffset = the half stripe's first word
    // + the unit (16 lane + 1024 c: one register for every slot), soffset =
    // the slot's planes (bytes from the descriptor base, lane s of pad_v), M0
    // = the row's LDS address: a load costs its soffset (v_readlane) and its
    // M0 (s_add) besides itself.  The raw buffer's range check covers voffset
    // + soffset (tools/fused_probe.hip k_soff: lane 32 of an in-range voffset
    // with a soffset past the range loads 0), so a short slot's rows past the
    // bundle's last plane word (its half stripes beyond its read; at the planes
    // allocation's end for the batch's last read) load zeros and never reach
    // past the allocation.  Half stripe 0 starts 2 words before the reads:
    // voffset wraps for lane 0 there, which then loads zeros or the 16 bytes
    // before the read (positions -64 .. -1, masked in the walk's prologue)
    const uint32_t pad_v = sl[lane & (NT_BUNDLE - 1)].pad;
    // the buffer's LDS address, provably wave-uniform (the loads' M0)
    const uint32_t stage_lds = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(unsigned long)(__attribute__((address_space(3))) void*)stage);
    auto fetch = [&](int hs) {
      const uint32_t vl = 16u * (uint32_t)lane + (uint32_t)(St::first_word(hs) * 8);  // (mod 2^32)
      // (the M0 values summed here, on the scalar unit: hoisted out of the
      // loop they were 32 SGPRs, spilled to VGPR lanes and read back a load)
      uint32_t m0 = stage_lds;
      asm volatile("" : "+s"(m0));
#pragma unroll
      for (int c = 0; c < St::kLoads; ++c) {
        // (the slots' offsets are read with every lane active: a lane the
        // load's mask leaves out has no defined value to read)
        uint32_t pad[NT_BUNDLE];
#pragma unroll
        for (int s = 0; s < NT_BUNDLE; ++s) pad[s] = (uint32_t)__builtin_amdgcn_readlane((int)pad_v, s);
        if (kWave * c + lane < St::kRowUnits) {
#pragma unroll
          for (int s = 0; s < NT_BUNDLE; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void*)(unsigned long)(m0 + 8u * (s * St::kRow + 2 * kWave * c)),
                16, 1024u * c + vl, pad[s], 0, 0);
        }
      }
    };
    fetch(0);
    // this lane's slot (ms) of the output stage: windows, aux base, and the
    // covered bases of the windows before the stripe, per pass (both halves)
    const int m_nw = (int)sl[ms].nw;
    const uint64_t m_ab = u64of(sl[ms].ab_lo, sl[ms].ab_hi);
    uint32_t run[3] = {0u, 0u, 0u};
    uint32_t oacc[3][8];  // the output stripe's counts: lane l + 32 h = window 32 (2 st + h) + l
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int t = 0; t < 8; ++t) oacc[p][t] = 0u;
    for (int hs = 0; hs < nhs; ++hs) {
      // ---- this half stripe's rows have landed (the loads write LDS and
      // count as vmcnt)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // ---- walk the half windows (the next half stripe's loads start once
      // the buffer has been read), add the halves
      {
        int w = wq - St::first_word(hs) + hs * kL;  // the lane's first word in the row
        asm volatile("" : "+v"(w));  // (the row addresses are cut per half stripe, not held in registers)
        uint32_t acc[3][8];
        Wk wk;
        wk.walk(
            stage, w, sh, hs == 0 && lane == 0, cmask, rot, acc,
            [&]() {
              // (every read of the buffer has returned before a load may write it)
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
              if (hs + 1 < nhs) fetch(hs + 1);
            });
        // the halves added: v_permlane32_swap of x with itself gives the lower
        // half's x in both halves of one result and the upper half's in both
        // halves of the other, so their sum needs no per-lane select; the sums
        // go to this half stripe's lanes of the output stripe by a mask
        // (v_bitop3: a select on a lane condition is a v_cndmask, which
        // issues at a fifth of the rate at one wave a SIMD, tools/
        // valu_issue_bench.hip).  An even half stripe leaves the upper lanes
        // as they were: when no odd one follows, their windows lie past every
        // read of the bundle (masked bitmask bits, padding counts, no
        // checkpoint)
        uint32_t sel = mh == (hs & 1) ? ~0u : 0u;
        if constexpr (ts_mask_selects<TP>()) asm volatile("" : "+v"(sel));
#pragma unroll
        for (int p = 0; p < kNP; ++p) {
          if constexpr (!ts_mask_selects<TP>()) {
            uint32_t x[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) x[t] = xor32(acc[p][t], mh == 0);
            bitsliced_add(acc[p], x);
#pragma unroll
            for (int t = 0; t < 8; ++t)  // (an even half stripe clears the second half: none follows the last)
              oacc[p][t] = mh == (hs & 1) ? acc[p][t] : ((hs & 1) ? oacc[p][t] : 0u);
            continue;
          }
          uint32_t a[8], x[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const auto r = __builtin_amdgcn_permlane32_swap(acc[p][t], acc[p][t], false, false);
            a[t] = r[0];
            x[t] = r[1];
          }
          bitsliced_add(a, x);
#pragma unroll
          for (int t = 0; t < 8; ++t) oacc[p][t] = __builtin_amdgcn_bitop3_b32(sel, a[t], oacc[p][t], 0xCA);
        }
      }
      if (!(hs & 1) && hs + 1 < nhs) continue;
      const int st = hs >> 1;
      uint32_t (&acc)[3][8] = oacc;
      // ---- outputs.  Lane k holds the counts of window k of the stripe for
      // the 32 slots, bit-sliced.  A byte transpose (in registers, then LDS)
      // gives row s = slot s's 64 counts: out as whole 128-byte lines (8 lanes
      // per slot), and at lane 32 h + s (windows 32 h ..) for the checkpoint
      // sums; the telomeric bits come from a bit-sliced compare and a bit
      // transpose.  Bitmask words and checkpoints wait in LDS for the flush.
      // Every pass's rows are written before one wave_sync and read back
      // after it (one LDS round trip a stripe, not one a pass).
      const int k0 = st * kWave + 32 * mh;  // this lane's first window
      uint32_t hmask = 0u - (uint32_t)mh;   // (a mask, not a select: see the halves' add)
      if constexpr (ts_mask_selects<TP>()) asm volatile("" : "+v"(hmask));
      const int nv = m_nw - k0 < 0 ? 0 : (m_nw - k0 > 32 ? 32 : m_nw - k0);  // its windows in the read
      const int fs = st % Aux::kF;          // the stripe's place in the flush buffers
      const int half = (st % Aux::kRS) * 16;  // this stripe's 16 words of a row
#pragma unroll
      for (int p = 0; p < kNP; ++p) {
        uint32_t* ctp = ct + p * NT_BUNDLE * Aux::kRow;  // this pass's rows
        uint32_t W[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) W[t] = acc[p][t];
        // telomeric: count >= thr_full, bit-sliced over the slots (bit s = slot s)
        uint32_t ge = ~0u;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const uint32_t tm = ((thr_full >> t) & 1u) ? ~0u : 0u;
          ge = (W[t] & ge) | (~tm & (W[t] | ge));
        }
        if (thr_full > 255u) ge = 0u;
        transpose8(W);  // W[j] byte g = count of slot 8 g + j
        // lane 4 q + i: W[j] byte b = count of slot 8 i + j, window 4 q + b
#pragma unroll
        for (int j = 0; j < 8; ++j) W[j] = quad_byte_transpose(W[j], sel2, sel1);
#pragma unroll
        for (int j = 0; j < 8; ++j) ctp[(8 * (lane & 3) + j) * Aux::kRow + half + (lane >> 2)] = W[j];
        const uint32_t tb = half_bit_transpose(ge, lane) & (nv >= 32 ? ~0u : ((1u << nv) - 1u));
        tmb[((p * NT_BUNDLE + ms) * Aux::kF + fs) * 2 + mh] = tb;
      }
      wave_sync();
      // window counts (uint8: L <= 170), every second stripe: the rows' 128
      // windows as whole lines, store c covers slots 8 c .. 8 c + 7, lane 8 i +
      // q = the 16 bytes (windows 16 q ..) of slot 8 c + i
      // (every LDS read first, then the stores: one round trip, not one a store)
      // (kRS = 1: stores c cover slots 16 c .. 16 c + 15, lane 4 i + q the 16
      // bytes (windows 16 q ..) of slot 16 c + i, 64 bytes a slot)
      if ((st % Aux::kRS) == Aux::kRS - 1 || st == nst - 1) {
        constexpr int kC = 2 * Aux::kRS, kQ = 4 * Aux::kRS;  // stores; lanes a slot
        uint4 m[kC], x[kNP][kC];
#pragma unroll
        for (int c = 0; c < kC; ++c) {
          const int s = (kWave / kQ) * c + lane / kQ, q = lane % kQ;
          m[c] = *reinterpret_cast<const uint4*>(sl + s);  // nw, wb_lo, wb_hi
#pragma unroll
          for (int p = 0; p < kNP; ++p)
            x[p][c] = *reinterpret_cast<const uint4*>(ct + (p * NT_BUNDLE + s) * Aux::kRow + 4 * q);
        }
#pragma unroll
        for (int c = 0; c < kC; ++c) {
          const int kq = (st / Aux::kRS) * Aux::kRS * kWave + 16 * (lane % kQ);
          if (kq < (int)m[c].x) {
#pragma unroll
            for (int p = 0; p < kNP; ++p) {
              uint8_t* w = reinterpret_cast<uint8_t*>(O.win_counts) + u64of(m[c].y, m[c].z) +
                           (uint64_t)p * NT_WIN_ROWS((uint64_t)m[c].x) + kq;
              typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
              const u32x4 vv = {x[p][c].x, x[p][c].y, x[p][c].z, x[p][c].w};
              __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(w));  // (-6 % scan time)
            }
          }
        }
      }
#pragma unroll
      for (int p = 0; p < kNP; ++p) {
        const uint32_t* ctp = ct + p * NT_BUNDLE * Aux::kRow;
        // checkpoints: covered bases before windows 16 jj, jj = 4 st + g
        const uint4 va = *reinterpret_cast<const uint4*>(ctp + ms * Aux::kRow + half + 8 * mh);
        const uint4 vb = *reinterpret_cast<const uint4*>(ctp + ms * Aux::kRow + half + 8 * mh + 4);
        uint32_t ga = 0u, gb = 0u;
        ga = __builtin_amdgcn_udot4(va.x, 0x01010101u, ga, false);
        ga = __builtin_amdgcn_udot4(va.y, 0x01010101u, ga, false);
        ga = __builtin_amdgcn_udot4(va.z, 0x01010101u, ga, false);
        ga = __builtin_amdgcn_udot4(va.w, 0x01010101u, ga, false);
        gb = __builtin_amdgcn_udot4(vb.x, 0x01010101u, gb, false);
        gb = __builtin_amdgcn_udot4(vb.y, 0x01010101u, gb, false);
        gb = __builtin_amdgcn_udot4(vb.z, 0x01010101u, gb, false);
        gb = __builtin_amdgcn_udot4(vb.w, 0x01010101u, gb, false);
        const uint32_t mine = ga + gb;
        uint32_t c0, both;  // before window k0; both halves' sum
        if constexpr (ts_mask_selects<TP>()) {
          // (lower half's sum in both halves of lo2, the upper half's in hi2)
          const auto r2 = __builtin_amdgcn_permlane32_swap(mine, mine, false, false);
          const uint32_t lo2 = r2[0], hi2 = r2[1];
          c0 = run[p] + (lo2 & hmask);
          both = lo2 + hi2;
        } else {
          const uint32_t other = xor32(mine, mh == 0);
          c0 = run[p] + (mh ? other : 0u);
          both = mine + other;
        }
        uint32_t* ckr = ckb + (p * NT_BUNDLE + ms) * 4 * Aux::kF + 4 * fs + 2 * mh;
        ckr[0] = c0;
        ckr[1] = c0 + ga;
        // the read's total when its windows end with the bundle's last stripe
        // (no later stripe holds that checkpoint)
        if (mh && st == nst - 1 && 16 * ((k0 >> 4) + 2) == m_nw)
          reinterpret_cast<uint32_t*>(tmask + m_ab + (uint64_t)kNP * aux_nmw(m_nw))[p * aux_nck(m_nw) + (m_nw >> 4)] =
              c0 + mine;
        run[p] += both;
      }
      // ---- flush the bitmask words and checkpoints of stripes st0 .. st
      // lane -> (slot, stripe) / (slot, checkpoint): coalesced runs of each
      // read's row; every LDS read of a pass first (slot metadata, words), then
      // its stores (c10k scan -1.4 %; one lane per slot instead, its words
      // batched, scattered the stores: +2-5 %)
      if (fs == Aux::kF - 1 || st == nst - 1) {
        wave_sync();
        const int st0 = st - fs;
        constexpr int kI1 = NT_BUNDLE * Aux::kF / kWave, kI2 = NT_BUNDLE * 4 * Aux::kF / kWave;
        // every LDS read of every pass first (slot metadata once), then the stores
        uint32_t n1[kI1], n2[kI2], c2[kNP][kI2];
        uint2 a1[kI1], a2[kI2];
        uint64_t v1[kNP][kI1];
#pragma unroll
        for (int i = 0; i < kI1; ++i) {
          const int e = i * kWave + lane, s = e / Aux::kF, w = e % Aux::kF;
          const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + s);
          n1[i] = ts[0];
          a1[i] = *reinterpret_cast<const uint2*>(ts + 4);
#pragma unroll
          for (int p = 0; p < kNP; ++p)
            v1[p][i] = *reinterpret_cast<const uint64_t*>(tmb + ((p * NT_BUNDLE + s) * Aux::kF + w) * 2);
        }
#pragma unroll
        for (int i = 0; i < kI2; ++i) {
          const int e = i * kWave + lane, s = e / (4 * Aux::kF), g = e % (4 * Aux::kF);
          const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + s);
          n2[i] = ts[0];
          a2[i] = *reinterpret_cast<const uint2*>(ts + 4);
#pragma unroll
          for (int p = 0; p < kNP; ++p) c2[p][i] = ckb[(p * NT_BUNDLE + s) * 4 * Aux::kF + g];
        }
#pragma unroll
        for (int i = 0; i < kI1; ++i) {
          const int e = i * kWave + lane, w = e % Aux::kF, sw = st0 + w;
          const int nw = (int)n1[i];
          if (w <= fs && sw * kWave < nw) {
#pragma unroll
            for (int p = 0; p < kNP; ++p) tmask[u64of(a1[i].x, a1[i].y) + (uint64_t)p * aux_nmw(nw) + sw] = v1[p][i];
          }
        }
#pragma unroll
        for (int i = 0; i < kI2; ++i) {
          const int e = i * kWave + lane, g = e % (4 * Aux::kF), jj = 4 * st0 + g;
          const int nw = (int)n2[i];
          if (g < 4 * (fs + 1) && nw > 0 && 16 * jj <= nw) {
#pragma unroll
            for (int p = 0; p < kNP; ++p)
              reinterpret_cast<uint32_t*>(tmask + u64of(a2[i].x, a2[i].y) + (uint64_t)kNP * aux_nmw(nw))[
                  p * aux_nck(nw) + jj] = c2[p][i];
          }
        }
        wave_sync();
      }
      wave_sync();
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int t = 0; t < 8; ++t) oacc[p][t] = 0u;
    }
    wave_sync();
  }
}
}  // namespace nt
