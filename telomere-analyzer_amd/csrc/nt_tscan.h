// nt_tscan.h -- the bundle scan ("T-scan") of the NanoTel hot path on gfx950.
//
// The same outputs as scan_reads (nt_scan.h): per read and pass the covered
// bases of every subseq_length window (analyze_subtelos / get_density_iranges
// / get_sub_density, NanoTel.R:717-766, 308-397, 449-468), the telomeric-window
// bitmask (class -5, NanoTel.R:749-758) and the running-count checkpoints the
// calling kernel sums with -- computed from the T-layout (nt_common.h): reads
// grouped 32 to a BUNDLE, every plane word holding ONE position of all 32
// reads (bit s = slot s).  A shift by one position is then a register rename,
// and the whole walk -- the letter tests of matchPattern, the 3-letter
// majority combine (<= 1 mismatch, Biostrings' out-of-bound rule), the
// coverage spread (trim + IRanges::reduce) and the per-window counts
// (bit-sliced carry-save adders) -- is plain 3-input bit logic, which gfx950
// issues at full rate (v_bitop3 / v_and / v_or / v_xor), where the per-read
// layout spends its instructions on funnel shifts, DPP neighbour moves and
// popcounts, all of them half rate (tools/valu_issue_bench.hip).
//
// Work split.  A wave claims a bundle from the per-XCD queues and walks its
// stripes: lane k of stripe st owns block 64 st + k = positions [kL, kL + L),
// i.e. split_telo window k of every read.  It walks positions [kL - H,
// (k+1) L + H) (H = longest pattern - 1; the left halo feeds the coverage of
// the block's first bases, the right halo the letter tests of its last
// starts), fully unrolled at compile time (L and the patterns are baked into
// the hiprtc build), and counts the covered bases of its block into 8 bit
// planes per pass (acc[b] bit s = bit b of read s's count; counts <= L <= 170).
//
// Output, lane = window, per stripe and pass: the telomeric bits (count >=
// thr[L]) by a bit-sliced compare and a 32 x 32 bit transpose inside each
// half wave; the counts (uint8: L <= 170) by an 8 x 8 bit transpose within
// every byte, a 4 x 4 byte transpose inside every quad of lanes and an LDS row
// per read, stored from LDS as whole 128-byte lines every second stripe
// (non-temporal); the checkpoints every 16 windows from v_dot4 sums of the
// same rows.  Bitmask words and checkpoints wait in LDS and go out as runs of
// a read's row (TsAux).  The read ends are not masked (the T-layout holds A
// past a read), so the LAST window of every read -- whose width may differ
// from L, and into which split_telo may have merged a short last block
// (NanoTel.R:220) -- is recounted exactly by the calling kernel from the
// per-read planes (call_fix_windows, nt_call.h).
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
  static constexpr int kLam = kH + (kH & 1);      // counting lag (even: loop runs start on slot boundaries)
  static constexpr int kNPos = kL + 2 * kH;       // positions walked per block
  static constexpr int kT = (kL + 1) / 2;         // 16-byte slots per block
  // slots the walk loads, in position order: block k-1 (left halo), k, k+1
  static constexpr int kS0 = kH ? (kL - 1) / 2 - (kL - kH) / 2 + 1 : 0;
  static constexpr int kS1 = kT;
  static constexpr int kS2 = kH ? (kH - 1) / 2 + 1 : 0;
  static constexpr int kNS = kS0 + kS1 + kS2;
  // position index i of the walk -> block (-1, 0, +1), offset in the block
  static constexpr int rel(int i) { return i < kH ? -1 : (i < kH + kL ? 0 : 1); }
  static constexpr int off(int i) { return i < kH ? kL - kH + i : (i < kH + kL ? i - kH : i - kH - kL); }
  static constexpr int fslot(int i) {  // walk slot of position i
    return rel(i) < 0 ? off(i) / 2 - (kL - kH) / 2 : (rel(i) == 0 ? kS0 + off(i) / 2 : kS0 + kS1 + off(i) / 2);
  }
  static constexpr int slot_rel(int f) { return f < kS0 ? -1 : (f < kS0 + kS1 ? 0 : 1); }
  static constexpr int slot_t(int f) { return f < kS0 ? (kL - kH) / 2 + f : (f < kS0 + kS1 ? f - kS0 : f - kS0 - kS1); }
  static constexpr int first_pos(int f) {  // first walk position that reads slot f
    int i = 0;
    while (i < kNPos && fslot(i) != f) ++i;
    return i;
  }
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
  template <int N, bool kCount, bool kVarV, class Get, class Hook>
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
        uint32_t e = 0u;
        static_for<0, kNTvr>([&](auto ti) {
          using D = typename LAt<Tvrs, decltype(ti)::value>::type;
          uint32_t q[kMT];
#pragma unroll
          for (int j = 0; j < kMT; ++j) q[j] = Ts[D::kTT[j] & 15][j0 + j];
          uint32_t b0, b1;
          tcombine<kMT, true>(q, b0, b1);
          e |= b0;
        });
        at[0][x] = e;
        static_for<1, kST + 1>([&](auto si) {
          constexpr int s = decltype(si)::value;
          at[s][x] = stage<ST, s, x>(at[s - 1]);
        });
      }
      if constexpr (kCount) {  // the coverage of position P - kLam
        constexpr int kLam = TP::kLam;
        constexpr int y0 = x - (kLam + 1 - kMP);
        const uint32_t c1 = a1[kSP][y0];
        bc[0].template push<0, u>(a0[kSP][y0]);
        bc[1].template push<0, u>(c1);
        if constexpr (kNTvr > 0) {
          constexpr int yt = x - (kLam + 1 - kMT);
          bc[2].template push<0, u>(c1 | at[kST][yt]);
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

  template <int N, bool kCount, bool kVarV, class Get, class Hook>
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
        bc[0].template push<0, u>(c0);
        bc[1].template push<0, u>(c1);
        if constexpr (kNTvr > 0) {
          static_for<0, GT>([&](auto gi) {
            constexpr int g = decltype(gi)::value, m = mt<g>();
            constexpr int y = x - (kLam + 1 - m);
            ct |= at[g][Spread<m>::kS][y];
          });
          bc[2].template push<0, u>(c1 | ct);
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

#ifndef NT_TS_PIN
#define NT_TS_PIN 1
#endif
// 1: the epilogue prefetches the next stripe's first slots (the ring then
// stays live across the output stage); 0: every stripe starts with prime()
#ifndef NT_TS_DBG_NOAUX  // timing experiments only: no telomeric bitmasks / checkpoints
#define NT_TS_DBG_NOAUX 0
#endif
#ifndef NT_TS_DBG_NOCNT
#define NT_TS_DBG_NOCNT 0
#endif
#ifndef NT_TS_DBG_HALFCNT  // timing experiments only: half of the count stores
#define NT_TS_DBG_HALFCNT 0
#endif
#ifndef NT_TS_LOAD_AUX  // cache policy bits of the T-layout loads (experiments)
#define NT_TS_LOAD_AUX 0
#endif
#ifndef NT_TS_NTSTORE  // non-temporal window-count stores (experiments)
#define NT_TS_NTSTORE 1
#endif
#ifndef NT_TS_XPRIME
#define NT_TS_XPRIME 0
#endif
#ifndef NT_TS_RING  // slots in the walk's prefetch ring (8: one 16-position run ahead; 16: 32)
#define NT_TS_RING 8
#endif
#ifndef NT_TS_HALO  // 1: block halos from the neighbour lanes (TWalkerH), 0: loaded (TWalker)
#define NT_TS_HALO 0
#endif

// The walk of one stripe's block per lane, as a continuous stream of 16-byte
// slots with a register ring of 8 slots (loads issued 8 slots ahead, the
// ring slot refilled right after the tests of its last position, across the
// prologue / loop / epilogue and into the next stripe: no dependent memory
// round trip inside a bundle).  Block k = 64 st + lane walks P = -kLam ..
// kL + kLam - 1 relative to its start; the counts of the covered bases of
// [0, kL) per pass go to acc.  P < 0 of block 0 are outside every read
// (Biostrings' out-of-bound start -1, masked in the prologue); the read ends
// are not masked -- the T-layout holds A there -- so the calling kernel
// recounts the last window of every read (call_fix_windows).
template <class TP, class Pats, class Tvrs>
struct TWalker {
  static constexpr int kL = TP::kL, kLam = TP::kLam, kT = TP::kT;
  static constexpr int D = NT_TS_RING, U = 2 * D;  // ring slots; positions per loop run
  static constexpr int PA = -kLam, PB = kLam;         // prologue positions [PA, PB)
  static constexpr int C = (kL - kLam) / U;           // loop runs: P in [kLam + U c, + U), all < kL
  static constexpr int P1 = kLam + U * C, P2 = kL + kLam;  // epilogue positions [P1, P2)
  static constexpr int NP0 = PB - PA, NE = P2 - P1;
  static constexpr int rel(int P) { return P < 0 ? -1 : (P < kL ? 0 : 1); }
  static constexpr int off(int P) { return P - rel(P) * kL; }
  static constexpr int key(int P) { return (rel(P) + 1) * 65536 + off(P) / 2; }
  // slot index of position P within its static segment [a, P]
  static constexpr int sidx(int a, int P) {
    int j = 0;
    for (int q = a + 1; q <= P; ++q) j += key(q) != key(q - 1);
    return j;
  }
  static constexpr int NA = sidx(PA, PB - 1) + 1;      // prologue slots
  static constexpr int NEs = sidx(P1, P2 - 1) + 1;     // epilogue slots
  static constexpr int NS0 = NA + D * C + NEs;
  static constexpr int NS = (NS0 + D - 1) / D * D;    // stream slots per stripe (padded)
  // first position of segment slot j of the segment starting at a
  static constexpr int spos(int a, int b, int j) {
    for (int q = a; q < b; ++q)
      if (sidx(a, q) == j) return q;
    return b;
  }
  // static stream slot f (not a loop slot): kind 0 = slot (rel, t), 1 = pad (no load)
  static constexpr int srel(int f) {
    return f < NA ? rel(spos(PA, PB, f)) : (f >= NA + D * C && f < NS0 ? rel(spos(P1, P2, f - NA - D * C)) : 2);
  }
  static constexpr int st_(int f) {
    return f < NA ? off(spos(PA, PB, f)) / 2 : (f >= NA + D * C && f < NS0 ? off(spos(P1, P2, f - NA - D * C)) / 2 : 0);
  }

  __amdgpu_buffer_rsrc_t rs;
  int vb[3];   // byte offset of block k + r's slot 0 (r = -1, 0, 1) in this stripe; < 0 / past the end: zeros
  int vbn[3];  // the same in the next stripe
  uint4 S[D];  // the ring: stream slot f sits in S[f % D]
  typename TPipeSel<TP, Pats, Tvrs>::type pp;

  __device__ __forceinline__ uint4 ld(int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, NT_TS_LOAD_AUX);
#if NT_TS_PIN
    __builtin_amdgcn_sched_barrier(0);  // keep the load where it is issued (8 slots ahead)
#endif
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  // load static stream slot f (of this stripe, or of the next one when f >= NS)
  template <int F>
  __device__ __forceinline__ void load_static() {
    constexpr bool nxt = F >= NS;
    constexpr int f = nxt ? F - NS : F;
    if constexpr (f >= NA && f < NA + D * C) {  // a loop slot (only run 0's, from the prime)
      constexpr int so = (kLam / 2 + (f - NA)) * 1024;
      S[F % D] = ld(nxt ? vbn[1] : vb[1], so);
    } else if constexpr (srel(f) == 2) {
      S[F % D] = make_uint4(0u, 0u, 0u, 0u);
    } else {
      constexpr int r = srel(f), so = st_(f) * 1024;
      S[F % D] = ld(nxt ? vbn[r + 1] : vb[r + 1], so);
    }
  }
  // the first D stream slots of a bundle's first stripe
  __device__ __forceinline__ void prime() {
    static_for<0, D>([&](auto fi) { load_static<decltype(fi)::value>(); });
  }
  __device__ __forceinline__ void set_stripe(int st, int lane, bool active) {
#pragma unroll
    for (int r = -1; r <= 1; ++r) {
      const int lr = lane + r;
      const int stl = st + (lr >> 6);  // arithmetic shift: -1 for lane 0, r = -1
      const int o = (stl * kT * kWave + (lr & (kWave - 1))) * 16;  // < 0: out of range (zeros)
      vb[r + 1] = active ? o : -1;
      vbn[r + 1] = active ? o + kT * kWave * 16 : -1;
    }
  }

  // one stripe: counts into acc (the ring then holds the next stripe's first slots)
  __device__ __forceinline__ void walk(bool first, uint32_t (&acc)[3][8]) {
    pp.init();
    {  // prologue: static slots
      auto get = [&](auto ii) {
        constexpr int i = decltype(ii)::value, P = PA + i, f = sidx(PA, P);
        const uint4 v = S[f % D];
        return (off(P) & 1) ? make_uint3(v.z, v.w, (P < 0 && first) ? 0u : 0xFFFFFFFFu)
                            : make_uint3(v.x, v.y, (P < 0 && first) ? 0u : 0xFFFFFFFFu);
      };
      pp.template run<NP0, false, true>(get, [&](auto ui) {
        constexpr int i = decltype(ui)::value, P = PA + i;
        if constexpr (i == NP0 - 1 || key(P + 1) != key(P)) load_static<sidx(PA, P) + D>();
      });
    }
#pragma nounroll
    for (int c = 0; c < C; ++c) {  // loop runs: stream slots NA + D c + i
      auto get = [&](auto ui) {
        constexpr int u = decltype(ui)::value;
        const uint4 v = S[(NA + (u >> 1)) % D];
        return (u & 1) ? make_uint3(v.z, v.w, 0u) : make_uint3(v.x, v.y, 0u);
      };
      const bool last = c == C - 1;
      pp.template run<U, true, false>(get, [&](auto ui) {
        constexpr int u = decltype(ui)::value;
        if constexpr (u & 1) {  // slot i = u / 2 consumed: refill with stream slot NA + D (c + 1) + i
          constexpr int i = u >> 1, fe = NA + D * C + i;  // the target when c is the last run
          constexpr int re = fe < NS0 ? srel(fe) : 2;
          constexpr int soe = fe < NS0 ? st_(fe) * 1024 : 0;
          const int vo_loop = vb[1], so_loop = (kLam / 2 + D * (c + 1) + i) * 1024;
          int vo, so;
          if constexpr (fe < NS && re != 2) {
            vo = last ? vb[re + 1] : vo_loop;
            so = last ? soe : so_loop;
          } else {
            vo = last ? -1 : vo_loop;
            so = so_loop;
          }
          S[(NA + i) % D] = ld(vo, so);
        }
      });
    }
    {  // epilogue: static slots; the refills reach into the next stripe
      auto get = [&](auto ii) {
        constexpr int i = decltype(ii)::value, P = P1 + i, f = NA + D * C + sidx(P1, P);
        const uint4 v = S[f % D];
        return (off(P) & 1) ? make_uint3(v.z, v.w, 0u) : make_uint3(v.x, v.y, 0u);
      };
      pp.template run<NE, true, false>(get, [&](auto ui) {
        constexpr int i = decltype(ui)::value, P = P1 + i;
        if constexpr (i == NE - 1 || key(P + 1) != key(P)) {
          constexpr int f = NA + D * C + sidx(P1, P);
          if constexpr (NT_TS_XPRIME || f + D < NS) load_static<f + D>();
          if constexpr (NT_TS_XPRIME && i == NE - 1) {  // the pad slots of the stream: their refills too
            static_for<f + 1, NS>([&](auto gi) { load_static<decltype(gi)::value + D>(); });
          }
        }
      });
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[p][b] = pp.bc[p].acc[b];
  }
};

// The walk without halo loads (NT_TS_HALO): a block's head slots (positions
// [0, kLam)) and tail slots ([kL - kLam, kL)) are loaded once into registers
// at the stripe start; the prologue takes the left neighbour's tail and the
// epilogue the right neighbour's head from the next / previous lane by DPP
// (wave_shr:1 / wave_shl:1), lane 0 and lane 63 from the previous / next
// stripe's edge block (one uniform load each, the DPP's bound value).  The
// ring streams the own slots in between: block slots kNH .. in order.  The
// block halos are ~8 % of the T-layout reads (FETCH 13.8 vs 12.8 GB at 1 M x
// 50 kb), but this walk measured slower (1 M x 50 kb step 3.10 -> 3.16 ms, same
// box): the halo re-reads hit the caches, the edge loads and DPP do not pay.
// Off (kept for the record and further tries).
template <class TP, class Pats, class Tvrs>
struct TWalkerH {
  static constexpr int kL = TP::kL, kLam = TP::kLam, kT = TP::kT;
  static constexpr int U = 16, D = 8;
  static constexpr int C = (kL - kLam) / U;           // loop runs: P in [kLam + U c, + U), all < kL
  static constexpr int P1 = kLam + U * C, P2 = kL + kLam;  // epilogue positions [P1, P2)
  static constexpr int NP0 = 2 * kLam, NE = P2 - P1;
  static constexpr int kNH = kLam / 2;                // head slots 0 .. kNH - 1
  static constexpr int kT0 = (kL - kLam) / 2;         // tail slots kT0 .. kT - 1
  static constexpr int kNT = kT - kT0;
  static constexpr int NS0 = cmax(8 * C, kT0 - kNH);  // ring stream: block slots kNH + f, f < NS0

  __amdgpu_buffer_rsrc_t rs;
  int vb;          // byte offset of this lane's block in the stripe (< 0: zeros)
  int vl, vr;      // uniform: the previous stripe's last block, the next stripe's first block
  uint4 S[D];      // the ring: stream slot f sits in S[f % D]
  uint4 Hs[kNH > 0 ? kNH : 1], Ts[kNT];  // own head / tail slots
  uint4 XL[kNT], XR[kNH > 0 ? kNH : 1];  // lane 0's left / lane 63's right neighbour slots
  typename TPipeSel<TP, Pats, Tvrs>::type pp;

  __device__ __forceinline__ uint4 ld(int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, NT_TS_LOAD_AUX);
#if NT_TS_PIN
    __builtin_amdgcn_sched_barrier(0);  // keep the load where it is issued
#endif
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  __device__ __forceinline__ void set_stripe(int st, int lane, bool active, int nst) {
    vb = active ? (st * kT * kWave + lane) * 16 : -1;
    vl = st > 0 ? ((st - 1) * kT * kWave + (kWave - 1)) * 16 : -1;
    vr = st + 1 < nst ? (st + 1) * kT * kWave * 16 : -1;
  }
  // the stripe's first loads: edges, neighbours' edges, the ring's first D
  __device__ __forceinline__ void prime() {
#pragma unroll
    for (int j = 0; j < kNT; ++j) Ts[j] = ld(vb, (kT0 + j) * 1024);
#pragma unroll
    for (int j = 0; j < kNH; ++j) Hs[j] = ld(vb, j * 1024);
#pragma unroll
    for (int j = 0; j < kNT; ++j) XL[j] = ld(vl, (kT0 + j) * 1024);
#pragma unroll
    for (int j = 0; j < kNH; ++j) XR[j] = ld(vr, j * 1024);
#pragma unroll
    for (int f = 0; f < D; ++f) S[f] = f < NS0 ? ld(vb, (kNH + f) * 1024) : make_uint4(0u, 0u, 0u, 0u);
  }
  // the neighbour's slot: DPP by one lane, the edge lane's from the uniform load
  template <int kCtrl>
  __device__ __forceinline__ static uint4 nb(const uint4& own, const uint4& edge) {
    return make_uint4((uint32_t)__builtin_amdgcn_update_dpp((int)edge.x, (int)own.x, kCtrl, 0xf, 0xf, false),
                      (uint32_t)__builtin_amdgcn_update_dpp((int)edge.y, (int)own.y, kCtrl, 0xf, 0xf, false),
                      (uint32_t)__builtin_amdgcn_update_dpp((int)edge.z, (int)own.z, kCtrl, 0xf, 0xf, false),
                      (uint32_t)__builtin_amdgcn_update_dpp((int)edge.w, (int)own.w, kCtrl, 0xf, 0xf, false));
  }

  __device__ __forceinline__ void walk(bool first, uint32_t (&acc)[3][8]) {
    pp.init();
    {  // prologue: the left neighbour's tail (wave_shr:1), then the own head
      auto get = [&](auto ii) {
        constexpr int i = decltype(ii)::value, P = -kLam + i;
        uint4 v;
        if constexpr (P < 0) v = nb<0x138>(Ts[(kL + P) / 2 - kT0], XL[(kL + P) / 2 - kT0]);
        else v = Hs[P / 2];
        constexpr bool odd = ((P < 0 ? kL + P : P) & 1) != 0;
        const uint32_t vm = (P < 0 && first) ? 0u : 0xFFFFFFFFu;
        return odd ? make_uint3(v.z, v.w, vm) : make_uint3(v.x, v.y, vm);
      };
      pp.template run<NP0, false, true>(get, [&](auto) {});
    }
#pragma nounroll
    for (int c = 0; c < C; ++c) {  // loop runs: stream slots 8 c + i
      auto get = [&](auto ui) {
        constexpr int u = decltype(ui)::value;
        const uint4 v = S[(u >> 1) % D];
        return (u & 1) ? make_uint3(v.z, v.w, 0u) : make_uint3(v.x, v.y, 0u);
      };
      pp.template run<U, true, false>(get, [&](auto ui) {
        constexpr int u = decltype(ui)::value;
        if constexpr (u & 1) {  // stream slot 8 c + i consumed: refill with 8 (c + 1) + i
          constexpr int i = u >> 1;
          const int f = 8 * (c + 1) + i;
          S[i] = ld(f < NS0 ? vb : -1, (kNH + f) * 1024);
        }
      });
    }
    {  // epilogue: the own slots (ring, then the tail), then the right neighbour's head (wave_shl:1)
      auto get = [&](auto ii) {
        constexpr int i = decltype(ii)::value, P = P1 + i;
        uint4 v;
        if constexpr (P >= kL) v = nb<0x130>(Hs[(P - kL) / 2], XR[(P - kL) / 2]);
        else if constexpr (P / 2 >= kT0) v = Ts[P / 2 - kT0];
        else v = S[(P / 2 - kNH) % D];
        constexpr bool odd = ((P >= kL ? P - kL : P) & 1) != 0;
        return odd ? make_uint3(v.z, v.w, 0u) : make_uint3(v.x, v.y, 0u);
      };
      pp.template run<NE, true, false>(get, [&](auto ui) {
        constexpr int i = decltype(ui)::value, P = P1 + i;
        // a ring slot consumed in the epilogue: refill when the stream goes on
        if constexpr (P < kL && P / 2 < kT0 && (P & 1) && P / 2 - kNH + D < NS0)
          S[(P / 2 - kNH) % D] = ld(vb, (P / 2 + D) * 1024);
      });
    }
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[p][b] = pp.bc[p].acc[b];
  }
};

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
// of two stripes per pass (row s = slot s, 32 words = 128 windows, 4 to a
// word: byte b = window 4 q + b of word q -- the uint8 counts, stored as
// whole 128-byte lines every second stripe); and the telomeric bitmask words
// / checkpoints of kF stripes, written out together (whole runs of a read's
// row instead of 4-byte pieces: a partly written line costs a
// read-modify-write in the memory system).  22.5 KB at most: one workgroup
// per CU (the scan runs at one wave per SIMD) leaves room for two of the
// calling kernel's beside it.
#ifndef NT_TS_KF2  // stripes per flush of a 2-pass program (even)
#define NT_TS_KF2 8
#endif
#ifndef NT_TS_KF3  // ... of a 3-pass program
#define NT_TS_KF3 4
#endif
template <int kNP>
struct TsAux {
  static constexpr int kF = kNP == 3 ? NT_TS_KF3 : NT_TS_KF2;  // stripes per flush (even)
  static_assert(kF >= 2 && kF % 2 == 0, "flush depth");
  static constexpr int kCtWords = kNP * NT_BUNDLE * 32;       // [p][s][2 stripes x 16 words]
  static constexpr int kTmWords = kNP * NT_BUNDLE * kF * 2;   // [p][s][stripe] u64
  static constexpr int kCkWords = kNP * NT_BUNDLE * 4 * kF;   // [p][s][4 stripe + g] u32
  static constexpr int kWords = kCtWords + kTmWords + kCkWords;
};
// per-wave LDS words of a kNP-pass program's bundle scan
template <int kNP>
constexpr int ts_lds_words() {
  return NT_BUNDLE * kTsSlotWords + TsAux<kNP>::kWords;
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

// The bundle scan: every bundle of the batch, one wave per bundle (claimed
// from 8 per-XCD queues).
template <class TP, class Pats, class Tvrs>
__device__ __forceinline__ void tscan_bundles(const NtBatch& B, const NtOut& O, uint64_t* __restrict__ tmask,
                                              unsigned long long* __restrict__ queue,
                                              uint32_t thr_full, uint32_t* wlds) {
  constexpr int kL = TP::kL, kNP = TP::kNP, kT = TP::kT;
  static_assert(kL <= 170, "8-bit counts (nt_tscan_eligible)");
  const int lane = threadIdx.x & (kWave - 1);
  TSlot* sl = reinterpret_cast<TSlot*>(wlds);
  uint32_t* ct = wlds + NT_BUNDLE * kTsSlotWords;  // the count rows
  using Aux = TsAux<kNP>;
  uint32_t* tmb = ct + Aux::kCtWords;  // bitmask words of the flush
  uint32_t* ckb = tmb + Aux::kTmWords;  // checkpoints of the flush
  // quad_byte_transpose selectors (v_perm: bytes 0-3 from x, 4-7 from the partner)
  const uint32_t sel2 = (lane & 2) ? 0x03020706u : 0x05040100u;
  const uint32_t sel1 = (lane & 1) ? 0x03070105u : 0x06020400u;
  const int ms = lane & (NT_BUNDLE - 1), mh = lane >> 5;  // output lane = slot ms, windows 32 mh..
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
    // ---- slot metadata into LDS (lanes 0..31 = slots)
    uint32_t occ, n_max;
    {
      const uint32_t r = B.bnd_read[b * NT_BUNDLE + (lane & 31)];
      const bool o = r != 0xFFFFFFFFu;
      const uint32_t len = o ? B.len[r] : 0u;
      const uint64_t wo = o ? B.win_off[r] : 0ull;
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
        t.pad = 0u;
        sl[lane] = t;
      }
      occ = (uint32_t)__ballot(o && lane < NT_BUNDLE);
      n_max = (uint32_t)__builtin_amdgcn_readfirstlane((int)len);  // slot 0 = the longest
    }
    const int nblk = ((int)n_max + kL - 1) / kL;
    const int nst = (nblk + kWave - 1) / kWave;
    const uint64_t g0 = uniform_u64(B.bnd_stripe[b]), g1 = uniform_u64(B.bnd_stripe[b + 1]);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(B.tplanes) + g0 * (uint64_t)kT * kWave * 4, (short)0,
        (int)((g1 - g0) * (uint64_t)kT * kWave * 16), 0x00020000);
    wave_sync();
#if NT_TS_HALO
    TWalkerH<TP, Pats, Tvrs> wk;
    wk.rs = rs;
    wk.set_stripe(0, lane, lane < nblk, nst);
#else
    TWalker<TP, Pats, Tvrs> wk;
    wk.rs = rs;
    wk.set_stripe(0, lane, lane < nblk);
    if (NT_TS_XPRIME) wk.prime();
#endif
    for (int st = 0; st < nst; ++st) {
      const int k = st * kWave + lane;  // this lane's block = window
      if (!NT_TS_XPRIME || NT_TS_HALO) wk.prime();
      uint32_t acc[3][8];
#if NT_TS_DBG_NOWALK  // timing experiments only: results are wrong
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[p][b] = (uint32_t)(k * 0x9E3779B9u) >> (p + b);
#else
      wk.walk(k == 0, acc);
#endif
#if NT_TS_HALO
      wk.set_stripe(st + 1, lane, k + kWave < nblk, nst);  // lanes past the bundle's last block load nothing
#else
      wk.set_stripe(st + 1, lane, k + kWave < nblk);  // lanes past the bundle's last block load nothing
#endif
#if NT_TS_DBG_NOOUT  // timing experiments only: results are wrong
      {
        uint32_t x = 0;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int b = 0; b < 8; ++b) x ^= acc[p][b] * (b + 1);
        if (x == 0x1234567u) O.flags[0] = 1;
        continue;
      }
#endif
      // ---- outputs.  Lane k holds the counts of window k of the stripe for
      // the 32 slots, bit-sliced.  A byte transpose (in registers, then LDS)
      // gives row s = slot s's 64 counts: out as whole 128-byte lines (8 lanes
      // per slot), and at lane 32 h + s (windows 32 h ..) for the checkpoint
      // sums; the telomeric bits come from a bit-sliced compare and a bit
      // transpose.  Bitmask words and checkpoints wait in LDS for the flush.
      const TSlot& mt = sl[ms];
      const int m_nw = (int)mt.nw;
      const int k0 = st * kWave + 32 * mh;  // this lane's first window
      const int nv = m_nw - k0 < 0 ? 0 : (m_nw - k0 > 32 ? 32 : m_nw - k0);  // its windows in the read
      const int fs = st % Aux::kF;          // the stripe's place in the flush buffers
#pragma unroll
      for (int p = 0; p < kNP; ++p) {
        uint32_t* ctp = ct + p * NT_BUNDLE * 32;  // this pass's rows
        const int half = (st & 1) * 16;            // this stripe's 16 words of a row
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
        for (int j = 0; j < 8; ++j) ctp[(8 * (lane & 3) + j) * 32 + half + (lane >> 2)] = W[j];
        const uint32_t tb = half_bit_transpose(ge, lane) & (nv >= 32 ? ~0u : ((1u << nv) - 1u));
        tmb[((p * NT_BUNDLE + ms) * Aux::kF + fs) * 2 + mh] = tb;
        wave_sync();
        // window counts (uint8: L <= 170), every second stripe: the rows' 128
        // windows as whole lines, store c covers slots 8 c .. 8 c + 7, lane 8 i +
        // q = the 16 bytes (windows 16 q ..) of slot 8 c + i
        if ((st & 1) || st == nst - 1) {
#pragma unroll
          for (int c = 0; c < (NT_TS_DBG_HALFCNT ? 2 : 4); ++c) {  // (HALFCNT: timing only)
            const int s = 8 * c + (lane >> 3), q = lane & 7, kq = (st >> 1) * 2 * kWave + 16 * q;
            const uint4 m = *reinterpret_cast<const uint4*>(sl + s);  // nw, wb_lo, wb_hi
            const uint4 x = *reinterpret_cast<const uint4*>(ctp + s * 32 + 4 * q);
            if (kq < (int)m.x && !NT_TS_DBG_NOCNT) {
              uint8_t* w = reinterpret_cast<uint8_t*>(O.win_counts) + u64of(m.y, m.z) +
                           (uint64_t)p * NT_WIN_ROWS((uint64_t)m.x) + kq;
#if NT_TS_NTSTORE
              typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
              const u32x4 vv = {x.x, x.y, x.z, x.w};
              __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(w));
#else
              *reinterpret_cast<uint4*>(w) = x;
#endif
            }
          }
        }
        // checkpoints: covered bases before windows 16 jj, jj = 4 st + g
        const uint4 va = *reinterpret_cast<const uint4*>(ctp + ms * 32 + half + 8 * mh);
        const uint4 vb = *reinterpret_cast<const uint4*>(ctp + ms * 32 + half + 8 * mh + 4);
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
        const uint32_t other = (uint32_t)__shfl_xor((int)mine, 32, kWave);
        const uint32_t run = mt.run[p];
        const uint32_t c0 = run + (mh ? other : 0u);  // before window k0
        uint32_t* ckr = ckb + (p * NT_BUNDLE + ms) * 4 * Aux::kF + 4 * fs + 2 * mh;
        ckr[0] = c0;
        ckr[1] = c0 + ga;
        // the read's total when its windows end with the bundle's last stripe
        // (no later stripe holds that checkpoint)
        if (mh && st == nst - 1 && 16 * ((k0 >> 4) + 2) == m_nw && !NT_TS_DBG_NOAUX)
          reinterpret_cast<uint32_t*>(tmask + u64of(mt.ab_lo, mt.ab_hi) + (uint64_t)kNP * aux_nmw(m_nw))[
              p * aux_nck(m_nw) + (m_nw >> 4)] = c0 + mine;
        wave_sync();  // every lane has read ct and run[p]
        if (mh == 0) sl[ms].run[p] = run + mine + other;
      }
      // ---- flush the bitmask words and checkpoints of stripes st0 .. st
      // lane -> (slot, stripe) / (slot, checkpoint): coalesced runs of each
      // read's row; every LDS read of a pass first (slot metadata, words), then
      // its stores (c10k scan -1.4 %; one lane per slot instead, its words
      // batched, scattered the stores: +2-5 %)
      if ((fs == Aux::kF - 1 || st == nst - 1) && !NT_TS_DBG_NOAUX) {
        wave_sync();
        const int st0 = st - fs;
        constexpr int kI1 = NT_BUNDLE * Aux::kF / kWave, kI2 = NT_BUNDLE * 4 * Aux::kF / kWave;
#pragma unroll
        for (int p = 0; p < kNP; ++p) {
          uint32_t n1[kI1], n2[kI2], c2[kI2];
          uint2 a1[kI1], a2[kI2];
          uint64_t v1[kI1];
#pragma unroll
          for (int i = 0; i < kI1; ++i) {
            const int e = i * kWave + lane, s = e / Aux::kF, w = e % Aux::kF;
            const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + s);
            n1[i] = ts[0];
            a1[i] = *reinterpret_cast<const uint2*>(ts + 4);
            v1[i] = *reinterpret_cast<const uint64_t*>(tmb + ((p * NT_BUNDLE + s) * Aux::kF + w) * 2);
          }
#pragma unroll
          for (int i = 0; i < kI2; ++i) {
            const int e = i * kWave + lane, s = e / (4 * Aux::kF), g = e % (4 * Aux::kF);
            const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + s);
            n2[i] = ts[0];
            a2[i] = *reinterpret_cast<const uint2*>(ts + 4);
            c2[i] = ckb[(p * NT_BUNDLE + s) * 4 * Aux::kF + g];
          }
#pragma unroll
          for (int i = 0; i < kI1; ++i) {
            const int e = i * kWave + lane, w = e % Aux::kF, sw = st0 + w;
            const int nw = (int)n1[i];
            if (w <= fs && sw * kWave < nw) tmask[u64of(a1[i].x, a1[i].y) + (uint64_t)p * aux_nmw(nw) + sw] = v1[i];
          }
#pragma unroll
          for (int i = 0; i < kI2; ++i) {
            const int e = i * kWave + lane, g = e % (4 * Aux::kF), jj = 4 * st0 + g;
            const int nw = (int)n2[i];
            if (g < 4 * (fs + 1) && nw > 0 && 16 * jj <= nw)
              reinterpret_cast<uint32_t*>(tmask + u64of(a2[i].x, a2[i].y) + (uint64_t)kNP * aux_nmw(nw))[
                  p * aux_nck(nw) + jj] = c2[i];
          }
        }
        wave_sync();
      }
      wave_sync();
    }
    wave_sync();
  }
}


// ======================================================================
// Walker / writer waves (NT_TS_WS=1; off by default: measured no faster).
//
// On gfx9 a wave's vector-memory counter covers its loads AND its stores, in
// issue order: once a wave has issued a store, every later wait for one of its
// loads also waits for that store to be acknowledged.  The bundle scan's walk
// keeps 8 loads in flight per lane and waits on the oldest; with any global
// store in the stripe loop -- the count rows every second stripe, the bitmask /
// checkpoint flush every kF -- those waits took the stores' write latency:
// 0.3 ms of a 1.47 ms launch (c50k; timing builds: no stores 1.17 ms, either
// kind alone 1.47-1.52).  tools/rw_mix_bench.hip isolates it: a read stream
// with one store per 1,000 loads runs 28 % slower, whether the stores go to
// HBM or to a 4 MB L2-resident region; the same stores from OTHER waves cost
// nothing.  So the stores move to a writer wave:
//  * workgroup = 4 walker waves (one per SIMD, the walk and the output stage's
//    arithmetic exactly as before, into LDS) + 1 writer wave;
//  * a walker posts store jobs (the count rows of a stripe pair; a flush of
//    bitmask words and checkpoints) to its ring in LDS; the writer takes them
//    in order, reads the rows from the walker's LDS and issues the global
//    stores; it never waits on its stores;
//  * the walker's LDS rows are single-buffered (the writer drains a job in
//    about a microsecond, a stripe's walk takes ~9): before overwriting them the
//    walker checks that the writer is done with the job that read them; the
//    slot metadata alternate between two buffers per bundle.
// Synchronisation is LDS only (s_waitcnt lgkmcnt(0) before publishing a
// counter, never a vmcnt wait in the walker): counters posted / done per
// walker, a finished flag; the writer exits when every walker has finished
// and every posted job is done.
//
// Measured (1 M x 50 kb, one launch, no calling beside it):
// the walkers then never wait on a store and the job handshake costs nothing
// (writer acknowledging without storing: 2.03-2.08 ms, as the old kernel
// without stores), but the writer's stores still cost 0.6 ms (2.61-2.78 ms,
// the old kernel 2.72-2.76): with them the step moves 15.1 GB (13.7 read, 1.4
// written) at 5.5-5.8 TB/s against the ~6.2 TB/s a read + write stream
// sustains, so the scan is bound by HBM read + write bandwidth, not by the
// stores' latency -- and the fifth wave's registers and LDS leave the calling
// kernel beside the scan a third of its room (0.53 -> 1.5 ms).  Off by
// default; NT_TS_WS=1 (NT_JIT_OPTS=-DNT_TS_WS=1) builds it.
#ifndef NT_TS_WS
#define NT_TS_WS 0
#endif
constexpr int kTsRing = 16;   // store jobs in flight per walker
constexpr int kTsCtl = 4 + kTsRing;  // per walker: posted, done, finished, pad, ring
constexpr uint32_t kJobCnt = 1u, kJobFlush = 2u;

template <int kNP>
constexpr int ts_ws_walker_words() {
  return 2 * NT_BUNDLE * kTsSlotWords + TsAux<kNP>::kWords + kNP * NT_BUNDLE;
}
template <int kNP>
constexpr int ts_ws_lds_words() {
  return 4 * (ts_ws_walker_words<kNP>() + kTsCtl);
}

// LDS-typed volatile accesses (a volatile access through a generic pointer
// stays a FLAT access -- counted in vmcnt, waited with vmcnt(0) -- which put
// every writer job behind its own stores' acknowledgements)
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
__device__ __forceinline__ void lds_publish_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_peek(const uint32_t* p) {
  const uint32_t v = *(const volatile lds_u32_t*)(p);
  asm volatile("" ::: "memory");
  return v;
}
__device__ __forceinline__ void lds_put(uint32_t* p, uint32_t v) {
  asm volatile("" ::: "memory");
  *(volatile lds_u32_t*)(p) = v;
}

#ifndef NT_TS_WS_DBG  // timing experiments only (results wrong): 1 = the writer stores nothing,
#define NT_TS_WS_DBG 0   // 2 = no jobs at all (walkers post nothing, the writer returns at once),
#endif                   // 3 = no flush stores, 4 = no count stores, 5 = counts as 1 KB pieces, no flush
template <int kNP>
struct TsWsRegion {  // one walker's LDS (uint32 words)
  uint32_t* base;
  __device__ __forceinline__ TSlot* sl(int buf) const {
    return reinterpret_cast<TSlot*>(base + buf * NT_BUNDLE * kTsSlotWords);
  }
  __device__ __forceinline__ uint32_t* ct() const { return base + 2 * NT_BUNDLE * kTsSlotWords; }
  __device__ __forceinline__ uint32_t* tmb() const { return ct() + TsAux<kNP>::kCtWords; }
  __device__ __forceinline__ uint32_t* ckb() const { return tmb() + TsAux<kNP>::kTmWords; }
  __device__ __forceinline__ uint32_t* tot() const { return ckb() + TsAux<kNP>::kCkWords; }
};

// The writer's side of a count-row job: stripe pair ending at st (or the
// bundle's last, single stripe), every pass -- the rows' 128 windows as whole
// lines, store c covering slots 8 c .. 8 c + 7, lane 8 i + q = the 16 bytes
// (windows 16 q ..) of slot 8 c + i.
template <int kNP>
__device__ __forceinline__ void ts_write_counts(const NtOut& O, const TsWsRegion<kNP>& R, const TSlot* sl, int st,
                                                int lane, uint32_t dbg_seq = 0u, int dbg_w = 0) {
#pragma unroll
  for (int p = 0; p < kNP; ++p) {
    const uint32_t* ctp = R.ct() + p * NT_BUNDLE * 32;
    uint4 m[4], x[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int s = 8 * c + (lane >> 3), q = lane & 7;
      m[c] = *reinterpret_cast<const uint4*>(sl + s);
      x[c] = *reinterpret_cast<const uint4*>(ctp + s * 32 + 4 * q);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int q = lane & 7, kq = (st >> 1) * 2 * kWave + 16 * q;
      if (kq < (int)m[c].x) {
        uint8_t* w = reinterpret_cast<uint8_t*>(O.win_counts) + u64of(m[c].y, m[c].z) +
                     (uint64_t)p * NT_WIN_ROWS((uint64_t)m[c].x) + kq;
        if (NT_TS_WS_DBG == 5)  // timing only: the same bytes as 1 KB contiguous pieces
          w = reinterpret_cast<uint8_t*>(O.win_counts) + ((uint64_t)blockIdx.x * 4 + dbg_w) * 65536 +
              ((dbg_seq * 8 + p * 4 + c) % 64) * 1024 + lane * 16;
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 vv = {x[c].x, x[c].y, x[c].z, x[c].w};
        __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(w));
      }
    }
  }
}

// The writer's side of a flush job: the bitmask words and checkpoints of
// stripes st0 .. st0 + fs (and, at the bundle's last stripe, the reads'
// totals), coalesced runs of each read's row.
template <int kNP>
__device__ __forceinline__ void ts_write_flush(uint64_t* __restrict__ tmask, const TsWsRegion<kNP>& R,
                                               const TSlot* sl, int st0, int fs, bool last, int lane) {
  using Aux = TsAux<kNP>;
  const uint32_t* tmb = R.tmb();
  const uint32_t* ckb = R.ckb();
  constexpr int kI1 = NT_BUNDLE * Aux::kF / kWave, kI2 = NT_BUNDLE * 4 * Aux::kF / kWave;
#pragma unroll
  for (int p = 0; p < kNP; ++p) {
    uint32_t n1[kI1], n2[kI2], c2[kI2];
    uint2 a1[kI1], a2[kI2];
    uint64_t v1[kI1];
#pragma unroll
    for (int i = 0; i < kI1; ++i) {
      const int e = i * kWave + lane, s = e / Aux::kF, w = e % Aux::kF;
      const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + s);
      n1[i] = ts[0];
      a1[i] = *reinterpret_cast<const uint2*>(ts + 4);
      v1[i] = *reinterpret_cast<const uint64_t*>(tmb + ((p * NT_BUNDLE + s) * Aux::kF + w) * 2);
    }
#pragma unroll
    for (int i = 0; i < kI2; ++i) {
      const int e = i * kWave + lane, s = e / (4 * Aux::kF), g = e % (4 * Aux::kF);
      const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + s);
      n2[i] = ts[0];
      a2[i] = *reinterpret_cast<const uint2*>(ts + 4);
      c2[i] = ckb[(p * NT_BUNDLE + s) * 4 * Aux::kF + g];
    }
#pragma unroll
    for (int i = 0; i < kI1; ++i) {
      const int e = i * kWave + lane, w = e % Aux::kF, sw = st0 + w;
      const int nw = (int)n1[i];
      if (w <= fs && sw * kWave < nw) tmask[u64of(a1[i].x, a1[i].y) + (uint64_t)p * aux_nmw(nw) + sw] = v1[i];
    }
#pragma unroll
    for (int i = 0; i < kI2; ++i) {
      const int e = i * kWave + lane, g = e % (4 * Aux::kF), jj = 4 * st0 + g;
      const int nw = (int)n2[i];
      if (g < 4 * (fs + 1) && nw > 0 && 16 * jj <= nw)
        reinterpret_cast<uint32_t*>(tmask + u64of(a2[i].x, a2[i].y) + (uint64_t)kNP * aux_nmw(nw))[
            p * aux_nck(nw) + jj] = c2[i];
    }
  }
  if (last && lane < NT_BUNDLE) {  // a read whose windows end with the bundle's last stripe: its total
    const uint32_t* ts = reinterpret_cast<const uint32_t*>(sl + lane);
    const int nw = (int)ts[0];
    const uint2 ab = *reinterpret_cast<const uint2*>(ts + 4);
#pragma unroll
    for (int p = 0; p < kNP; ++p) {
      const uint32_t v = R.tot()[p * NT_BUNDLE + lane];
      if (v != 0xFFFFFFFFu && nw > 0)
        reinterpret_cast<uint32_t*>(tmask + u64of(ab.x, ab.y) + (uint64_t)kNP * aux_nmw(nw))[
            p * aux_nck(nw) + (nw >> 4)] = v;
    }
  }
}

template <int kNP>
__device__ void ts_writer(const NtOut& O, uint64_t* __restrict__ tmask, uint32_t* lds) {
  if (NT_TS_WS_DBG == 2) return;
  const int lane = threadIdx.x & (kWave - 1);
  uint32_t* ctl = lds + 4 * ts_ws_walker_words<kNP>();
  uint32_t dn[4] = {0u, 0u, 0u, 0u};
  for (;;) {
    bool any = false;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      uint32_t* c = ctl + w * kTsCtl;
      const uint32_t posted = lds_peek(c);
      while (dn[w] < posted) {
        const uint32_t job = c[4 + dn[w] % kTsRing];
        const TsWsRegion<kNP> R{lds + w * ts_ws_walker_words<kNP>()};
        const TSlot* sl = R.sl((job >> 2) & 1u);
        const int st = (int)(job >> 10), fs = (int)((job >> 4) & 63u);
        if (NT_TS_WS_DBG == 1) {
        } else if (job & kJobCnt) {
          if (NT_TS_WS_DBG != 4) ts_write_counts<kNP>(O, R, sl, st, lane, dn[w], w);
        } else {
          if (NT_TS_WS_DBG != 3 && NT_TS_WS_DBG != 5) ts_write_flush<kNP>(tmask, R, sl, st - fs, fs, (job >> 3) & 1u, lane);
        }
        lds_publish_wait();  // the job's LDS reads have returned: its rows may be overwritten
        lds_put(c + 1, ++dn[w]);
        any = true;
      }
    }
    if (!any) {
      bool all = true;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t* c = ctl + w * kTsCtl;
        all = all && lds_peek(c + 2) != 0u && lds_peek(c) == dn[w];
      }
      if (all) return;
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

// A walker: tscan_bundles' loop with its global stores posted to the writer.
template <class TP, class Pats, class Tvrs>
__device__ void ts_walker(const NtBatch& B, uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue,
                          uint32_t thr_full, uint32_t* lds, int wv) {
  constexpr int kL = TP::kL, kNP = TP::kNP, kT = TP::kT;
  static_assert(kL <= 170, "8-bit counts (nt_tscan_eligible)");
  using Aux = TsAux<kNP>;
  const int lane = threadIdx.x & (kWave - 1);
  const TsWsRegion<kNP> R{lds + wv * ts_ws_walker_words<kNP>()};
  uint32_t* ctl = lds + 4 * ts_ws_walker_words<kNP>() + wv * kTsCtl;
  uint32_t* ct = R.ct();
  uint32_t* tmb = R.tmb();
  uint32_t* ckb = R.ckb();
  uint32_t posted = 0u;
  int64_t cnt_job = -1, flush_job = -1, buf_job[2] = {-1, -1};
  auto wait_done = [&](int64_t seq) {  // the writer has finished job seq
    if (seq < 0 || NT_TS_WS_DBG == 2) return;
    while ((int64_t)lds_peek(ctl + 1) <= seq) __builtin_amdgcn_s_sleep(1);
  };
  auto post = [&](uint32_t job) -> int64_t {
    if (NT_TS_WS_DBG == 2) return -1;
    while (posted - lds_peek(ctl + 1) >= (uint32_t)kTsRing) __builtin_amdgcn_s_sleep(1);
    ctl[4 + posted % kTsRing] = job;
    lds_publish_wait();  // the job's rows and its ring entry are in LDS
    lds_put(ctl, ++posted);
    return (int64_t)posted - 1;
  };
  const uint32_t sel2 = (lane & 2) ? 0x03020706u : 0x05040100u;
  const uint32_t sel1 = (lane & 1) ? 0x03070105u : 0x06020400u;
  const int ms = lane & (NT_BUNDLE - 1), mh = lane >> 5;
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
  int bi = 0;  // bundles this walker has taken (slot buffer bi & 1)
  for (uint64_t b = claim(); b < nb; b = claim(), ++bi) {
    const int sb = bi & 1;
    wait_done(buf_job[sb]);  // the writer is done with the bundle that used this slot buffer
    TSlot* sl = R.sl(sb);
    uint32_t n_max;
    {
      const uint32_t r = B.bnd_read[b * NT_BUNDLE + (lane & 31)];
      const bool o = r != 0xFFFFFFFFu;
      const uint32_t len = o ? B.len[r] : 0u;
      const uint64_t wo = o ? B.win_off[r] : 0ull;
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
        t.pad = 0u;
        sl[lane] = t;
      }
      n_max = (uint32_t)__builtin_amdgcn_readfirstlane((int)len);  // slot 0 = the longest
    }
    const int nblk = ((int)n_max + kL - 1) / kL;
    const int nst = (nblk + kWave - 1) / kWave;
    const uint64_t g0 = uniform_u64(B.bnd_stripe[b]), g1 = uniform_u64(B.bnd_stripe[b + 1]);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(B.tplanes) + g0 * (uint64_t)kT * kWave * 4, (short)0,
        (int)((g1 - g0) * (uint64_t)kT * kWave * 16), 0x00020000);
    wave_sync();
    TWalker<TP, Pats, Tvrs> wk;
    wk.rs = rs;
    wk.set_stripe(0, lane, lane < nblk);
    if (NT_TS_XPRIME) wk.prime();
    for (int st = 0; st < nst; ++st) {
      const int k = st * kWave + lane;
      if (!NT_TS_XPRIME) wk.prime();
      uint32_t acc[3][8];
      wk.walk(k == 0, acc);
      wk.set_stripe(st + 1, lane, k + kWave < nblk);
      const TSlot& mt = sl[ms];
      const int m_nw = (int)mt.nw;
      const int k0 = st * kWave + 32 * mh;
      const int nv = m_nw - k0 < 0 ? 0 : (m_nw - k0 > 32 ? 32 : m_nw - k0);
      const int fs = st % Aux::kF;
      if ((st & 1) == 0) wait_done(cnt_job);  // a new stripe pair: the last pair's rows are stored
      if (fs == 0) wait_done(flush_job);      // a new flush group: the last group's words are stored
      const bool last = st == nst - 1;
#pragma unroll
      for (int p = 0; p < kNP; ++p) {
        uint32_t* ctp = ct + p * NT_BUNDLE * 32;
        const int half = (st & 1) * 16;
        uint32_t W[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) W[t] = acc[p][t];
        uint32_t ge = ~0u;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const uint32_t tm = ((thr_full >> t) & 1u) ? ~0u : 0u;
          ge = (W[t] & ge) | (~tm & (W[t] | ge));
        }
        if (thr_full > 255u) ge = 0u;
        transpose8(W);
#pragma unroll
        for (int j = 0; j < 8; ++j) W[j] = quad_byte_transpose(W[j], sel2, sel1);
#pragma unroll
        for (int j = 0; j < 8; ++j) ctp[(8 * (lane & 3) + j) * 32 + half + (lane >> 2)] = W[j];
        const uint32_t tb = half_bit_transpose(ge, lane) & (nv >= 32 ? ~0u : ((1u << nv) - 1u));
        tmb[((p * NT_BUNDLE + ms) * Aux::kF + fs) * 2 + mh] = tb;
        wave_sync();
        const uint4 va = *reinterpret_cast<const uint4*>(ctp + ms * 32 + half + 8 * mh);
        const uint4 vb = *reinterpret_cast<const uint4*>(ctp + ms * 32 + half + 8 * mh + 4);
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
        const uint32_t other = (uint32_t)__shfl_xor((int)mine, 32, kWave);
        const uint32_t run = mt.run[p];
        const uint32_t c0 = run + (mh ? other : 0u);
        uint32_t* ckr = ckb + (p * NT_BUNDLE + ms) * 4 * Aux::kF + 4 * fs + 2 * mh;
        ckr[0] = c0;
        ckr[1] = c0 + ga;
        if (last && mh)  // the read's total when its windows end with this stripe
          R.tot()[p * NT_BUNDLE + ms] = 16 * ((k0 >> 4) + 2) == m_nw ? c0 + mine : 0xFFFFFFFFu;
        wave_sync();
        if (mh == 0) sl[ms].run[p] = run + mine + other;
      }
      if ((st & 1) || last) cnt_job = post(kJobCnt | ((uint32_t)sb << 2) | ((uint32_t)st << 10));
      if (fs == Aux::kF - 1 || last) {
        flush_job = post(kJobFlush | ((uint32_t)sb << 2) | ((last ? 1u : 0u) << 3) | ((uint32_t)fs << 4) |
                         ((uint32_t)st << 10));
      }
      buf_job[sb] = (int64_t)posted - 1;
      wave_sync();
    }
    wave_sync();
  }
  lds_publish_wait();
  lds_put(ctl + 2, 1u);  // finished (after the last job was posted)
}

// The bundle scan with walker / writer waves: 5 waves a workgroup.
template <class TP, class Pats, class Tvrs>
__device__ __forceinline__ void tscan_bundles_ws(const NtBatch& B, const NtOut& O, uint64_t* __restrict__ tmask,
                                                 unsigned long long* __restrict__ queue, uint32_t thr_full,
                                                 uint32_t* lds) {
  constexpr int kNP = TP::kNP;
  const int wv = threadIdx.x >> 6;
  if (threadIdx.x < 4 * kTsCtl) lds[4 * ts_ws_walker_words<kNP>() + threadIdx.x] = 0u;  // control words
  __syncthreads();
  if (wv < 4) ts_walker<TP, Pats, Tvrs>(B, tmask, queue, thr_full, lds, wv);
  else ts_writer<kNP>(O, tmask, lds);
}
}  // namespace nt
