// nt_scan.h -- the streaming scan of the NanoTel hot path on gfx950.
//
// Computes, per read and pass (P1 exact, P2 <= 1 mismatch, P3 = P2 U exact
// TVR matches), the covered-base count of every subseq_length window
// (analyze_subtelos / get_density_iranges / get_sub_density, NanoTel.R:
// 717-766, 308-397, 449-468), the telomeric-window bitmask (class -5,
// NanoTel.R:749-758) and the matchPattern hit counts.
//
// Compiled twice: ahead of time (nt_kernels.hip) with the pattern set read
// from NtProgram at run time, and at nt_compile() time through hiprtc
// (nt_jit.cpp) with the pattern set baked in as compile-time truth tables, so
// that every letter test is one v_bitop3 and identical letter tests and
// shifts are shared across letters and patterns.
//
// Work split: one wave per read (grid-stride), the read cut into 64-base
// SEGMENTS (two 32-base words A, B = one 16-byte load of the bit planes).
// Chunk c of a read covers segments g0 = 63c - 1 ... g0 + 63: lane l holds
// segment g0 + l; lanes 0..62 OWN theirs, lane 63 only lends its letter
// tests to lane 62 (the matches starting in a segment read up to m-1 bases
// into the next one).  Chunk 0 starts at segment -1 so that Biostrings'
// out-of-bound start (-1, one mismatch) is an ordinary hit of lane 0.
//
// Neighbour data moves with wave-wide DPP (wave_shl:1 / wave_shr:1); the
// coverage a segment spills into the next one ("overflow") travels right
// the same way, lane 62's overflow is carried into the next chunk's lane 0.
// Window counts: the per-lane covered-base counts of passes 0 and 1 are
// packed into one u32 (16+16 bit), prefix-summed across the wave with DPP
// row_shr / row_bcast, and the lane holding a window boundary kL stores the
// running count there (cum[k]); count(window k) = cum[k+1] - cum[k].  No
// atomics, no zero-fill: every boundary belongs to exactly one owned lane.
#pragma once
#include "nt_common.h"
#include "nt_device.h"

namespace nt {

// floor(p / L), 0 <= p < 2^31 (multiply-shift, exact; see nt_compile)
struct DivL {
  uint32_t m, s;
};
__device__ __forceinline__ int div_l(DivL d, int p) {
  if (d.m == 0u) return p;  // L == 1
  return (int)(__umulhi((uint32_t)p, d.m) >> d.s);
}
__device__ __forceinline__ int div_l(const NtProgram* prog, int p) {
  return div_l(DivL{prog->div32_m, prog->div32_s}, p);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-read auxiliary block of the scan for the calling kernel, in uint64
// units from aux_base(): the telomeric-window bitmasks (pass p at p * nmw,
// nmw = ceil(nw / 64)), then the running covered-base counts at every 16th
// window boundary as uint32 (pass p at p * nck, nck = nw / 16 + 1):
// cnt16[p][j] = covered bases before window 16 j.  With R = the read's rows /
// 64 (win_off is a prefix sum of rows, multiples of 64) the block needs <=
// np (3 R + 1) words and gets 8 np (R + 2): the blocks start 128-byte aligned
// for np = 2 (64 with 3 passes), so the bundle scan's flush of a read's block
// writes whole lines, not pieces of lines its neighbours write.
__device__ __forceinline__ uint64_t aux_base(uint64_t win_off, uint64_t r, int np) {
  return ((win_off >> 6) + 2 * r) * 8 * (uint64_t)np;
}
__device__ __forceinline__ int aux_nmw(int nw) { return (nw + 63) >> 6; }
__device__ __forceinline__ int aux_nck(int nw) { return (nw >> 4) + 1; }

// ISA reading aid (tools/jit_isa.sh builds with -DNT_ISA_MARKS)
#ifdef NT_ISA_MARKS
#define NT_MARK(s) asm volatile("; " s)
#else
#define NT_MARK(s)
#endif

template <int I>
struct IC {
  static constexpr int value = I;
};
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IC<I>{});
    static_for<I + 1, N>(f);
  }
}

// ------------------------------------------------------------------ DPP

constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i+1
constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i-1
constexpr int kDppRowShr = 0x110;    // + n: row_shr:n
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

// lane i <- lane i+1 (lane 63 <- 0: bound_ctrl, one v_mov_b32_dpp)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppWaveShl1, 0xf, 0xf, true);
}
// lane i <- lane i-1 (lane 0 <- lane0)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t lane0) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)lane0, (int)v, kDppWaveShr1, 0xf, 0xf, false);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xf, false);
}
// 32x32 bit transpose inside each half wave: lane 32 h + s gets bit s of the
// half's lanes (bit i from lane 32 h + i) -- five butterfly exchanges (lane ^
// 16 by v_permlane16_swap, ^ 8 / ^ 2 / ^ 1 by DPP, ^ 4 by two DPP shifts),
// each merged with one rotate and one bit-field select whose per-lane
// operands (BitTr) are set once.
struct BitTr {
  uint32_t rot[5], keep[5];  // stage J = 16 >> i: rotate right by rot, keep the own bits in keep
  __device__ __forceinline__ explicit BitTr(int lane) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int J = 16 >> i;
      const uint32_t M = i == 0 ? 0x0000FFFFu : i == 1 ? 0x00FF00FFu : i == 2 ? 0x0F0F0F0Fu : i == 3 ? 0x33333333u : 0x55555555u;
      const bool hi = (lane & J) != 0;
      rot[i] = hi ? (uint32_t)J : (uint32_t)(32 - J);
      keep[i] = hi ? ~M : M;
    }
  }
};
__device__ __forceinline__ uint32_t half_bit_transpose(uint32_t a, int lane, const BitTr& bt) {
  uint32_t pv;
  {
    const auto r = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    pv = (lane & 16) ? r[0] : r[1];
  }
  a = (bt.keep[0] & a) | (~bt.keep[0] & __builtin_amdgcn_alignbit(pv, pv, bt.rot[0]));
  pv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x128, 0xf, 0xf, false);  // row_ror:8 = lane ^ 8
  a = (bt.keep[1] & a) | (~bt.keep[1] & __builtin_amdgcn_alignbit(pv, pv, bt.rot[1]));
  {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x104, 0xf, 0xf, false);  // row_shl:4: lane + 4
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x114, 0xf, 0xf, false);  // row_shr:4: lane - 4
    pv = (lane & 4) ? dn : up;
  }
  a = (bt.keep[2] & a) | (~bt.keep[2] & __builtin_amdgcn_alignbit(pv, pv, bt.rot[2]));
  pv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x4E, 0xf, 0xf, false);  // quad_perm 2301: lane ^ 2
  a = (bt.keep[3] & a) | (~bt.keep[3] & __builtin_amdgcn_alignbit(pv, pv, bt.rot[3]));
  pv = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0xB1, 0xf, 0xf, false);  // quad_perm 1032: lane ^ 1
  a = (bt.keep[4] & a) | (~bt.keep[4] & __builtin_amdgcn_alignbit(pv, pv, bt.rot[4]));
  return a;
}
__device__ __forceinline__ uint32_t half_bit_transpose(uint32_t a, int lane) {
  return half_bit_transpose(a, lane, BitTr(lane));
}

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += dpp0<kDppRowShr + 1, 0xf>(v);
  v += dpp0<kDppRowShr + 2, 0xf>(v);
  v += dpp0<kDppRowShr + 4, 0xf>(v);
  v += dpp0<kDppRowShr + 8, 0xf>(v);
  v += dpp0<kDppRowBcast15, 0xa>(v);
  v += dpp0<kDppRowBcast31, 0xc>(v);
  return v;
}

// ------------------------------------------------------ letter tests

// Bit i of the result: base (L_i, H_i) (A=00 C=01 G=10 T=11, H:L) is in the
// 4-bit set tt (bit c = base c).  tt constant -> one v_bitop3 (or nothing).
__device__ __forceinline__ uint32_t tt_test(int tt, uint32_t L, uint32_t H) {
  switch (tt & 15) {
    case 0: return 0u;
    case 1: return ~(L | H);    // A
    case 2: return L & ~H;      // C
    case 3: return ~H;          // M = A|C
    case 4: return ~L & H;      // G
    case 5: return ~L;          // R = A|G
    case 6: return L ^ H;       // S = C|G
    case 7: return ~(L & H);    // V = A|C|G
    case 8: return L & H;       // T
    case 9: return ~(L ^ H);    // W = A|T
    case 10: return L;          // Y = C|T
    case 11: return L | ~H;     // H = A|C|T
    case 12: return H;          // K = G|T
    case 13: return ~L | H;     // D = A|G|T
    case 14: return L | H;      // B = C|G|T
    default: return 0xFFFFFFFFu;  // N
  }
}

// Pattern descriptors: kM (compile-time length, 0 = run time), m(), and
// E(j, L, H) = letter j of the pattern tested against the 32 bases (L, H).
// Run-time one-hot letters: (L ^ xl) & (H ^ xh), two VALU ops.
template <int M>
struct RtOneHot {
  static constexpr int kM = M;
  const NtPat* P;
  __device__ __forceinline__ int m() const { return M > 0 ? M : P->m; }
  __device__ __forceinline__ uint32_t E(int j, uint32_t L, uint32_t H) const {
    return (L ^ P->xl[j]) & (H ^ P->xh[j]);
  }
};
// Run-time IUPAC letters (scan semantics): truth table as bit-select masks.
template <int M>
struct RtTable {
  static constexpr int kM = M;
  const NtPat* P;
  __device__ __forceinline__ int m() const { return M > 0 ? M : P->m; }
  __device__ __forceinline__ uint32_t E(int j, uint32_t L, uint32_t H) const {
    const uint32_t* t = P->tm_scan[j];
    return bfi(H, bfi(L, t[3], t[2]), bfi(L, t[1], t[0]));
  }
};

__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
  return (a & b) | (a & c) | (b & c);  // v_bitop3 0xe8
}

// a0 = AND of the kM letter words (exact), a1 = at most one zero (<= 1
// mismatch): three letters at a time -- all-3 and at-least-2-of-3 per group,
// then a1 = (a1 & all) | (a0 & two), a0 &= all.
template <int kM, bool kExact>
__device__ __forceinline__ void combine(const uint32_t* q, uint32_t& a0, uint32_t& a1) {
  uint32_t x0 = q[0], x1 = 0xFFFFFFFFu;
  if constexpr (kExact) {
#pragma unroll
    for (int j = 1; j < kM; ++j) x0 &= q[j];
    a0 = x0;
    a1 = 0u;
    return;
  }
  int j = 1;
  if constexpr (kM >= 3) {
    x0 = q[0] & q[1] & q[2];
    x1 = maj3(q[0], q[1], q[2]);
    j = 3;
  } else if constexpr (kM == 2) {
    x0 = q[0] & q[1];
    x1 = q[0] | q[1];
    j = 2;
  }
#pragma unroll
  for (; j + 3 <= kM; j += 3) {
    const uint32_t all = q[j] & q[j + 1] & q[j + 2], two = maj3(q[j], q[j + 1], q[j + 2]);
    x1 = (x1 & all) | (x0 & two);
    x0 &= all;
  }
  if constexpr (kM >= 3 && kM % 3 == 2) {
    const uint32_t all = q[kM - 2] & q[kM - 1], one = q[kM - 2] | q[kM - 1];
    x1 = (x1 & all) | (x0 & one);
    x0 &= all;
  } else if constexpr (kM >= 3 && kM % 3 == 1) {
    x1 = (x1 & q[kM - 1]) | x0;
    x0 &= q[kM - 1];
  }
  a0 = x0;
  a1 = x1;
}

// Planes and validity of one segment (word A, word B).
struct Seg {
  uint32_t LA, HA, LB, HB;
  uint32_t VA, VB;  // positions inside the read (kValid chunks only)
};

// Hits of pattern d at the 64 starts of the segment: a0 exact, a1 <= 1
// mismatch (matchPattern max.mismatch 0 / 1; letters outside the read are
// mismatches).  Letter tests are made on the unshifted words and shifted by
// j (v_alignbit); the next segment's word-A tests come from lane+1 by DPP,
// and for letters j >= 32 (TVRs of 33..64 letters) its word-B tests too.
template <bool kValid, bool kExact, class D>
__device__ __forceinline__ void seg_hits(const D& d, const Seg& s, uint32_t& a0A, uint32_t& a1A,
                                         uint32_t& a0B, uint32_t& a1B) {
  constexpr int kM = D::kM;
  auto q = [&](int j, uint32_t& qA, uint32_t& qB) {
    uint32_t eA = d.E(j, s.LA, s.HA), eB = d.E(j, s.LB, s.HB);
    if (kValid) {
      eA &= s.VA;
      eB &= s.VB;
    }
    const uint32_t eN = from_next_lane(eA);
    if (j < 32) {
      qA = funnel(eB, eA, (uint32_t)j);
      qB = funnel(eN, eB, (uint32_t)j);
    } else {
      const uint32_t eNB = from_next_lane(eB);
      qA = funnel(eN, eB, (uint32_t)(j - 32));
      qB = funnel(eNB, eN, (uint32_t)(j - 32));
    }
  };
  if constexpr (kM > 0) {
    uint32_t qa[kM], qb[kM];
#pragma unroll
    for (int j = 0; j < kM; ++j) q(j, qa[j], qb[j]);
    combine<kM, kExact>(qa, a0A, a1A);
    combine<kM, kExact>(qb, a0B, a1B);
  } else {
    uint32_t x0A = 0xFFFFFFFFu, x1A = 0xFFFFFFFFu, x0B = 0xFFFFFFFFu, x1B = 0xFFFFFFFFu;
    const int m = d.m();
    for (int j = 0; j < m; ++j) {
      uint32_t qA, qB;
      q(j, qA, qB);
      x1A = (x1A & qA) | x0A;
      x0A &= qA;
      x1B = (x1B & qB) | x0B;
      x0B &= qB;
    }
    a0A = x0A;
    a1A = kExact ? 0u : x1A;
    a0B = x0B;
    a1B = kExact ? 0u : x1B;
  }
  if (kValid && !kExact && d.m() <= 1) {  // m <= k: no out-of-bound starts
    a1A &= s.VA;
    a1B &= s.VB;
  }
}

// OR into (cA, cB, ov) the coverage of hit starts hA (word A) and hB (word
// B): bit i covered iff a start in [i-m+1, i] (trim + IRanges::reduce).
// ov = coverage spilling into the next segment's word A, ovB (m > 32 only:
// TVRs) into its word B.  kM > 0: span doubling on the 96-bit value (ov:B:A),
// 128-bit (ovB:ov:B:A) for kM > 32.
template <int kM>
__device__ __forceinline__ void seg_spread(uint32_t hA, uint32_t hB, int m, uint32_t& cA,
                                           uint32_t& cB, uint32_t& ov, uint32_t& ovB) {
  if constexpr (kM > 32) {
    uint32_t w0 = hA, w1 = hB, w2 = 0u, w3 = 0u;
#pragma unroll
    for (int s = 1; s < kM;) {
      const int t = 2 * s <= kM ? s : kM - s;  // <= 32
      w3 |= funnel(w3, w2, (uint32_t)(32 - t));
      w2 |= funnel(w2, w1, (uint32_t)(32 - t));
      w1 |= funnel(w1, w0, (uint32_t)(32 - t));
      if (t < 32) w0 |= w0 << t;
      s += t;
    }
    cA |= w0;
    cB |= w1;
    ov |= w2;
    ovB |= w3;
  } else if constexpr (kM > 0) {
    uint32_t w0 = hA, w1 = hB, w2 = 0u;
#pragma unroll
    for (int s = 1; s < kM;) {
      const int t = 2 * s <= kM ? s : kM - s;
      w2 |= funnel(w2, w1, (uint32_t)(32 - t));
      w1 |= funnel(w1, w0, (uint32_t)(32 - t));
      w0 |= w0 << t;
      s += t;
    }
    cA |= w0;
    cB |= w1;
    ov |= w2;
  } else if (m > 32) {
    const uint64_t v = (uint64_t)hA | ((uint64_t)hB << 32);
    uint64_t lo = v, hi = 0ull;
    for (int j = 1; j < m; ++j) {
      lo |= v << j;
      hi |= v >> (64 - j);
    }
    cA |= (uint32_t)lo;
    cB |= (uint32_t)(lo >> 32);
    ov |= (uint32_t)hi;
    ovB |= (uint32_t)(hi >> 32);
  } else {
    cA |= hA;
    cB |= hB;
    for (int j = 1; j < m; ++j) {
      cA |= hA << j;
      cB |= funnel(hB, hA, (uint32_t)(32 - j));
      ov |= hB >> (32 - j);
    }
  }
}

// ------------------------------------------------------ pattern sets

// Pattern-set policies: passes, hit counters and a visitor over the patterns
// (f(index, descriptor)) and the TVRs.
// kRegHits: hit counters in registers (else per-lane LDS/global slots).
// Hit counter layout (per read): [exact per pattern][<=1 mismatch per
// pattern][exact per TVR] (nt_program_info.n_hits = 2*n_pat + n_tvr).
template <class D>
struct SingleSet {  // --patterns with one unique pattern, no TVRs
  static constexpr bool kRegHits = true;
  static constexpr int kNPat = 1;
  static constexpr int kNHits = 2;
  static constexpr int kNPass = 2;  // 0 = read from the program
  static constexpr bool kLongTvr = false;  // TVRs of > 32 letters possible (a second carry word)
  template <class F>
  __device__ __forceinline__ static void for_pat(const NtProgram* prog, F&& f) {
    f(0, D{&prog->pat[0]});
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr(const NtProgram*, F&&) {}
};

struct GenericSet {  // any program: run-time lists
  static constexpr bool kRegHits = false;
  static constexpr int kNPat = 0;
  static constexpr int kNHits = 1;
  static constexpr int kNPass = 0;
  static constexpr bool kLongTvr = true;
  template <class F>
  __device__ __forceinline__ static void for_pat(const NtProgram* prog, F&& f) {
    for (int p = 0; p < prog->n_pat; ++p) f(p, RtTable<0>{&prog->pat[p]});
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr(const NtProgram* prog, F&& f) {
    for (int t = 0; t < prog->n_tvr; ++t) f(t, RtTable<0>{&prog->tvr[t]});
  }
};

// Compile-time pattern (JIT): the host generates JitPat<...> lists.
template <int M, int... TT>
struct CtPat {
  static constexpr int kM = M;
  static constexpr int kTT[sizeof...(TT)] = {TT...};  // letter truth tables (nt_tscan.h)
  const NtPat* P;  // run-time twin (exception fix-ups)
  __device__ __forceinline__ int m() const { return M; }
  __device__ __forceinline__ uint32_t E(int j, uint32_t L, uint32_t H) const {
    constexpr int tt[] = {TT...};
    return tt_test(tt[j], L, H);
  }
};
template <class... P>
struct CtList {
  static constexpr int kN = sizeof...(P);
};
// Longest pattern of a compile-time list (0 for an empty one).
template <class List>
struct CtMaxM {
  static constexpr int value = 0;
};
template <class H, class... T>
struct CtMaxM<CtList<H, T...>> {
  static constexpr int kRest = CtMaxM<CtList<T...>>::value;
  static constexpr int value = H::kM > kRest ? H::kM : kRest;
};
template <int I, class Head, class... Tail>
struct CtAt {
  using type = typename CtAt<I - 1, Tail...>::type;
};
template <class Head, class... Tail>
struct CtAt<0, Head, Tail...> {
  using type = Head;
};
template <class List>
struct CtVisit;
template <class... P>
struct CtVisit<CtList<P...>> {
  template <class F>
  __device__ __forceinline__ static void run(const NtPat* base, F&& f) {
    static_for<0, (int)sizeof...(P)>([&](auto i) {
      constexpr int I = decltype(i)::value;
      using D = typename CtAt<I, P...>::type;
      f(I, D{base + I});
    });
  }
};
template <>
struct CtVisit<CtList<>> {
  template <class F>
  __device__ __forceinline__ static void run(const NtPat*, F&&) {}
};

template <class Pats, class Tvrs>
struct CtSet {
  static constexpr int kNPat = Pats::kN, kNTvr = Tvrs::kN;
  static constexpr bool kRegHits = true;
  static constexpr int kNHits = 2 * kNPat + kNTvr;
  static constexpr int kNPass = kNTvr > 0 ? 3 : 2;
  static constexpr bool kLongTvr = CtMaxM<Tvrs>::value > 32;
  template <class F>
  __device__ __forceinline__ static void for_pat(const NtProgram* prog, F&& f) {
    CtVisit<Pats>::run(prog->pat, f);
  }
  template <class F>
  __device__ __forceinline__ static void for_tvr(const NtProgram* prog, F&& f) {
    CtVisit<Tvrs>::run(prog->tvr, f);
  }
};

// ------------------------------------------------------------ the scan

// Segment g of the read (zero outside it).  The load itself is
// unconditional (address clamped into the read's slot) so that the compiler
// keeps the prefetch ring in flight with counted s_waitcnt vmcnt(N).  (The
// zeroing is not needed for correctness -- every use in the edge chunks is
// masked by the position-validity words -- but dropping it measured 6 %
// slower: 3.89 -> 4.11 ms at c50k.)
__device__ __forceinline__ uint4 load_seg(const uint4* __restrict__ seg, int nseg, int g) {
  const int gc = g < 0 ? 0 : (g >= nseg ? nseg - 1 : g);
  const uint4 x = seg[gc];
  const bool ok = (g >= 0) & (g < nseg);
  return make_uint4(ok ? x.x : 0u, ok ? x.y : 0u, ok ? x.z : 0u, ok ? x.w : 0u);
}

// NT_BUFLOAD: segment ring through buffer descriptors (range-checked loads);
// NT_RING3: three ring slots, unrolled (1M x 50 kb: scan 3.76 -> 3.52 ms
// with both).  0 selects the plain-load / rotating-ring forms (tuning).
#ifndef NT_BUFLOAD
#define NT_BUFLOAD 1
#endif
#ifndef NT_RING3
#define NT_RING3 1
#endif
#if NT_BUFLOAD
// The same through a buffer descriptor over the read's segments: the
// hardware range check returns 0 for g outside [0, nseg) (a negative g is a
// huge unsigned offset), so no address clamp and no zeroing VALU.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t seg_rsrc(const void* base, int nseg) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           __builtin_amdgcn_readfirstlane(nseg * 16), 0x00020000);
}
__device__ __forceinline__ uint4 load_segb(__amdgpu_buffer_rsrc_t r, int g) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, g * 16, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
#endif

// NT_DBG_CHECK (debugging aid, off): every HBM address the scan forms is
// checked against the limits in a DbgRec the host passes as gscr (planes in
// 16-byte segments, window counts, aux words); a violation is recorded (the
// first one in full) and the access skipped.
#ifndef NT_DBG_CHECK
#define NT_DBG_CHECK 0
#endif
struct DbgRec {
  unsigned long long lim[4];
  unsigned long long nbad;
  unsigned long long first[4];  // kind, index, read, limit
};
__device__ __forceinline__ bool dbg_ok(DbgRec* d, int kind, uint64_t idx, uint64_t r) {
  if (!NT_DBG_CHECK || !d || idx < d->lim[kind]) return true;
  if (atomicAdd(&d->nbad, 1ull) == 0ull) {
    d->first[0] = (unsigned long long)kind;
    d->first[1] = idx;
    d->first[2] = r;
    d->first[3] = d->lim[kind];
  }
  return false;
}

template <int kNHits>
struct ScanState {
  uint32_t ov0, ov1, ov2;  // overflow carried into the next chunk's lane 0
  uint32_t ov2b;           // pass 2 overflow into lane 0's word B (TVRs > 32 letters)
  uint32_t T0, T1, T2;     // covered bases before this chunk, per pass
  uint32_t acc[kNHits];    // register hit counters (per lane)
};

// One chunk (lane's segment g = g0 + lane).  kHits: count the matchPattern
// hits (only when the caller asked for them: 6 VALU per chunk otherwise).
template <class S, bool kValid, bool kHits>
__device__ __forceinline__ void scan_chunk(const NtProgram* __restrict__ prog, const ReadCtx& rc,
                                           int g0, int lane, int np, int nw, int L, DivL div,
                                           uint4 cur, uint2* cum01, uint32_t* cum2,
                                           uint32_t* hitacc, ScanState<S::kNHits>& st) {
  NT_MARK("NT_CHUNK_BEGIN");
  const int n = (int)rc.n;
  const int g = g0 + lane, base = 64 * g;
  Seg s;
  s.LA = cur.x;
  s.HA = cur.y;
  s.LB = cur.z;
  s.HB = cur.w;
  s.VA = s.VB = 0xFFFFFFFFu;
  if (kValid) {
    s.VA = range_mask(base, 0, n - 1);
    s.VB = range_mask(base + 32, 0, n - 1);
  }
  const int n_pat = S::kRegHits ? S::kNPat : prog->n_pat;
  uint32_t cA0 = 0u, cB0 = 0u, ov0 = 0u, cA1 = 0u, cB1 = 0u, ov1 = 0u;
  S::for_pat(prog, [&](int p, auto d) {
    uint32_t a0A, a1A, a0B, a1B;
    seg_hits<kValid, false>(d, s, a0A, a1A, a0B, a1B);
    if (rc.n_exc) {
      patch_exceptions(rc, base, 0, n - 1, *d.P, false, a0A, a1A);
      patch_exceptions(rc, base + 32, 0, n - 1, *d.P, false, a0B, a1B);
    }
    // matchPattern hit counts (lane 63's are dropped in the final sum)
    if constexpr (kHits) {
      const uint32_t h0 = __builtin_popcount(a0A) + __builtin_popcount(a0B);
      const uint32_t h1 = __builtin_popcount(a1A) + __builtin_popcount(a1B);
      if constexpr (S::kRegHits) {
        st.acc[p] += h0;
        st.acc[S::kNPat + p] += h1;
      } else {
        hitacc[p * kWave + lane] += h0;
        hitacc[(n_pat + p) * kWave + lane] += h1;
      }
    }
    uint32_t ovx = 0u;  // (patterns are <= 18 letters)
    seg_spread<decltype(d)::kM>(a0A, a0B, d.m(), cA0, cB0, ov0, ovx);
    seg_spread<decltype(d)::kM>(a1A, a1B, d.m(), cA1, cB1, ov1, ovx);
  });
  const bool three = S::kNPass == 3 || (S::kNPass == 0 && np == 3);
  uint32_t cA2 = 0u, cB2 = 0u, ov2 = 0u, ov2b = 0u;
  if (three) {  // P3 = P2 U exact TVR matches
    cA2 = cA1;
    cB2 = cB1;
    ov2 = ov1;
    S::for_tvr(prog, [&](int t, auto d) {
      uint32_t a0A, a1A, a0B, a1B;
      seg_hits<kValid, true>(d, s, a0A, a1A, a0B, a1B);
      if (rc.n_exc) {
        patch_exceptions(rc, base, 0, n - 1, *d.P, false, a0A, a1A);
        patch_exceptions(rc, base + 32, 0, n - 1, *d.P, false, a0B, a1B);
      }
      if constexpr (kHits) {
        const uint32_t h0 = __builtin_popcount(a0A) + __builtin_popcount(a0B);
        if constexpr (S::kRegHits) st.acc[2 * S::kNPat + t] += h0;
        else hitacc[(2 * n_pat + t) * kWave + lane] += h0;
      }
      seg_spread<decltype(d)::kM>(a0A, a0B, d.m(), cA2, cB2, ov2, ov2b);
    });
  }
  // coverage spilled from the previous segment (lane 0: previous chunk's lane 62)
  cA0 |= from_prev_lane(ov0, st.ov0);
  cA1 |= from_prev_lane(ov1, st.ov1);
  st.ov0 = __builtin_amdgcn_readlane(ov0, kWave - 2);
  st.ov1 = __builtin_amdgcn_readlane(ov1, kWave - 2);
  if (three) {
    cA2 |= from_prev_lane(ov2, st.ov2);
    st.ov2 = __builtin_amdgcn_readlane(ov2, kWave - 2);
    if constexpr (S::kLongTvr) {
      cB2 |= from_prev_lane(ov2b, st.ov2b);
      st.ov2b = __builtin_amdgcn_readlane(ov2b, kWave - 2);
    }
  }
  if (kValid) {  // trim to [1, n]
    cA0 &= s.VA;
    cB0 &= s.VB;
    cA1 &= s.VA;
    cB1 &= s.VB;
    cA2 &= s.VA;
    cB2 &= s.VB;
  }
  if (nw <= 0) return;
  // ---- window accounting: packed prefix sum of passes 0 | 1 << 16
  const uint32_t packA = __builtin_popcount(cA0) | (__builtin_popcount(cA1) << 16);
  const uint32_t own = packA + __builtin_popcount(cB0) + (__builtin_popcount(cB1) << 16);
  const uint32_t excl = wave_incl_scan(own) - own;
  uint32_t own2 = 0u, excl2 = 0u;
  if (three) {
    own2 = __builtin_popcount(cA2) + __builtin_popcount(cB2);
    excl2 = wave_incl_scan(own2) - own2;
  }
  // boundary k*L of this segment (o = offset in the segment): running counts
  // of the bases before it go to cum01[k] (passes 0, 1) and cum2[k] (pass 2)
  auto store = [&](int k, int o) {
    const uint32_t t = (1u << (uint32_t)(o & 31)) - 1u;  // v_bfm_b32
    const bool hi = o >= 32;
    const uint32_t w0 = hi ? cB0 : cA0, w1 = hi ? cB1 : cA1;
    const uint32_t v = excl + (hi ? packA : 0u) +
                       (__builtin_popcount(w0 & t) | (__builtin_popcount(w1 & t) << 16));
    cum01[k] = make_uint2(st.T0 + (v & 0xFFFFu), st.T1 + (v >> 16));
    if (three)
      cum2[k] = st.T2 + excl2 + (hi ? __builtin_popcount(cA2) : 0u) + __builtin_popcount((hi ? cB2 : cA2) & t);
  };
  if ((!kValid || g >= 0) && lane < kWave - 1) {
    int k = div_l(div, base + L - 1);  // first window start >= base
    if (L >= 64) {  // at most one boundary per segment
      const int o = k * L - base;
      if (k >= 1 && k < nw && o <= 63) store(k, o);
    } else {
      for (k = k < 1 ? 1 : k; k < nw && k * L - base <= 63; ++k) store(k, k * L - base);
    }
  }
  const uint32_t tot = __builtin_amdgcn_readlane(excl + own, kWave - 2);
  st.T0 += tot & 0xFFFFu;
  st.T1 += tot >> 16;
  if (three) st.T2 += __builtin_amdgcn_readlane(excl2 + own2, kWave - 2);
  NT_MARK("NT_CHUNK_END");
}

// The whole scan of the reads with len in (len_lo, len_hi] (grid-stride, one
// wave per read).  wmem: this wave's LDS (kLds) or global scratch:
// [n_hits][64] hit slots (run-time sets only), then the running window counts
// cum01 (uint2 {pass 0, pass 1} [nw+1]) and cum2 (pass 2 [nw+1]).
#ifndef NT_RING
#define NT_RING 2
#endif
constexpr int kRing = NT_RING;  // prefetch depth in chunks (tuning knob)

#ifndef NT_WOFF_UNIFORM
#define NT_WOFF_UNIFORM 0  // tuning knob (c10k 2 % slower with it)
#endif
struct ReadMeta {
  uint64_t rid;         // read index (B.list[r] or r)
  uint32_t len;
  uint64_t boff, woff;  // block offset (uniform), window offset
  uint32_t e0, e1;      // exception list range (0, 0 without exceptions)
};

// Wave-uniform copy of a 64-bit value.  v_readfirstlane_b32 yields an int:
// each half is kept unsigned before widening (a sign-extended low half once
// turned every block offset >= 2^31 -- reads past ~1.37M x 50 kb -- into a
// wild address).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}

// The per-read metadata, all loads independent (one memory round trip).
__device__ __forceinline__ ReadMeta load_meta(const NtBatch& B, uint64_t i) {
  ReadMeta m;
  const uint64_t r = B.list ? (uint64_t)B.list[i] : i;
  m.rid = r;
  m.len = B.len[r];
  m.boff = uniform_u64(B.blk_off[r]);  // uniform: SGPR base
#if NT_WOFF_UNIFORM
  m.woff = uniform_u64(B.win_off[r]);  // uniform: SGPR bases of the window outputs
#else
  m.woff = B.win_off[r];
#endif
  m.e0 = m.e1 = 0u;
  if (B.exc_off) {
    m.e0 = B.exc_off[r];
    m.e1 = B.exc_off[r + 1];
  }
  return m;
}

template <class S, bool kLds, bool kHits = true>
__device__ __forceinline__ void scan_reads(const NtProgram* __restrict__ prog,
                                           const uint32_t* __restrict__ thr, const NtBatch& B,
                                           const NtOut& O, uint64_t* __restrict__ tmask,
                                           unsigned long long* __restrict__ queue,
                                           uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t* wmem,
                                           DbgRec* dbg = nullptr) {
  const int lane = threadIdx.x & (kWave - 1);
  const int np = S::kNPass ? S::kNPass : prog->n_pass;
  const int nh = S::kRegHits ? S::kNHits : prog->n_hits, L = prog->L;
  uint32_t* hitacc = wmem;
  const int tsz = (int)prog->thr_size;
  const DivL div{prog->div32_m, prog->div32_s};
  const uint32_t thr_full = thr[L < tsz ? L : tsz - 1];

  // Read distribution: 8 queues, one per XCD (blocks are dealt round-robin
  // to the XCDs), each over an eighth of the reads and claimed `claim` reads
  // at a time; a wave whose queue is drained moves on to the next one.  A
  // single device-scope counter serialises near 13 ns per claim across the
  // chip, which bound the scan of short reads (1M x 10 kb: 3.2 ms at 4 reads
  // per claim, 1.18 ms with the 8 queues).  A static round-robin share of
  // the reads before the queues (`nstatic` per wave, tuning) measured slower
  // at every fraction tried (1M x 50 kb: 5.1 ms at 3/4 static, 3.8 ms at 0).
  const uint64_t nR = B.list ? B.n_list : B.n_reads;  // queue positions (list entries)
  const uint64_t W = (uint64_t)gridDim.x * kNWaves;
  const uint64_t w = (uint64_t)blockIdx.x * kNWaves + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint64_t st_n = (uint64_t)nstatic * W < nR ? nstatic : nR / W;
  const uint64_t D0 = st_n * W, Dn = nR - D0;
  const uint64_t kc = claim ? claim : 1u;
  uint32_t qi = blockIdx.x % NT_QUEUES, qtried = 0;
  // next range [lo, hi) of reads from the queues, hi == lo == nR when drained
  auto claim_next = [&](uint64_t& lo, uint64_t& hi) {
    while (qtried < NT_QUEUES) {
      const uint64_t q0 = D0 + Dn * qi / NT_QUEUES, q1 = D0 + Dn * (qi + 1) / NT_QUEUES;
      unsigned long long v = 0;
      if (lane == 0) v = atomicAdd(queue + qi * NT_QUEUE_STRIDE, (unsigned long long)kc);
      const uint64_t o = uniform_u64(v);
      if (o < q1 - q0) {
        lo = q0 + o;
        hi = q1 - q0 - o > kc ? lo + kc : q1;
        return;
      }
      qi = qi + 1 == NT_QUEUES ? 0 : qi + 1;
      ++qtried;
    }
    lo = hi = nR;
  };
  // Read sequence: the current range [aLo, aHi) step aStep and the one
  // claimed ahead [bLo, bHi).  While read r is scanned, the metadata of the next read is
  // already in flight, and the ring's last loads are its first two chunks.
  uint64_t aLo = w, aHi = D0, aStep = W, bLo, bHi;
  if (st_n == 0) {
    claim_next(aLo, aHi);
    aStep = 1;
  }
  claim_next(bLo, bHi);
  uint64_t r = aLo;
  ReadMeta m = r < nR ? load_meta(B, r) : ReadMeta{};
  uint4 nx0 = make_uint4(0u, 0u, 0u, 0u), nx1 = nx0, nx2 = nx0;
  bool ring_ok = false;  // the ring holds chunks 0 and 1 of read r (after the realignment)
#if NT_RING3
  int ring_ph = 2;  // the slot phase the last read ended in
#endif
  while (r < nR) {
    const bool cross = r + aStep >= aHi;
    const uint64_t rn = cross ? bLo : r + aStep;  // next read (>= nR: none)
    ReadMeta mn{};
    if (rn < nR) mn = load_meta(B, rn);
    const bool skip = m.len <= len_lo || m.len > len_hi;
    const bool skip_n = rn >= nR || mn.len <= len_lo || mn.len > len_hi || (mn.boff & 1u);
    if (!skip && (m.boff & 1u)) {  // layout contract: 16-byte aligned segments
      if (lane == 0) O.flags[m.rid] = NT_FLAG_ERR_ALIGN;
    } else if (!skip) {
    const uint32_t n32 = m.len;
    const uint64_t boff = m.boff;
    ReadCtx rc;
    rc.n = n32;
    rc.nblk = (int32_t)((n32 + 31u) >> 5);
    rc.blk = reinterpret_cast<const uint2*>(B.planes) + boff;
#ifdef NT_ISA_NO_EXC  // ISA reading aid only: exception fix-ups compiled out
    rc.n_exc = 0;
#else
    rc.n_exc = (int32_t)(m.e1 - m.e0);
#endif
    rc.exc_pos = B.exc_off ? B.exc_pos + m.e0 : nullptr;
    rc.exc_code = B.exc_off ? B.exc_code + m.e0 : nullptr;
    const int n = (int)n32;
    const int nseg = (n + 63) >> 6;
    const int nw = (int)split_window_count(n, L);
    uint2* cum01 = reinterpret_cast<uint2*>(wmem + (S::kRegHits ? 0 : nh * kWave));
    uint32_t* cum2 = reinterpret_cast<uint32_t*>(cum01 + (nw + 1));
    if (kHits && !S::kRegHits)
      for (int c = 0; c < nh; ++c) hitacc[c * kWave + lane] = 0u;  // per-lane slots

    // ------------------------------------------------------------ scan
    ScanState<S::kNHits> st;
    st.ov0 = st.ov1 = st.ov2 = st.ov2b = 0u;
    st.T0 = st.T1 = st.T2 = 0u;
#pragma unroll
    for (int c = 0; c < S::kNHits; ++c) st.acc[c] = 0u;
    {
      // 2-deep prefetch ring over the chunk stream of this read and the next
      // one: the ring's last two loads of this read are the next read's
      // chunks 0 and 1 (when both reads have >= 2 chunks), so no wave waits
      // on a cold load at a read boundary
      const uint4* seg = reinterpret_cast<const uint4*>(rc.blk);
      const int K = (nseg + kOwned) / kOwned;  // chunks: g0 = -1, 62, ... < nseg
      const uint4* segn = reinterpret_cast<const uint4*>(B.planes) + (mn.boff >> 1);
      const int nsegn = ((int)mn.len + 63) >> 6;
      bool pf = !skip_n && K >= 2 && (nsegn + kOwned) / kOwned >= 2;
      if (NT_DBG_CHECK) {
        if (!dbg_ok(dbg, 0, (boff >> 1) + (uint64_t)(nseg > 0 ? nseg - 1 : 0), r)) break;
        if (pf && !dbg_ok(dbg, 0, (mn.boff >> 1) + (uint64_t)(nsegn - 1), rn)) pf = false;
      }
#if NT_BUFLOAD
      const __amdgpu_buffer_rsrc_t rs = seg_rsrc(seg, nseg);
      const __amdgpu_buffer_rsrc_t rsn = seg_rsrc(segn, pf ? nsegn : 0);
      auto ld = [&](bool own, int g) { return load_segb(own ? rs : rsn, g); };
#else
      auto ld = [&](bool own, int g) { return load_seg(own ? seg : segn, own ? nseg : nsegn, g); };
#endif
      // chunk c of the stream: read the segments of cur, load position c + 2
      // (this read's chunk, or the next read's chunk c + 2 - K) into dst
      auto step = [&](int c, const uint4& cur, uint4& dst) {
        const int g0 = c * kOwned - 1;
        const int t = c + 2;
        const bool own_t = t < K || !pf;
        dst = ld(own_t, (own_t ? g0 + 2 * kOwned : (t - K) * kOwned - 1) + lane);
        if (g0 >= 0 && 64 * (g0 + kWave) <= n)
          scan_chunk<S, false, kHits>(prog, rc, g0, lane, np, nw, L, div, cur, cum01, cum2, hitacc, st);
        else
          scan_chunk<S, true, kHits>(prog, rc, g0, lane, np, nw, L, div, cur, cum01, cum2, hitacc, st);
      };
#if NT_RING3
      // three ring slots, unrolled by three: no register rotation per chunk
      // (moving an in-flight load's registers would wait for it); the slots
      // are realigned once per read, before the next read's first chunk
      if (ring_ph == 0) {
        nx0 = nx1;
        nx1 = nx2;
      } else if (ring_ph == 1) {
        const uint4 t = nx0;
        nx0 = nx2;
        nx1 = t;
      }
      if (!ring_ok) {
        nx0 = ld(true, lane - 1);
        nx1 = ld(true, kOwned - 1 + lane);
      }
      for (int c = 0;;) {
        step(c, nx0, nx2);
        if (++c >= K) { ring_ph = 0; break; }
        step(c, nx1, nx0);
        if (++c >= K) { ring_ph = 1; break; }
        step(c, nx2, nx1);
        if (++c >= K) { ring_ph = 2; break; }
      }
#else
      if (!ring_ok) {
        nx1 = ld(true, lane - 1);
        nx2 = ld(true, kOwned - 1 + lane);
      }
      for (int c = 0; c < K; ++c) {
        const uint4 cur = nx1;
        nx1 = nx2;
        step(c, cur, nx2);
      }
#endif
      ring_ok = pf;
    }
    if (lane == 0 && nw > 0) {
      cum01[0] = make_uint2(0u, 0u);
      cum01[nw] = make_uint2(st.T0, st.T1);
      if (np == 3) {
        cum2[0] = 0u;
        cum2[nw] = st.T2;
      }
    }
    wave_sync();

    // ------------------------------------------------ window outputs
    // the pass rows: uint8 or uint16 counts (prog->cnt8, uniform)
    const bool c8 = prog->cnt8 != 0;
    uint8_t* wout8 = reinterpret_cast<uint8_t*>(O.win_counts) + m.woff * np;
    uint16_t* wout = reinterpret_cast<uint16_t*>(O.win_counts) + m.woff * np;
    const int nr = (int)NT_WIN_ROWS(nw);  // the padded row of a pass
    // telomeric window (class -5) iff !(count / width < min_density) iff
    // count >= thr[width] (exact, host-computed); the last window may be wider
    uint32_t thr_last = thr_full;
    if (nw > 0) {
      const int wl = n - (nw - 1) * L;
      thr_last = thr[wl < tsz ? wl : tsz - 1];
    }
    const int nmw = aux_nmw(nw), nck = aux_nck(nw);
    uint64_t* tmo = tmask + aux_base(m.woff, m.rid, np);
    uint32_t* cko = reinterpret_cast<uint32_t*>(tmo + np * nmw);
    const uint64_t ab = aux_base(m.woff, m.rid, np);
    // passes 0 and 1 together from the packed running counts (one LDS read
    // per window boundary), pass 2 after them
    for (int j = lane; j < nck; j += kWave) {
      const int i = 16 * j;  // i <= nw
      const uint2 c01 = nw == 0 ? make_uint2(0u, 0u) : cum01[i];
      if (dbg_ok(dbg, 2, ab + (uint64_t)(np * nmw) + (uint64_t)(nck + j) / 2, r)) {
        cko[j] = c01.x;
        cko[nck + j] = c01.y;
      }
      if (np == 3 && dbg_ok(dbg, 2, ab + (uint64_t)(np * nmw) + (uint64_t)(2 * nck + j) / 2, r))
        cko[2 * nck + j] = nw == 0 ? 0u : cum2[i];
    }
    // 64 windows per step: counts from the running sums (one ds_read2 per
    // lane), the count stores and one ballot per pass against the full-width
    // threshold; the last window (wider) is re-tested once after its step.
    for (int ch = 0; ch < nmw; ++ch) {
      const int i = ch * 64 + lane;
      const bool ok = i < nw;
      uint32_t c0 = 0u, c1 = 0u, c2 = 0u;
      if (ok) {
        const uint2 a0 = cum01[i], a1 = cum01[i + 1];
        c0 = a1.x - a0.x;
        c1 = a1.y - a0.y;
        if (dbg_ok(dbg, 1, m.woff * np + (uint64_t)(nr + i), r)) {
          if (c8) {
            wout8[i] = (uint8_t)c0;
            wout8[nr + i] = (uint8_t)c1;
          } else {
            wout[i] = (uint16_t)c0;
            wout[nr + i] = (uint16_t)c1;
          }
        }
        if (np == 3) {
          c2 = cum2[i + 1] - cum2[i];
          if (dbg_ok(dbg, 1, m.woff * np + (uint64_t)(2 * nr + i), r)) {
            if (c8) wout8[2 * nr + i] = (uint8_t)c2;
            else wout[2 * nr + i] = (uint16_t)c2;
          }
        }
      }
      // (counts are 0 past the read's windows; the mask only matters for a zero threshold)
      const uint64_t okm = __ballot(ok);
      uint64_t b0 = __ballot(c0 >= thr_full) & okm, b1 = __ballot(c1 >= thr_full) & okm;
      uint64_t b2 = np == 3 ? __ballot(c2 >= thr_full) & okm : 0ull;
      if (ch == nmw - 1 && thr_last != thr_full) {  // the last window: its own width's threshold
        const int ll = (nw - 1) & 63;
        const uint64_t bit = 1ull << ll;
        const uint32_t l0 = (uint32_t)__builtin_amdgcn_readlane((int)c0, ll);
        const uint32_t l1 = (uint32_t)__builtin_amdgcn_readlane((int)c1, ll);
        b0 = (b0 & ~bit) | (l0 >= thr_last ? bit : 0ull);
        b1 = (b1 & ~bit) | (l1 >= thr_last ? bit : 0ull);
        if (np == 3) {
          const uint32_t l2 = (uint32_t)__builtin_amdgcn_readlane((int)c2, ll);
          b2 = (b2 & ~bit) | (l2 >= thr_last ? bit : 0ull);
        }
      }
      if (lane == 0 && dbg_ok(dbg, 2, ab + (uint64_t)((np - 1) * nmw + ch), r)) {
        tmo[ch] = b0;
        tmo[nmw + ch] = b1;
        if (np == 3) tmo[2 * nmw + ch] = b2;
      }
    }
    if (kHits && O.hits) {
      if constexpr (S::kRegHits) {
#pragma unroll
        for (int c = 0; c < S::kNHits; ++c) {
          const uint32_t v = wave_sum_u32(lane < kOwned ? st.acc[c] : 0u);
          if (lane == 0) O.hits[m.rid * (uint64_t)nh + c] = v;
        }
      } else {
        for (int c = 0; c < nh; ++c) {
          const uint32_t v = wave_sum_u32(lane < kOwned ? hitacc[c * kWave + lane] : 0u);
          if (lane == 0) O.hits[m.rid * (uint64_t)nh + c] = v;
        }
      }
    }
    wave_sync();
    }  // scanned read
    if (skip || (m.boff & 1u)) ring_ok = false;
    if (cross) {
      aLo = bLo;
      aHi = bHi;
      aStep = 1;
      if (aLo < nR) claim_next(bLo, bHi);
    }
    r = rn;
    m = mn;
  }
}

}  // namespace nt
