// nt_pack.cpp -- the host-only half of the C-ABI (no HIP): pattern parsing and
// the program (A1, extract_patterns NanoTel.R:2322-2334), the 2-bit packer
// with the reverse complement fused (A14, NanoTel.R:2219-2221), serials and row order (A15, NanoTel.R:2050-2070,
// 2234-2258), the summary columns (NanoTel.R:1820-1837, 1926-1974) and the
// host twin of the synthetic-read generator.  Built into libnanotel.so and,
// with the reader and the oracle, into the sanitizer test driver
// (tests/san/, AddressSanitizer + UndefinedBehaviorSanitizer).
#include <immintrin.h>

#include <algorithm>
#include <charconv>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "nanotel.h"
#include "nt_common.h"
#include "nt_pack.h"
#include "nt_rng.h"

namespace nt_host {

static inline uint32_t bitrev32(uint32_t x) {
#if defined(__clang__)
  return __builtin_bitreverse32(x);
#else
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
  return __builtin_bswap32(x);
#endif
}

// Biostrings DNA_ALPHABET codes (A=1 C=2 G=4 T=8, IUPAC = OR, '-'=16 '+'=32 '.'=64);
// lower case letters are upper-cased by DNAString().
struct LetterTab {
  uint8_t t[256] = {};
  LetterTab() {
    const char* up = "ACGTMRWSYKVHDBN";
    const uint8_t codes[] = {1, 2, 4, 8, 3, 5, 9, 6, 10, 12, 7, 11, 13, 14, 15};
    for (int i = 0; i < 15; ++i) {
      t[(unsigned char)up[i]] = codes[i];
      t[(unsigned char)(up[i] - 'A' + 'a')] = codes[i];
    }
    t[(unsigned char)'-'] = 16;
    t[(unsigned char)'+'] = 32;
    t[(unsigned char)'.'] = 64;
  }
};
uint8_t letter_code(unsigned char c) {
  static const LetterTab tab;  // thread-safe one-time init (the packer runs on many threads)
  return tab.t[c];
}

// 2-bit code for A/C/G/T (either case), else -1.
inline int base2(unsigned char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
  }
}

inline uint8_t complement_code(uint8_t x) {
  return (uint8_t)((x & 0xF0) | ((x & 1) << 3) | ((x & 8) >> 3) | ((x & 2) << 1) | ((x & 4) >> 1));
}

// 32 bases at a time: the 2-bit code of A/C/G/T (either case) is
// lo = bit1 ^ bit2, hi = bit2 of the ASCII byte (A 0x41 -> 00, C 0x43 -> 01,
// G 0x47 -> 10, T 0x54 -> 11).  pack32 returns false when any of the 32
// bytes is not A/C/G/T; the caller then takes the per-base path (exceptions,
// bad letters).  AVX2 when the host has it (runtime dispatch), else scalar.
__attribute__((target("avx2"))) static bool pack32_avx2(const unsigned char* p, uint32_t& lo,
                                                        uint32_t& hi) {
  const __m256i v = _mm256_loadu_si256((const __m256i*)p);
  const __m256i l = _mm256_or_si256(v, _mm256_set1_epi8(0x20));
  const __m256i ok = _mm256_or_si256(
      _mm256_or_si256(_mm256_cmpeq_epi8(l, _mm256_set1_epi8('a')), _mm256_cmpeq_epi8(l, _mm256_set1_epi8('c'))),
      _mm256_or_si256(_mm256_cmpeq_epi8(l, _mm256_set1_epi8('g')), _mm256_cmpeq_epi8(l, _mm256_set1_epi8('t'))));
  if ((uint32_t)_mm256_movemask_epi8(ok) != 0xFFFFFFFFu) return false;
  const uint32_t b1 = (uint32_t)_mm256_movemask_epi8(_mm256_slli_epi16(v, 6));
  const uint32_t b2 = (uint32_t)_mm256_movemask_epi8(_mm256_slli_epi16(v, 5));
  lo = b1 ^ b2;
  hi = b2;
  return true;
}

static bool pack32_scalar(const unsigned char* p, uint32_t& lo, uint32_t& hi) {
  uint32_t l = 0, h = 0;
  for (int i = 0; i < 32; ++i) {
    const int c = base2(p[i]);
    if (c < 0) return false;
    l |= (uint32_t)(c & 1) << i;
    h |= (uint32_t)(c >> 1) << i;
  }
  lo = l;
  hi = h;
  return true;
}

static const bool g_avx2 = __builtin_cpu_supports("avx2");

inline bool pack32(const unsigned char* p, uint32_t& lo, uint32_t& hi) {
  return g_avx2 ? pack32_avx2(p, lo, hi) : pack32_scalar(p, lo, hi);
}

// number of non-A/C/G/T bytes in s[0, n)
static uint64_t count_non_acgt(const unsigned char* s, uint64_t n) {
  uint64_t e = 0, i = 0;
  uint32_t lo, hi;
  for (; i + 32 <= n; i += 32)
    if (!pack32(s + i, lo, hi))
      for (int k = 0; k < 32; ++k) e += base2(s[i + k]) < 0;
  for (; i < n; ++i) e += base2(s[i]) < 0;
  return e;
}

int64_t window_count(int64_t n, int L) {
  if (n <= 0 || L <= 0) return 0;
  int64_t c = (n - 1) / L + 1;                      // seq(1, n, by = L)
  const int64_t last_start = 1 + (c - 1) * (int64_t)L;
  if ((double)(n - last_start) < (double)L / 2.0) c -= 1;  // NanoTel.R:220
  return c;
}

// 32-base blocks in a read's slot: whole 64-base segments (16-byte loads)


// One token list of --patterns / --tvr_patterns: str_split(x, "\\s+"), as.list
// when > 1 token, unique() (NanoTel.R:2322-2334, 328, 362).
int parse_tokens(const char* s, std::vector<std::string>& uniq, bool& is_list, std::string& err) {
  std::vector<std::string> toks;
  const char* p = s;
  auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; };
  for (;;) {
    const char* b = p;
    while (*p && !ws(*p)) ++p;
    toks.emplace_back(b, p);
    if (!*p) break;
    while (*p && ws(*p)) ++p;
  }
  is_list = toks.size() > 1;
  for (auto& t : toks) {
    if (t.empty()) {
      err = "empty pattern (leading/trailing whitespace in the pattern list)";
      return NT_E_PATTERN;
    }
    if (std::find(uniq.begin(), uniq.end(), t) == uniq.end()) uniq.push_back(t);
  }
  return NT_OK;
}

int build_pat(const std::string& s, int max_m, NtPat& P, std::string& err) {
  if ((int)s.size() > max_m) {
    err = "pattern '" + s + "' is longer than " + std::to_string(max_m) + " letters";
    return max_m == NT_MAX_M ? NT_E_PATTERN : NT_E_LIMIT;
  }
  std::memset(&P, 0, sizeof P);
  P.m = (int32_t)s.size();
  P.fixed = 1;
  for (char ch : s)
    if (std::strchr("WSMKRYBDHVN", ch)) P.fixed = 0;  // uppercase-only regex, NanoTel.R:334
  for (int j = 0; j < P.m; ++j) {
    const uint8_t c = letter_code((unsigned char)s[j]);
    if (!c) {
      err = "pattern '" + s + "' has a letter outside DNA_ALPHABET";
      return NT_E_PATTERN;
    }
    P.code[j] = c;
    uint8_t ts = 0, te = 0;
    for (int b = 0; b < 4; ++b) {
      const uint8_t bc = (uint8_t)(1u << b);
      if (P.fixed ? (c == bc) : ((c & bc) != 0)) ts |= (uint8_t)(1u << b);
      if (c == bc) te |= (uint8_t)(1u << b);
    }
    P.tt_scan[j] = ts;
    P.tt_eq[j] = te;
  }
  return NT_OK;
}


// The program of a parameter set (host only): patterns, passes, the divisor
// magic and the telomeric threshold table.
int make_program(const nt_params* prm, NtProgram& P, std::vector<uint32_t>& thr, std::string& err) {
  if (!prm) return NT_E_ARG;
  if (!prm->patterns) { err = "Missing required parameter:  --patterns"; return NT_E_ARG; }
  if (prm->subseq_length <= 0) { err = "--subseq_length must be >= 1"; return NT_E_ARG; }
  if (prm->subseq_length > 43690)
    { err = "--subseq_length > 43690 overflows the uint16 window counts"; return NT_E_LIMIT; }
  std::memset(&P, 0, sizeof P);
  std::vector<std::string> pats, tvrs;
  bool pat_list = false, tvr_list = false;
  int rc = parse_tokens(prm->patterns, pats, pat_list, err);
  if (rc) return rc;
  if (pats.size() > NT_MAX_PAT) { err = "more than 64 unique patterns"; return NT_E_LIMIT; }
  for (size_t i = 0; i < pats.size(); ++i) {
    rc = build_pat(pats[i], NT_MAX_M, P.pat[i], err);
    if (rc) return rc;
  }
  if (prm->tvr_patterns) {
    rc = parse_tokens(prm->tvr_patterns, tvrs, tvr_list, err);
    if (rc) return rc;
    if (tvrs.size() > NT_MAX_PAT) { err = "more than 64 unique TVR patterns"; return NT_E_LIMIT; }
    for (size_t i = 0; i < tvrs.size(); ++i) {
      rc = build_pat(tvrs[i], NT_MAX_TVR_M, P.tvr[i], err);
      if (rc) return rc;
    }
  }
  P.n_pat = (int32_t)pats.size();
  P.n_tvr = (int32_t)tvrs.size();
  P.n_pass = prm->tvr_patterns ? 3 : 2;
  P.raw_p1 = (!pat_list && P.pat[0].fixed) ? 1 : 0;  // NanoTel.R:347-355
  P.L = prm->subseq_length;
  P.right_edge = prm->check_right_edge ? 1 : 0;
  P.legacy_no_ext = prm->legacy_no_ext ? 1 : 0;
  P.n_hits = 2 * P.n_pat + P.n_tvr;
  P.min_density = prm->min_density;
  // floor(p / L) by multiply-shift: l = ceil(log2 L), M = floor(2^(32+l) / L) + 1
  // is exact for every p < 2^32 (error < 2^-l <= 1/L).
  {
    uint32_t l = 0;
    while ((1ull << l) < (uint64_t)P.L) ++l;
    P.div_s = 32 + l;
    P.div_m = (uint64_t)((((unsigned __int128)1) << (32 + l)) / (uint64_t)P.L) + 1;
    // 32-bit form for p < 2^31: M = floor(2^(31+l) / L) + 1 < 2^32, error < 2^-l <= 1/L
    if (P.L >= 2) {
      const uint64_t m32 = ((1ull << (31 + l)) / (uint64_t)P.L) + 1;
      if (m32 > 0xFFFFFFFFull) { err = "divisor magic overflow"; return NT_E_LIMIT; }
      P.div32_m = (uint32_t)m32;
      P.div32_s = l - 1;
    } else {
      P.div32_m = 0;
      P.div32_s = 0;
    }
  }
  // Telomeric class (NanoTel.R:749-758): -5 iff !(count / width < min_density).
  // fl(c / w) is monotone in c, so the class is count >= thr[w] with thr[w]
  // the smallest such count -- found here with the very fp64 division R does.
  const uint32_t wmax = (uint32_t)P.L + (uint32_t)(P.L + 1) / 2 + 1;
  thr.assign(wmax + 1, 0);
  for (uint32_t w = 1; w <= wmax; ++w) {
    uint32_t c = 0;
    while (c <= w && ((double)c / (double)w < P.min_density)) ++c;
    thr[w] = c;  // w + 1 = never telomeric
  }
  P.thr_size = wmax + 1;
  // 8-bit window counts when every window is under 256 bases: the last window
  // (merged with a short tail by split_telo) is < 1.5 L wide
  P.cnt8 = P.L <= 170 ? 1 : 0;
  P.m_max = 1;
  for (int i = 0; i < P.n_pat + P.n_tvr; ++i) {
    NtPat& X = i < P.n_pat ? P.pat[i] : P.tvr[i - P.n_pat];
    P.m_max = X.m > P.m_max ? X.m : P.m_max;
    for (int j = 0; j < X.m; ++j)
      for (int b = 0; b < 4; ++b) {
        X.tm_scan[j][b] = ((X.tt_scan[j] >> b) & 1u) ? 0xFFFFFFFFu : 0u;
        X.tm_eq[j][b] = ((X.tt_eq[j] >> b) & 1u) ? 0xFFFFFFFFu : 0u;
      }
    X.onehot = 1;
    for (int j = 0; j < X.m; ++j) {
      const uint32_t t = X.tt_scan[j];
      if (t != 1 && t != 2 && t != 4 && t != 8) { X.onehot = 0; continue; }
      const uint32_t c = t == 1 ? 0 : t == 2 ? 1 : t == 4 ? 2 : 3;  // base code l + 2h
      X.xl[j] = (c & 1u) ? 0u : 0xFFFFFFFFu;
      X.xh[j] = (c & 2u) ? 0u : 0xFFFFFFFFu;
    }
  }
  return NT_OK;
}


// The planes of one read (reverse-complemented when rc): 32 bases per step
// on runs of plain bases, per base around anything else.  Non-ACGT letters
// are A in the planes and, when exc_pos is given, listed at exc_pos/exc_code
// (IUPAC code, complemented under rc).  Returns the number of non-ACGT
// letters, or -1 if one is outside DNA_ALPHABET.
int64_t pack_one(const unsigned char* s, uint64_t n, int rc, uint32_t* out, uint32_t* exc_pos,
                        uint8_t* exc_code) {
  int64_t e = 0;
  bool bad = false;
  for (uint64_t blk = 0; blk * 32 < n; ++blk) {
    uint32_t lo = 0, hi = 0;
    if (blk * 32 + 32 <= n) {  // whole block of plain bases: 32 at a time
      // reverse complement: base i of the block is the complement of q[31 - i]
      const unsigned char* q = rc ? s + (n - 32 - blk * 32) : s + blk * 32;
      if (pack32(q, lo, hi)) {
        if (rc) {
          lo = ~bitrev32(lo);
          hi = ~bitrev32(hi);
        }
        out[2 * blk] = lo;
        out[2 * blk + 1] = hi;
        continue;
      }
    }
    for (uint32_t i = 0; i < 32 && blk * 32 + i < n; ++i) {
      const uint64_t pos = blk * 32 + i;
      // reverseComplement: position pos of the RC read is the complement of n-1-pos
      const unsigned char ch = rc ? s[n - 1 - pos] : s[pos];
      int c = base2(ch);
      if (c < 0) {
        uint8_t code = letter_code(ch);
        if (!code) bad = true;
        if (exc_pos && code) {
          exc_pos[e] = (uint32_t)pos;
          exc_code[e] = rc ? complement_code(code) : code;
        }
        ++e;
        c = 0;  // planes hold A at exception positions
      } else if (rc) {
        c = 3 - c;
      }
      lo |= (uint32_t)(c & 1) << i;
      hi |= (uint32_t)((c >> 1) & 1) << i;
    }
    out[2 * blk] = lo;
    out[2 * blk + 1] = hi;
  }
  if ((n + 31) / 32 < read_blocks(n)) {  // zero the pad block of the 64-base segment
    out[2 * ((n + 31) / 32)] = 0u;
    out[2 * ((n + 31) / 32) + 1] = 0u;
  }
  return bad ? -1 : e;
}


NtSynth to_synth(const nt_synth_params* sp) {
  NtSynth S;
  S.seed = sp->seed;
  S.first_read = sp->first_read;
  S.read_len = sp->read_len;
  auto u24 = [](double p) {
    if (!(p > 0)) return 0u;
    if (p >= 1) return 1u << 24;
    return (uint32_t)std::llround(p * 16777216.0);
  };
  S.p_tract_u24 = u24(sp->p_tract);
  S.sub_u24 = u24(sp->sub_rate);
  S.variant_u24 = u24(sp->variant_rate);
  S.tract_min = sp->tract_min;
  S.tract_max = std::max(sp->tract_max, sp->tract_min);
  S.rc_layout = sp->rc_layout;
  return S;
}


// ---- summary.csv number formatting (write_csv of readr 2.1.4, restated:
// parity unpinned beyond Example_output; nanotel_amd/io.py format_double is
// the same rules in Python): NA; Inf / -Inf; integral values below 1e15 as
// integers (or "<digits>e<zeros>" at or above sci_threshold when that is > 0);
// else the shortest round-trip decimal, fixed for exponents -4..15, else
// "<mantissa>e<exponent>" (no '+', no zero padding).
static char* put_double(char* o, double x, double sci_threshold) {
  if (std::isnan(x)) {
    std::memcpy(o, "NA", 2);
    return o + 2;
  }
  if (std::isinf(x)) {
    const char* t = x > 0 ? "Inf" : "-Inf";
    const size_t n = std::strlen(t);
    std::memcpy(o, t, n);
    return o + n;
  }
  if (x == std::floor(x) && std::fabs(x) < 1e15) {
    long long i = (long long)x;
    if (sci_threshold > 0 && (double)std::llabs(i) >= sci_threshold && i % 10 == 0) {
      if (i < 0) *o++ = '-';
      unsigned long long u = (unsigned long long)std::llabs(i);
      int z = 0;
      while (u % 10 == 0) {
        u /= 10;
        ++z;
      }
      o = std::to_chars(o, o + 24, u).ptr;
      *o++ = 'e';
      return std::to_chars(o, o + 8, z).ptr;
    }
    return std::to_chars(o, o + 24, i).ptr;
  }
  char b[40];
  const auto r = std::to_chars(b, b + sizeof b, x, std::chars_format::scientific);  // shortest round trip
  *r.ptr = 0;
  // b = [-]d[.ddd]e(+|-)XX
  const char* p = b;
  if (*p == '-') *o++ = *p++;
  char dig[24];
  int nd = 0;
  while (*p && *p != 'e') {
    if (*p != '.') dig[nd++] = *p;
    ++p;
  }
  const int ex = std::atoi(p + 1);
  if (ex >= -4 && ex < 16) {  // Python repr's fixed range
    if (ex < 0) {
      *o++ = '0';
      *o++ = '.';
      for (int k = 0; k < -ex - 1; ++k) *o++ = '0';
      std::memcpy(o, dig, nd);
      return o + nd;
    }
    for (int k = 0; k <= ex; ++k) *o++ = k < nd ? dig[k] : '0';
    *o++ = '.';
    if (nd > ex + 1) {
      std::memcpy(o, dig + ex + 1, nd - ex - 1);
      return o + (nd - ex - 1);
    }
    *o++ = '0';
    return o;
  }
  *o++ = dig[0];
  if (nd > 1) {
    *o++ = '.';
    std::memcpy(o, dig + 1, nd - 1);
    o += nd - 1;
  }
  *o++ = 'e';
  return std::to_chars(o, o + 8, ex).ptr;
}

static char* put_int(char* o, int32_t v) {
  if (v == NT_NA_INT32) {
    std::memcpy(o, "NA", 2);
    return o + 2;
  }
  return std::to_chars(o, o + 16, v).ptr;
}

// readr's quoting: a field with the delimiter, a quote or a line break is
// quoted, quotes doubled
static char* put_field(char* o, const char* s, uint64_t n) {
  bool q = false;
  for (uint64_t i = 0; i < n && !q; ++i) q = s[i] == ',' || s[i] == '"' || s[i] == '\n' || s[i] == '\r';
  if (!q) {
    std::memcpy(o, s, n);
    return o + n;
  }
  *o++ = '"';
  for (uint64_t i = 0; i < n; ++i) {
    if (s[i] == '"') *o++ = '"';
    *o++ = s[i];
  }
  *o++ = '"';
  return o;
}

}  // namespace nt_host

using namespace nt_host;

extern "C" {

int64_t nt_window_count(int64_t n, int32_t subseq_length) { return window_count(n, subseq_length); }
uint64_t nt_window_rows(int64_t nw) { return nw <= 0 ? 0 : NT_WIN_ROWS((uint64_t)nw); }

uint64_t nt_read_blocks(uint64_t n) { return read_blocks(n); }


int nt_pack_count(const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                  int32_t subseq_length, uint64_t* total_blocks, uint64_t* total_windows,
                  uint64_t* total_exc, uint64_t* max_len, uint64_t* bad_read) {
  if ((!seqs || !lens) && n_reads) return NT_E_ARG;
  std::vector<uint64_t> exc(n_reads, 0);
  std::vector<int> bad(n_reads, 0);
  parallel_for(n_reads, [&](uint64_t r) {
    const unsigned char* s = (const unsigned char*)seqs[r];
    uint64_t e = 0;
    int b = lens[r] == 0 ? 2 : 0;
    uint32_t lo, hi;
    for (uint64_t i = 0; i < lens[r] && !b;) {
      if (i + 32 <= lens[r] && pack32(s + i, lo, hi)) {
        i += 32;
        continue;
      }
      const uint64_t end = std::min<uint64_t>(lens[r], i + 32);
      for (; i < end && !b; ++i) {
        if (base2(s[i]) >= 0) continue;
        if (letter_code(s[i])) ++e; else b = 1;
      }
    }
    exc[r] = e;
    bad[r] = b;
  });
  uint64_t tb = 0, tw = 0, te = 0, ml = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    if (bad[r]) {
      if (bad_read) *bad_read = r;
      return bad[r] == 2 ? NT_E_EMPTY_READ : NT_E_LETTER;
    }
    tb += read_blocks(lens[r]);
    tw += NT_WIN_ROWS((uint64_t)window_count((int64_t)lens[r], subseq_length));
    te += exc[r];
    ml = std::max(ml, lens[r]);
  }
  if (total_blocks) *total_blocks = tb;
  if (total_windows) *total_windows = tw;
  if (total_exc) *total_exc = te;
  if (max_len) *max_len = ml;
  return NT_OK;
}

int nt_pack_reads(const char* const* seqs, const uint64_t* lens, uint64_t n_reads, int32_t rc,
                  int32_t subseq_length, uint32_t* planes, uint64_t* blk_off, uint32_t* len,
                  uint64_t* win_off, uint32_t* exc_off, uint32_t* exc_pos, uint8_t* exc_code) {
  if (n_reads && (!seqs || !lens || !planes || !blk_off || !len || !win_off)) return NT_E_ARG;
  // prefix sums (serial, cheap), then the per-read fill in parallel
  std::vector<uint64_t> eoff(n_reads + 1, 0);
  uint64_t b = 0, w = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    if (lens[r] > 0xFFFFFFFFull) return NT_E_LIMIT;
    blk_off[r] = b;
    win_off[r] = w;
    len[r] = (uint32_t)lens[r];
    b += read_blocks(lens[r]);
    w += NT_WIN_ROWS((uint64_t)window_count((int64_t)lens[r], subseq_length));
  }
  if (exc_off) {
    std::vector<uint64_t> cnt(n_reads, 0);
    parallel_for(n_reads, [&](uint64_t r) {
      const unsigned char* s = (const unsigned char*)seqs[r];
      cnt[r] = count_non_acgt(s, lens[r]);
    });
    for (uint64_t r = 0; r < n_reads; ++r) eoff[r + 1] = eoff[r] + cnt[r];
    for (uint64_t r = 0; r <= n_reads; ++r) {
      if (eoff[r] > 0xFFFFFFFFull) return NT_E_LIMIT;
      exc_off[r] = (uint32_t)eoff[r];
    }
  }
  std::atomic<int> bad{0};
  parallel_for(n_reads, [&](uint64_t r) {
    const int64_t k = pack_one((const unsigned char*)seqs[r], lens[r], rc, planes + 2 * blk_off[r],
                               exc_off ? exc_pos + eoff[r] : nullptr, exc_off ? exc_code + eoff[r] : nullptr);
    if (k < 0 || (k > 0 && !exc_off)) bad.store(1);
  });
  return bad.load() ? NT_E_LETTER : NT_OK;
}


int64_t nt_assign_serials(const uint8_t* is_telo, uint64_t n, double* serial_start_io,
                          double* max_serial_io, double* serial_out, int64_t* order_out) {
  if (!serial_start_io || !max_serial_io || (n && (!is_telo || !serial_out || !order_out)))
    return NT_E_ARG;
  const uint64_t groups = 8;  // groups_length (NanoTel.R:2234)
  const double ss = *serial_start_io;
  double mx = *max_serial_io;
  int64_t rows = 0;
  for (uint64_t j = 0; j < n; ++j) serial_out[j] = std::nan("");
  auto run = [&](uint64_t first, uint64_t stride, double serial) {
    // search_patterns: current_serial advances only on telomeric reads (NanoTel.R:2050-2070)
    for (uint64_t j = first; j < n; j += stride) {
      if (!is_telo[j]) continue;
      serial_out[j] = serial;
      order_out[rows++] = (int64_t)j;
      if (serial > mx) mx = serial;
      serial = serial + 1.0;
    }
  };
  if (n < groups) {
    run(0, 1, ss);  // plan(sequential) (NanoTel.R:2236-2239)
  } else {
    // split(1:n, f = 1:8): group g = reads g, g+8, ...; serial_start of group g is
    // serial_start + number of reads in groups < g (NanoTel.R:2245-2252)
    uint64_t before = 0;
    for (uint64_t g = 0; g < groups; ++g) {
      run(g, groups, (double)before + ss);
      before += (n - g + groups - 1) / groups;
    }
  }
  *max_serial_io = mx;
  *serial_start_io = mx + 1.0;  // max(df_summary$Serial) + 1 (NanoTel.R:2258)
  return rows;
}

int64_t nt_rows_columns(const int32_t* start, const int32_t* end, const double* density,
                        const uint64_t* lens, uint64_t n_reads, int32_t n_pass,
                        const double* serial, const int64_t* order, int64_t rows,
                        double* col_serial, int32_t* col_length, double* col_density,
                        int32_t* col_start, int32_t* col_end, int32_t* col_width) {
  if (rows < 0 || n_pass < 1 || n_pass > NT_MAX_PASS) return NT_E_ARG;
  if (rows == 0) return 0;
  if (!start || !end || !density || !lens || !serial || !order || !col_serial || !col_length ||
      !col_density || !col_start || !col_end || !col_width)
    return NT_E_ARG;
  double na_real;
  const uint64_t na_bits = NT_NA_REAL_BITS;
  std::memcpy(&na_real, &na_bits, sizeof na_real);
  for (int64_t i = 0; i < rows; ++i) {
    const int64_t j = order[i];
    if (j < 0 || (uint64_t)j >= n_reads) return NT_E_ARG;
    if (lens[j] > 0x7FFFFFFFull) return NT_E_LIMIT;
    col_serial[i] = serial[j];
    col_length[i] = (int32_t)lens[j];  // length(current_seq_unlist), integer
    for (int p = 0; p < n_pass; ++p) {
      const int64_t o = (int64_t)p * rows + i;
      const int32_t s = start[3 * j + p], e = end[3 * j + p];
      if (s == -1) {  // start(telo_position) == -1: NA columns (NanoTel.R:1926-1940)
        col_density[o] = na_real;
        col_start[o] = col_end[o] = col_width[o] = NT_NA_INT32;
      } else {
        col_density[o] = density[3 * j + p];
        col_start[o] = s;
        col_end[o] = e;
        col_width[o] = (int32_t)((int64_t)e - s + 1);  // width(IRanges(s, e))
      }
    }
  }
  return rows;
}


int nt_synth_ascii(const nt_synth_params* sp, uint64_t read_index, char* out) {
  if (!sp || !out) return NT_E_ARG;
  const NtSynth S = to_synth(sp);
  const uint64_t r = S.first_read + read_index;
  const NtSynthRead R = nt_synth_read(S, r);
  static const char kBase[4] = {'A', 'C', 'G', 'T'};
  for (uint64_t p = 0; p < S.read_len; ++p) out[p] = kBase[nt_synth_base(S, R, r, p)];
  return NT_OK;
}

}  // extern "C"

extern "C" int64_t nt_rows_csv(const double* col_serial, const int32_t* col_length, const double* col_density,
                               const int32_t* col_start, const int32_t* col_end, const int32_t* col_width,
                               int64_t rows, int32_t n_pass, const char* const* names, const uint64_t* name_lens,
                               double sci_threshold, char* csv_out, uint64_t csv_cap, char* ids_out,
                               uint64_t ids_cap, uint64_t* ids_bytes) {
  if (rows < 0 || n_pass < 1 || n_pass > NT_MAX_PASS || !csv_out) return NT_E_ARG;
  if (rows && (!col_serial || !col_length || !col_density || !col_start || !col_end || !col_width || !names ||
               !name_lens))
    return NT_E_ARG;
  char* o = csv_out;
  char* const oe = csv_out + csv_cap;
  char* d = ids_out;
  for (int64_t i = 0; i < rows; ++i) {
    // room for the longest row this can write: the name quoted and doubled, 3 + 4 n_pass fields
    const uint64_t need = 2 * name_lens[i] + 3 + (uint64_t)(3 + 4 * n_pass) * 40;
    if ((uint64_t)(oe - o) < need) return NT_E_LIMIT;
    o = put_double(o, col_serial[i], sci_threshold);
    *o++ = ',';
    o = put_field(o, names[i], name_lens[i]);
    *o++ = ',';
    o = put_int(o, col_length[i]);
    for (int p = 0; p < n_pass; ++p) {
      const int64_t k = (int64_t)p * rows + i;
      *o++ = ',';
      o = put_double(o, col_density[k], 0.0);  // densities: never the integral sci form
      *o++ = ',';
      o = put_int(o, col_start[k]);
      *o++ = ',';
      o = put_int(o, col_end[k]);
      *o++ = ',';
      o = put_int(o, col_width[k]);
    }
    *o++ = '\n';
    if (ids_out) {
      if ((uint64_t)(d - ids_out) + name_lens[i] + 1 > ids_cap) return NT_E_LIMIT;
      std::memcpy(d, names[i], name_lens[i]);
      d += name_lens[i];
      *d++ = '\n';
    }
  }
  if (ids_bytes) *ids_bytes = ids_out ? (uint64_t)(d - ids_out) : 0;
  return (int64_t)(o - csv_out);
}
