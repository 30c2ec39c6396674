/*
 * nanotel_oracle.c -- CPU restatement of NanoTel's telomere hot path.
 *
 * TEST INFRASTRUCTURE ONLY (the checker; see nanotel_oracle.h).  Never linked
 * into the product.  Every function cites the reference file:line it restates
 * (paths relative to the Tzfatilab/Telomere-Analyzer checkout).
 *
 * Third-party semantics restated here (not vendored in the reference):
 *   Biostrings 2.66.0/2.68.1 (README.md:83; Example_output/log/run.log:8)
 *     matchPattern: start range [1-k, n-m+1+k] (naive-inexact "Pshift"
 *     loop: min_Pshift = m<=k ? 1-m : -k), positions outside the subject count
 *     as mismatches; fixed=TRUE compares letter codes for equality, fixed=FALSE
 *     matches iff (pattern_code & subject_code) != 0 (IUPAC bit sets).
 *   IRanges 2.32.0/2.34.1: trim(views) clips to [1, n]; union(x,y) =
 *     reduce(c(x,y)) merging overlapping AND adjacent ranges; intersect()
 *     works on the reduced sets.
 * Compile with -O2 -ffp-contract=off: every fp64 operation must be the single
 * IEEE operation R performs.
 */
#include "nanotel_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ codes */

uint8_t nto_dna_code(char c) {
  switch (c) {
    case 'A': case 'a': return 1;
    case 'C': case 'c': return 2;
    case 'G': case 'g': return 4;
    case 'T': case 't': return 8;
    case 'M': case 'm': return 3;
    case 'R': case 'r': return 5;
    case 'W': case 'w': return 9;
    case 'S': case 's': return 6;
    case 'Y': case 'y': return 10;
    case 'K': case 'k': return 12;
    case 'V': case 'v': return 7;
    case 'H': case 'h': return 11;
    case 'D': case 'd': return 13;
    case 'B': case 'b': return 14;
    case 'N': case 'n': return 15;
    case '-': return 16;
    case '+': return 32;
    case '.': return 64;
    default: return 0;
  }
}

static uint8_t comp_code(uint8_t x) {
  /* A<->T, C<->G on the bit set; '-', '+', '.' unchanged. */
  return (uint8_t)((x & 0xF0) | ((x & 1) << 3) | ((x & 8) >> 3) | ((x & 2) << 1) |
                   ((x & 4) >> 1));
}

static char code_letter(uint8_t x) {
  static const char* L = "?ACMGRSVTWYHKDBN";
  if (x < 16) return L[x];
  if (x == 16) return '-';
  if (x == 32) return '+';
  if (x == 64) return '.';
  return '?';
}

/* Biostrings::reverseComplement (NanoTel.R:2219-2221). */
int nto_reverse_complement(char* seq, int64_t n) {
  for (int64_t i = 0, j = n - 1; i <= j; i++, j--) {
    uint8_t a = nto_dna_code(seq[i]), b = nto_dna_code(seq[j]);
    if (!a || !b) return NTO_E_BAD_LETTER;
    seq[i] = code_letter(comp_code(b));
    seq[j] = code_letter(comp_code(a));
  }
  return NTO_OK;
}

/* --------------------------------------------------------------- patterns */

typedef struct {
  char str[NTO_MAX_M + 1];
  uint8_t code[NTO_MAX_M];
  int m;
  int fixed; /* !str_detect(pat, "[WSMKRYBDHVN]") -- uppercase only (NanoTel.R:334) */
} pat_t;

struct nto_patterns {
  pat_t pat[NTO_MAX_PAT];
  int n_pat;     /* after unique() */
  int pat_list;  /* length(tokens) > 1 -> as.list (NanoTel.R:2324-2326) */
  pat_t tvr[NTO_MAX_PAT];
  int n_tvr;
  int tvr_list;
  int has_tvr;
};

static int is_ws(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v';
}

/* extract_patterns = compose(unlist, partial(str_split, pattern="\\s+"))
 * (NanoTel.R:2322).  Leading/trailing whitespace yields empty tokens, which
 * matchPattern rejects ("empty pattern"). */
static int parse_list(const char* s, pat_t* out, int* n_out, int* is_list, int max_len) {
  int ntok = 0, nuniq = 0;
  const char* p = s;
  for (;;) {
    const char* b = p;
    while (*p && !is_ws(*p)) p++;
    int len = (int)(p - b);
    ntok++;
    if (len == 0) return NTO_E_EMPTY_PAT;
    if (len > max_len) return NTO_E_PAT_LONG;
    pat_t t;
    memset(&t, 0, sizeof t);
    memcpy(t.str, b, (size_t)len);
    t.m = len;
    t.fixed = 1;
    for (int i = 0; i < len; i++) {
      uint8_t c = nto_dna_code(b[i]);
      if (!c) return NTO_E_BAD_LETTER;
      t.code[i] = c;
      if (strchr("WSMKRYBDHVN", b[i])) t.fixed = 0;
    }
    int dup = 0; /* unique() on the character list (NanoTel.R:328, 362) */
    for (int i = 0; i < nuniq; i++)
      if (strcmp(out[i].str, t.str) == 0) dup = 1;
    if (!dup) {
      if (nuniq >= NTO_MAX_PAT) return NTO_E_ARG;
      out[nuniq++] = t;
    }
    if (!*p) break;
    while (*p && is_ws(*p)) p++;
    /* str_split keeps a trailing empty token after trailing whitespace */
  }
  *n_out = nuniq;
  *is_list = ntok > 1;
  return NTO_OK;
}

nto_patterns* nto_patterns_new(const char* patterns, const char* tvr_patterns, int* err_out) {
  int err = NTO_OK;
  nto_patterns* P = (nto_patterns*)calloc(1, sizeof *P);
  if (!P) { err = NTO_E_NOMEM; goto fail; }
  if (!patterns) { err = NTO_E_ARG; goto fail; }
  /* testit::assert(str_length(pattern) <= subseq_width=18) NanoTel.R:589,647 */
  err = parse_list(patterns, P->pat, &P->n_pat, &P->pat_list, 18);
  if (err) goto fail;
  if (tvr_patterns) {
    P->has_tvr = 1;
    err = parse_list(tvr_patterns, P->tvr, &P->n_tvr, &P->tvr_list, NTO_MAX_M);
    if (err) goto fail;
  }
  if (err_out) *err_out = NTO_OK;
  return P;
fail:
  free(P);
  if (err_out) *err_out = err;
  return NULL;
}

void nto_patterns_free(nto_patterns* p) { free(p); }
int nto_patterns_npass(const nto_patterns* p) { return p->has_tvr ? 3 : 2; }
int nto_patterns_count(const nto_patterns* p, int tvr) { return tvr ? p->n_tvr : p->n_pat; }

/* ------------------------------------------------------------ range lists */

typedef struct { int64_t s, e; } rng; /* 1-based inclusive (IRanges start/end) */
typedef struct { rng* v; int64_t n, cap; } rlist;

static int rl_push(rlist* l, int64_t s, int64_t e) {
  if (l->n == l->cap) {
    int64_t nc = l->cap ? 2 * l->cap : 64;
    rng* nv = (rng*)realloc(l->v, (size_t)nc * sizeof(rng));
    if (!nv) return NTO_E_NOMEM;
    l->v = nv;
    l->cap = nc;
  }
  l->v[l->n].s = s;
  l->v[l->n].e = e;
  l->n++;
  return NTO_OK;
}
static void rl_free(rlist* l) { free(l->v); l->v = NULL; l->n = l->cap = 0; }

static int rng_cmp(const void* a, const void* b) {
  const rng* x = (const rng*)a;
  const rng* y = (const rng*)b;
  if (x->s != y->s) return x->s < y->s ? -1 : 1;
  if (x->e != y->e) return x->e < y->e ? -1 : 1;
  return 0;
}

/* IRanges::reduce: sort, then merge overlapping or adjacent ranges; empty
 * ranges dropped (union() uses drop.empty.ranges=TRUE). */
static void rl_reduce(rlist* l) {
  int64_t w = 0;
  if (l->n > 1) qsort(l->v, (size_t)l->n, sizeof(rng), rng_cmp); /* (qsort of NULL, 0 is UB) */
  for (int64_t i = 0; i < l->n; i++) {
    rng r = l->v[i];
    if (r.e < r.s) continue;
    if (w > 0 && r.s <= l->v[w - 1].e + 1) {
      if (r.e > l->v[w - 1].e) l->v[w - 1].e = r.e;
    } else {
      l->v[w++] = r;
    }
  }
  l->n = w;
}

/* IRanges::union(x, y) = reduce(c(x, y)), result into x. */
static int rl_union(rlist* x, const rlist* y) {
  for (int64_t i = 0; i < y->n; i++) {
    int e = rl_push(x, y->v[i].s, y->v[i].e);
    if (e) return e;
  }
  rl_reduce(x);
  return NTO_OK;
}

/* trim(views): restrict to [1, n] (NanoTel.R:337-339, 351-353, 371-373). */
static void rl_trim(rlist* l, int64_t n) {
  for (int64_t i = 0; i < l->n; i++) {
    if (l->v[i].s < 1) l->v[i].s = 1;
    if (l->v[i].e > n) l->v[i].e = n;
  }
}

/* Reduced, sorted copy with width prefix sums, for intersect() widths. */
typedef struct { rlist red; int64_t* pre; } cover_t;

static int cover_build(cover_t* c, const rlist* ranges) {
  memset(c, 0, sizeof *c);
  for (int64_t i = 0; i < ranges->n; i++) {
    int e = rl_push(&c->red, ranges->v[i].s, ranges->v[i].e);
    if (e) return e;
  }
  rl_reduce(&c->red);
  c->pre = (int64_t*)malloc((size_t)(c->red.n + 1) * sizeof(int64_t));
  if (!c->pre) return NTO_E_NOMEM;
  c->pre[0] = 0;
  for (int64_t i = 0; i < c->red.n; i++)
    c->pre[i + 1] = c->pre[i] + (c->red.v[i].e - c->red.v[i].s + 1);
  return NTO_OK;
}
static void cover_free(cover_t* c) { rl_free(&c->red); free(c->pre); }

/* sum(width(IRanges::intersect(IRanges(a, b), ranges))) */
static int64_t cover_count(const cover_t* c, int64_t a, int64_t b) {
  if (b < a || c->red.n == 0) return 0;
  const rng* v = c->red.v;
  int64_t n = c->red.n;
  /* first range with e >= a */
  int64_t lo = 0, hi = n;
  while (lo < hi) { int64_t mid = (lo + hi) / 2; if (v[mid].e < a) lo = mid + 1; else hi = mid; }
  int64_t i0 = lo;
  /* first range with s > b */
  lo = i0; hi = n;
  while (lo < hi) { int64_t mid = (lo + hi) / 2; if (v[mid].s <= b) lo = mid + 1; else hi = mid; }
  int64_t i1 = lo; /* ranges [i0, i1) overlap */
  if (i1 <= i0) return 0;
  int64_t tot = c->pre[i1] - c->pre[i0];
  if (v[i0].s < a) tot -= a - v[i0].s;
  if (v[i1 - 1].e > b) tot -= v[i1 - 1].e - b;
  return tot;
}

/* get_sub_density (NanoTel.R:449-468): |range ∩ cover| / width(range) */
static double sub_density(const cover_t* c, int64_t s, int64_t e) {
  int64_t w = e - s + 1;
  return (double)cover_count(c, s, e) / (double)w;
}

/* ----------------------------------------------------------- matchPattern */

/* Biostrings naive-inexact / boyer-moore semantics on a code subject. */
static int match_codes(const uint8_t* P, int m, int fixed, const uint8_t* S, int64_t n, int k,
                       rlist* views) {
  int64_t minP = (m <= k) ? 1 - m : -k; /* Pshift, 0-based */
  int64_t maxn2 = n - minP;
  for (int64_t ps = minP; ps + m <= maxn2; ps++) {
    int nmis = 0;
    for (int j = 0; j < m && nmis <= k; j++) {
      int64_t pos = ps + j;
      if (pos < 0 || pos >= n) { nmis++; continue; }
      if (fixed ? (P[j] != S[pos]) : ((P[j] & S[pos]) == 0)) nmis++;
    }
    if (nmis <= k) {
      int e = rl_push(views, ps + 1, ps + m);
      if (e) return e;
    }
  }
  return NTO_OK;
}

int64_t nto_match_pattern(const char* pattern, const char* subject, int64_t n, int k, int fixed,
                          int32_t* starts, int64_t cap) {
  int m = (int)strlen(pattern);
  if (m == 0) return NTO_E_EMPTY_PAT;
  if (m > NTO_MAX_M) return NTO_E_PAT_LONG;
  uint8_t P[NTO_MAX_M];
  for (int i = 0; i < m; i++) {
    P[i] = nto_dna_code(pattern[i]);
    if (!P[i]) return NTO_E_BAD_LETTER;
  }
  uint8_t* S = (uint8_t*)malloc((size_t)(n > 0 ? n : 1));
  if (!S) return NTO_E_NOMEM;
  for (int64_t i = 0; i < n; i++) {
    S[i] = nto_dna_code(subject[i]);
    if (!S[i]) { free(S); return NTO_E_BAD_LETTER; }
  }
  rlist v = {0};
  int e = match_codes(P, m, fixed, S, n, k, &v);
  free(S);
  if (e) { rl_free(&v); return e; }
  if (starts)
    for (int64_t i = 0; i < v.n && i < cap; i++) starts[i] = (int32_t)v.v[i].s;
  int64_t cnt = v.n;
  rl_free(&v);
  return cnt;
}

/* ---------------------------------------------------- get_density_iranges */

/* get_density_iranges (NanoTel.R:308-397).  out = the pass's range set;
 * *raw = 1 when it is the raw (unreduced) view set: single fixed pattern at
 * max.mismatch 0 (NanoTel.R:349-355). hits (optional) = length(matchPattern). */
static int density_iranges(const uint8_t* S, int64_t n, const nto_patterns* P, int with_mismatch,
                           int use_tvr, rlist* out, int* raw, uint32_t* hits_in) {
  int k = with_mismatch ? 1 : 0;
  int e;
  /* hits_in counts the pattern matches, or (use_tvr) the TVR matches */
  uint32_t* hits = use_tvr ? NULL : hits_in;
  uint32_t* tvr_hits = use_tvr ? hits_in : NULL;
  *raw = 0;
  out->n = 0;
  if (P->pat_list) {
    for (int i = 0; i < P->n_pat; i++) {
      const pat_t* p = &P->pat[i];
      rlist cur = {0};
      e = match_codes(p->code, p->m, p->fixed, S, n, k, &cur);
      if (!e && hits) hits[i] = (uint32_t)cur.n;
      if (!e && (!p->fixed || k > 0)) rl_trim(&cur, n);
      if (!e) e = rl_union(out, &cur);
      rl_free(&cur);
      if (e) return e;
    }
    rl_reduce(out); /* union(mp_all, mp_all) NanoTel.R:345 */
  } else {
    const pat_t* p = &P->pat[0];
    e = match_codes(p->code, p->m, p->fixed, S, n, k, out);
    if (e) return e;
    if (hits) hits[0] = (uint32_t)out->n;
    if (!p->fixed || k > 0) {
      rl_trim(out, n);
      rl_reduce(out);
    } else {
      *raw = 1;
    }
  }
  if (use_tvr && P->has_tvr) {
    if (P->tvr_list) {
      for (int i = 0; i < P->n_tvr; i++) {
        const pat_t* p = &P->tvr[i];
        rlist cur = {0};
        e = match_codes(p->code, p->m, p->fixed, S, n, 0, &cur); /* default max.mismatch=0 */
        if (!e && tvr_hits) tvr_hits[i] = (uint32_t)cur.n;
        if (!e && (!p->fixed || k > 0)) rl_trim(&cur, n);
        if (!e) e = rl_union(out, &cur);
        rl_free(&cur);
        if (e) return e;
      }
      rl_reduce(out); /* NanoTel.R:380 */
    } else {
      const pat_t* p = &P->tvr[0];
      rlist cur = {0};
      e = match_codes(p->code, p->m, p->fixed, S, n, 0, &cur);
      if (!e && tvr_hits) tvr_hits[0] = (uint32_t)cur.n;
      if (!e && (!p->fixed || k > 0)) {
        rl_trim(&cur, n);
        e = rl_union(out, &cur); /* NanoTel.R:387-390 */
      }
      rl_free(&cur);
      if (e) return e;
      rl_reduce(out); /* NanoTel.R:391 */
    }
    *raw = 0;
  }
  return NTO_OK;
}

/* -------------------------------------------------------------- windows */

/* split_telo (NanoTel.R:199-227) */
int64_t nto_window_count(int64_t n, int L) {
  if (n <= 0 || L <= 0) return 0;
  int64_t c = (n - 1) / L + 1;             /* seq(1, n, by=L) */
  int64_t last_start = 1 + (c - 1) * (int64_t)L;
  if ((double)(n - last_start) < (double)L / 2.0) c -= 1; /* drop the short tail window */
  return c;
}

typedef struct {
  int64_t start, end; /* 1-based */
  double density;
  int cls; /* -5 telomeric ("CCCTAA"), 1 NONE, 0 SKIP  (NanoTel.R:749) */
} win_t;

#define CLS_TELO (-5)
#define CLS_NONE 1
#define CLS_SKIP 0

/* analyze_subtelos (NanoTel.R:717-766): window table of one pass. */
static void analyze_subtelos(int64_t n, int L, double min_density, const cover_t* cov,
                             win_t* W, int64_t nw, uint32_t* counts) {
  for (int64_t i = 0; i < nw; i++) {
    int64_t s = 1 + i * (int64_t)L;
    int64_t e = (i == nw - 1) ? n : s + L - 1;
    int64_t cnt = cover_count(cov, s, e);
    double d = (double)cnt / (double)(e - s + 1);
    int cls = CLS_TELO;
    if (d < min_density) cls = (d < 0.1) ? CLS_SKIP : CLS_NONE;
    W[i].start = s;
    W[i].end = e;
    W[i].density = d;
    W[i].cls = cls;
    if (counts) counts[i] = (uint32_t)cnt;
  }
}

typedef struct { int64_t s, e; } pos2;

/* find_telo_position (NanoTel.R:973-1077).  W is 0-based, R indices 1-based. */
static pos2 find_telo_position(const win_t* W, int64_t nw, int64_t min_in_a_row,
                               double min_density_score) {
  pos2 r = {-1, -1};
  double score = 0.0;
  int64_t start = -1, end = -1, in_a_row = 0, end_position = 0;
  for (int64_t i = 1; i <= nw; i++) {
    const win_t* t = &W[i - 1];
    if (t->cls == CLS_SKIP || t->cls == CLS_NONE) {
      score = 0;
      start = -1;
      in_a_row = 0;
    } else {
      in_a_row++;
      score = score + t->density;
      if (start == -1) start = t->start;
    }
    if (in_a_row >= min_in_a_row && score >= min_density_score) {
      end_position = i + 1;
      break;
    }
  }
  if (end_position == 0) return r;
  end = -1;
  score = 0.0;
  in_a_row = 0;
  if (end_position >= nw - min_in_a_row + 1) {
    int64_t i = nw;
    const win_t* t = &W[i - 1];
    while (t->cls != CLS_TELO && i > end_position) {
      i--;
      t = &W[i - 1];
    }
    end = t->end;
  } else {
    for (int64_t i = nw; i >= end_position; i--) {
      const win_t* t = &W[i - 1];
      if (t->cls == CLS_SKIP || t->cls == CLS_NONE) {
        score = 0.0;
        end = -1;
        in_a_row = 0;
      } else {
        in_a_row++;
        score = score + t->density;
        if (end == -1) end = t->end;
      }
      if (in_a_row >= min_in_a_row && score >= min_density_score) break;
    }
  }
  if (start > end) end = start + (W[0].end - W[0].start);
  r.s = start;
  r.e = end;
  return r;
}

/* get_accurate_end (NanoTel.R:1692-1721); ranges = raw views or runs. */
static int64_t get_accurate_end(int64_t telo_end, const rlist* R) {
  if (telo_end == -1) return -1;
  int64_t e_index = telo_end, best = INT64_MIN;
  for (int64_t i = 0; i < R->n; i++)
    if (R->v[i].e >= telo_end - 99 && R->v[i].e <= telo_end && R->v[i].e > best) best = R->v[i].e;
  if (best != INT64_MIN) e_index = best;
  best = INT64_MIN;
  for (int64_t i = 0; i < R->n; i++)
    if (R->v[i].e >= telo_end + 1 && R->v[i].e <= telo_end + 50 && R->v[i].e > best) best = R->v[i].e;
  if (best != INT64_MIN) e_index = best;
  return e_index;
}

static int64_t min_start_in(const rlist* R, int64_t a, int64_t b, int64_t fallback) {
  int64_t best = INT64_MAX;
  for (int64_t i = 0; i < R->n; i++)
    if (R->v[i].s >= a && R->v[i].s <= b && R->v[i].s < best) best = R->v[i].s;
  return best == INT64_MAX ? fallback : best;
}

/* get_accurate_start (NanoTel.R:1726-1764) */
static int64_t get_accurate_start(int64_t telo_start, const rlist* R, const cover_t* cov) {
  if (telo_start == -1) return telo_start;
  int64_t s = telo_start;
  double first_50 = sub_density(cov, telo_start, telo_start + 49); /* IRanges(start, width=50) */
  if (first_50 < 0.3) {
    telo_start = min_start_in(R, s + 48, s + 99, telo_start);
    telo_start = min_start_in(R, s + 33, s + 48, telo_start);
  } else {
    telo_start = min_start_in(R, s, s + 99, telo_start);
    if (first_50 >= 0.72) telo_start = min_start_in(R, s - 36, s - 1, telo_start);
  }
  return telo_start;
}

/* find_left_telo (NanoTel.R:906-959) */
static pos2 find_left_telo(const win_t* W, int64_t nw) {
  const int64_t max_diff = 200;
  pos2 r;
  int64_t start = 1, end = 1, last_i = 1;
  for (int64_t i = 1; i <= nw; i++) {
    const win_t* t = &W[i - 1];
    if (t->start > max_diff) { r.s = -1; r.e = -1; return r; } /* subt$start partial-matches start_index */
    if (t->cls == CLS_SKIP || t->cls == CLS_NONE) continue;
    start = t->start;
    last_i = i;
    break;
  }
  int64_t last_i_start = last_i;
  /* for (i in last_i:nrow): with nrow == 0 this is 1:0 and row 1 is all-NA -> break */
  for (int64_t i = last_i; i <= nw; i++) {
    const win_t* t = &W[i - 1];
    if (t->cls == CLS_SKIP || t->cls == CLS_NONE) break;
    end = t->end;
  }
  if (nw > 0 && start > end) end = start + (W[last_i_start - 1].end - W[last_i_start - 1].start);
  r.s = start;
  r.e = end;
  return r;
}

/* find_right_telo (NanoTel.R:843-899).  Returns err on a 0-row table. */
static int find_right_telo(int64_t n, const win_t* W, int64_t nw, pos2* out) {
  const int64_t max_diff = 200;
  if (nw == 0) return NTO_E_RIGHT_EMPTY; /* nrow:1 = 0:1 -> if(logical(0)) errors */
  int64_t start = 1, end = 1, last_i = 1;
  for (int64_t i = nw; i >= 1; i--) {
    const win_t* t = &W[i - 1];
    if (t->end < n - max_diff) { out->s = -1; out->e = -1; return NTO_OK; }
    if (t->cls == CLS_SKIP || t->cls == CLS_NONE) continue;
    end = t->end;
    last_i = i;
    break;
  }
  for (int64_t i = last_i; i >= 1; i--) {
    const win_t* t = &W[i - 1];
    if (t->cls == CLS_SKIP || t->cls == CLS_NONE) break;
    start = t->start;
    last_i = i;
  }
  if (start > end) end = start + (W[last_i - 1].end - W[last_i - 1].start);
  out->s = start;
  out->e = end;
  return NTO_OK;
}

/* ---------------------------------------------------- edge extension (A12) */

/* matchPattern(pat, subseq(read, a, b), max.mismatch=k) -- default fixed=TRUE,
 * no trim: out-of-bound relative to the *sub-sequence*.  want_end: return max
 * end (else min start) in read coordinates; found=0 if no match. */
static int step_match(const uint8_t* S, int64_t a, int64_t b, const pat_t* p, int k, int want_end,
                      int64_t* val, int* found) {
  rlist v = {0};
  int e = match_codes(p->code, p->m, 1, S + (a - 1), b - a + 1, k, &v);
  if (e) { rl_free(&v); return e; }
  *found = v.n > 0;
  if (v.n > 0) {
    int64_t best = want_end ? INT64_MIN : INT64_MAX;
    for (int64_t i = 0; i < v.n; i++) {
      if (want_end) { if (v.v[i].e > best) best = v.v[i].e; }
      else { if (v.v[i].s < best) best = v.v[i].s; }
    }
    *val = best + a - 1;
  }
  rl_free(&v);
  return NTO_OK;
}

/* multi_pattern_step_left/right (NanoTel.R:496-528, 544-575): min start /
 * max end over every pattern (k = with_mismatch) and TVR (k=0). */
static int multi_step(const uint8_t* S, int64_t a, int64_t b, const nto_patterns* P, int k,
                      int use_tvr, int want_end, int64_t* val, int* found) {
  int any = 0;
  int64_t best = want_end ? INT64_MIN : INT64_MAX;
  int e;
  int only_exact = use_tvr && !k; /* (is.null(tvr) || with_mismatches) == FALSE */
  for (int i = 0; i < P->n_pat; i++) {
    int64_t v;
    int f;
    e = step_match(S, a, b, &P->pat[i], only_exact ? 0 : k, want_end, &v, &f);
    if (e) return e;
    if (f) { any = 1; best = want_end ? (v > best ? v : best) : (v < best ? v : best); }
  }
  if (use_tvr) {
    for (int i = 0; i < P->n_tvr; i++) {
      int64_t v;
      int f;
      e = step_match(S, a, b, &P->tvr[i], 0, want_end, &v, &f);
      if (e) return e;
      if (f) { any = 1; best = want_end ? (v > best ? v : best) : (v < best ? v : best); }
    }
  }
  *found = any;
  if (any) *val = best;
  return NTO_OK;
}

/* search_right_patterns (NanoTel.R:635-697) with subseq_width=18, step 10, 4 steps */
static int search_right(const uint8_t* S, int64_t n, int64_t end_index, const nto_patterns* P, int k,
                        int use_tvr, int64_t* out) {
  const int64_t width = 18, step = 10, max_steps = 4;
  int64_t subseq_end = end_index + width < n ? end_index + width : n;
  int64_t new_end = end_index;
  for (int64_t it = 1; it <= max_steps; it++) {
    int64_t curr_start = subseq_end - width + 1 > 1 ? subseq_end - width + 1 : 1;
    int64_t v;
    int f, e;
    /* single pattern without TVR: one matchPattern; list / TVR: multi_pattern_step_right.
       Both reduce to "max end over the pattern set" (min/max are order-free). */
    e = multi_step(S, curr_start, subseq_end, P, k, use_tvr, 1, &v, &f);
    if (e) return e;
    if (!f) break;
    new_end = v;
    int64_t ne = subseq_end + step + 1 < n ? subseq_end + step + 1 : n;
    if (ne == subseq_end) break;
    subseq_end = ne;
  }
  *out = new_end;
  return NTO_OK;
}

/* search_left_patterns (NanoTel.R:576-633) */
static int search_left(const uint8_t* S, int64_t n, int64_t start_index, const nto_patterns* P, int k,
                       int use_tvr, int64_t* out) {
  const int64_t width = 18, step = 10, max_steps = 4;
  int64_t subseq_start = start_index - width > 1 ? start_index - width : 1;
  int64_t new_start = start_index;
  for (int64_t it = 1; it <= max_steps; it++) {
    int64_t curr_end = subseq_start + width - 1 < n ? subseq_start + width - 1 : n;
    int64_t v;
    int f, e;
    e = multi_step(S, subseq_start, curr_end, P, k, use_tvr, 0, &v, &f);
    if (e) return e;
    if (!f) break;
    new_start = v;
    int64_t ns = subseq_start - step + 1 > 1 ? subseq_start - step + 1 : 1;
    if (ns == subseq_start) break;
    subseq_start = ns;
  }
  *out = new_start;
  return NTO_OK;
}

/* find_telo_position_wraper (NanoTel.R:1080-1155) */
static int telo_wrapper(const uint8_t* S, int64_t n, const nto_patterns* P, int L, int k,
                        int use_tvr, int right_edge, int legacy_no_ext, const win_t* W, int64_t nw,
                        const rlist* R, const cover_t* cov, pos2* out) {
  pos2 tp = find_telo_position(W, nw, 3, 2.0);
  double telo_density = sub_density(cov, tp.s, tp.e);
  int64_t num_rows = (tp.e - tp.s + 1) / L; /* width %/% global_subseq_length (width >= 1) */
  if (telo_density < 0.85 && num_rows > 5) {
    int64_t min_rows = num_rows <= 7 ? num_rows - 2 : 7;
    double min_density = 0.6 * (double)min_rows;
    tp = find_telo_position(W, nw, min_rows, min_density);
  }
  int64_t start_acc = get_accurate_start(tp.s, R, cov);
  int64_t end_acc = get_accurate_end(tp.e, R);
  if (start_acc > end_acc) end_acc = start_acc;
  tp.s = start_acc;
  tp.e = end_acc;
  if (tp.e - tp.s + 1 < 100) {
    if (right_edge) {
      int e = find_right_telo(n, W, nw, &tp);
      if (e) return e;
    } else {
      tp = find_left_telo(W, nw);
    }
  }
  if (!legacy_no_ext) {
    int64_t e2 = tp.e, s2 = tp.s;
    int e;
    if (tp.e < n) {
      e = search_right(S, n, tp.e + 1, P, k, use_tvr, &e2);
      if (e) return e;
    }
    if (tp.s > 1) {
      e = search_left(S, n, tp.s - 1, P, k, use_tvr, &s2);
      if (e) return e;
    }
    tp.s = s2;
    tp.e = e2;
  }
  if (tp.e < tp.s - 1) return NTO_E_NEG_WIDTH; /* IRanges(start, end) validity */
  *out = tp;
  return NTO_OK;
}

/* ------------------------------------------------------------ analyze_read */

int nto_analyze_read(const char* seq, int64_t n, const nto_patterns* P, int L, double min_density,
                     int right_edge, int legacy_no_ext, nto_row* row, uint32_t* win_counts,
                     uint32_t* hit_counts) {
  if (!seq || !P || !row || L <= 0) return NTO_E_ARG;
  if (n <= 0) return NTO_E_EMPTY_READ;
  memset(row, 0, sizeof *row);
  uint8_t* S = (uint8_t*)malloc((size_t)n);
  if (!S) return NTO_E_NOMEM;
  for (int64_t i = 0; i < n; i++) {
    S[i] = nto_dna_code(seq[i]);
    if (!S[i]) { free(S); return NTO_E_BAD_LETTER; }
  }
  int npass = nto_patterns_npass(P);
  int64_t nw = nto_window_count(n, L);
  win_t* W = (win_t*)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(win_t));
  if (!W) { free(S); return NTO_E_NOMEM; }
  int err = NTO_OK;
  pos2 tp[3];
  double dens[3];
  for (int p = 0; p < npass && !err; p++) {
    int k = p == 0 ? 0 : 1;
    int use_tvr = p == 2;
    rlist R = {0};
    int raw = 0;
    uint32_t* hits = NULL;
    if (hit_counts) hits = p == 0 ? hit_counts : p == 1 ? hit_counts + P->n_pat : NULL;
    if (hit_counts && use_tvr) hits = hit_counts + 2 * P->n_pat; /* TVR k=0 counters */
    err = density_iranges(S, n, P, k, use_tvr, &R, &raw, hits);
    cover_t cov;
    if (!err) err = cover_build(&cov, &R);
    if (!err) {
      analyze_subtelos(n, L, min_density, &cov, W, nw, win_counts ? win_counts + (int64_t)p * nw : NULL);
      err = telo_wrapper(S, n, P, L, k, use_tvr, right_edge, legacy_no_ext, W, nw, &R, &cov, &tp[p]);
      if (!err) dens[p] = sub_density(&cov, tp[p].s, tp[p].e); /* NanoTel.R:1840-1844 */
      cover_free(&cov);
    }
    rl_free(&R);
  }
  free(W);
  free(S);
  if (err) return err;
  row->n_pass = npass;
  row->n_windows = nw;
  int64_t maxw = INT64_MIN;
  for (int p = 0; p < npass; p++) {
    row->start[p] = (int32_t)tp[p].s;
    row->end[p] = (int32_t)tp[p].e;
    row->width[p] = tp[p].e - tp[p].s + 1;
    row->density[p] = dens[p];
    row->na[p] = tp[p].s == -1; /* NanoTel.R:1926-1940, 1956-1961 */
    if (row->width[p] > maxw) maxw = row->width[p];
  }
  row->telomeric = maxw >= 30; /* NanoTel.R:1847, 1857 */
  return NTO_OK;
}

/* ----------------------------------------------------------- --use_filter */

/* filter_reads + filter_density (NanoTel.R:2083-2103, 2121-2163), as called
 * per chunk from run_future_worker_chuncks (NanoTel.R:2227-2232) with
 * do_rc = FALSE (the chunk is already in scan orientation), subread_width =
 * 200, trimm_length = 70, min_density = global_min_density * 0.8.  Reads
 * shorter than 1e3 are dropped.  The edge sub-read is subseq(start = 71,
 * width = 200) (left) or subseq(end = -71, width = 200) = [n-269, n-70]
 * (right_edge = --check_right_edge).  Density = sum(width(union of the exact
 * fixed=FALSE matches of every (unique) pattern)) / nchar(sub-read).
 * Returns 1 = kept, 0 = dropped, <0 = error. */
int nto_filter_read(const char* seq, int64_t n, const nto_patterns* P, double min_density,
                    int right_edge) {
  if (!seq || !P) return NTO_E_ARG;
  if (n < 1000) return 0; /* samples[width(samples) >= 1e3] */
  const int64_t w = 200;
  const int64_t a = right_edge ? n - 269 : 71; /* 1-based start of the sub-read */
  uint8_t S[200];
  for (int64_t i = 0; i < w; i++) {
    S[i] = nto_dna_code(seq[a - 1 + i]);
    if (!S[i]) return NTO_E_BAD_LETTER;
  }
  rlist all = {0};
  for (int i = 0; i < P->n_pat; i++) {
    rlist v = {0};
    int e = match_codes(P->pat[i].code, P->pat[i].m, 0, S, w, 0, &v);
    if (!e) e = rl_union(&all, &v);
    rl_free(&v);
    if (e) { rl_free(&all); return e; }
  }
  int64_t cov = 0;
  for (int64_t i = 0; i < all.n; i++) cov += all.v[i].e - all.v[i].s + 1;
  rl_free(&all);
  const double total_density = (double)cov / (double)w;
  return total_density >= min_density * 0.8;
}

/* ------------------------------------------------------------- serials A15 */

int64_t nto_assign_serials(const uint8_t* is_telo, int64_t n, double* serial_start_io,
                           double* max_serial_io, double* serial_out, int64_t* order_out) {
  const int64_t groups = 8; /* groups_length <- 8 (NanoTel.R:2234) */
  double serial_start = *serial_start_io;
  double mx = *max_serial_io;
  int64_t rows = 0;
  for (int64_t j = 0; j < n; j++) serial_out[j] = NAN;
  if (n < groups) {
    /* sequential search_patterns (NanoTel.R:2236-2239, 2050-2070) */
    double cur = serial_start;
    for (int64_t j = 0; j < n; j++) {
      if (!is_telo[j]) continue;
      serial_out[j] = cur;
      order_out[rows++] = j;
      if (cur > mx) mx = cur;
      cur = cur + 1;
    }
  } else {
    /* split(1:n, f = 1:8): read j (1-based) -> group ((j-1) %% 8) + 1 */
    int64_t before = 0; /* length(unlist(split_seq[1:(g-1)])) */
    for (int64_t g = 0; g < groups; g++) {
      int64_t gsize = (n - g + groups - 1) / groups;
      double cur = (double)before + serial_start; /* length(...) + serial_start */
      for (int64_t j = g; j < n; j += groups) {
        if (!is_telo[j]) continue;
        serial_out[j] = cur;
        order_out[rows++] = j;
        if (cur > mx) mx = cur;
        cur = cur + 1;
      }
      before += gsize;
    }
  }
  *max_serial_io = mx;
  *serial_start_io = mx + 1; /* max(df_summary$Serial) + 1, -Inf if no rows yet */
  return rows;
}
