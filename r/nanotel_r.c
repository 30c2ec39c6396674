/* nanotel_r.c -- the R .Call shim of the MI355X hot path (the reference-side
 * binding of include/nanotel.h).
 *
 * NanoTel is one R script (NanoTel.R).  Per nrec-record chunk its driver
 * run_future_worker_chuncks (NanoTel.R:2171-2268) fans the reads out to 8
 * forked futures of search_patterns (NanoTel.R:2234-2252), each of which runs
 * analyze_read (NanoTel.R:1774-1976) read by read, and joins their data.frames
 * with Reduce(union_all) (NanoTel.R:2254).  This shim replaces that block with
 * one call per chunk into libnanotel.so: the scan, the telomere calling, the
 * serials and the reference's group-major row order, returned as the chunk's
 * data.frame in analyze_read's columns (NanoTel.R:1820-1837).  r/nanotel.R
 * wraps the entry points; r/NanoTel.R.patch is the change to NanoTel.R.
 *
 * Build (R headers and libnanotel.so present):
 *   R CMD SHLIB -o libnanotel_r.so r/nanotel_r.c -I include \
 *       -L telomere-analyzer_amd/nanotel_amd -lnanotel
 *
 * Errors follow the reference's: a failure the reference raises (an invalid
 * letter in a read, an empty read, find_right_telo on a read without windows,
 * a negative IRanges width; NT_E_* in nanotel.h) becomes Rf_error with the
 * library's message, after the shim has released what it owns (R_alloc
 * memory is R's; no longjmp crosses the C-ABI).  HIP is initialised by
 * R_nt_create in the calling R process: never before a fork (the patch drops
 * future::multicore, one R process per GPU). */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nanotel.h"

static void nt_finalizer(SEXP p) {
  nt_ctx* ctx = (nt_ctx*)R_ExternalPtrAddr(p);
  if (ctx) {
    nt_destroy(ctx);
    R_ClearExternalPtr(p);
  }
}

static nt_ctx* nt_of(SEXP ptr) {
  nt_ctx* ctx = (nt_ctx*)R_ExternalPtrAddr(ptr);
  if (!ctx) Rf_error("nanotel: the context was destroyed");
  return ctx;
}

/* Errors: the message is copied out of the context first, then raised. */
static void nt_stop(nt_ctx* ctx, int rc) {
  char msg[512];
  snprintf(msg, sizeof msg, "%s", nt_last_error(ctx));
  Rf_error("nanotel: %d %s", rc, msg);
}

/* nt_create + nt_compile: --patterns / --tvr_patterns exactly as given on the
 * command line (extract_patterns, NanoTel.R:2322-2334, is the library's),
 * --subseq_length, --min_density, --check_right_edge, --rc.  The returned
 * external pointer carries n_pass (2, or 3 with TVRs), subseq_length and
 * min_density as attributes. */
SEXP R_nt_create(SEXP dev, SEXP pat, SEXP tvr, SEXP L, SEXP md, SEXP right, SEXP rc) {
  nt_ctx* ctx = NULL;
  int e = nt_create(Rf_asInteger(dev), &ctx);
  if (e) Rf_error("nanotel: nt_create failed (%d)", e);
  nt_params p;
  p.patterns = CHAR(STRING_ELT(pat, 0));
  p.tvr_patterns = Rf_isNull(tvr) ? NULL : CHAR(STRING_ELT(tvr, 0));
  p.subseq_length = Rf_asInteger(L);
  p.min_density = Rf_asReal(md);
  p.check_right_edge = Rf_asLogical(right);
  p.rc = Rf_asLogical(rc);
  p.legacy_no_ext = 0;
  nt_program_info info;
  if ((e = nt_compile(ctx, &p, &info))) {
    char msg[512];
    snprintf(msg, sizeof msg, "%s", nt_last_error(ctx));
    nt_destroy(ctx); /* free first, then raise */
    Rf_error("nanotel: %d %s", e, msg);
  }
  SEXP ptr = PROTECT(R_MakeExternalPtr(ctx, Rf_install("nt_ctx"), R_NilValue));
  R_RegisterCFinalizerEx(ptr, nt_finalizer, TRUE);
  Rf_setAttrib(ptr, Rf_install("n_pass"), Rf_ScalarInteger(info.n_pass));
  Rf_setAttrib(ptr, Rf_install("count_bytes"), Rf_ScalarInteger(info.count_bytes));
  Rf_setAttrib(ptr, Rf_install("subseq_length"), Rf_ScalarInteger(p.subseq_length));
  Rf_setAttrib(ptr, Rf_install("min_density"), Rf_ScalarReal(p.min_density));
  UNPROTECT(1);
  return ptr;
}

SEXP R_nt_destroy(SEXP ptr) {
  nt_finalizer(ptr);
  return R_NilValue;
}

static const char* kCols[] = {
    "Serial", "sequence_ID", "sequence_length",
    "telo_density", "Telomere_start", "Telomere_end", "Telomere_length",
    "telo_density_mismatch", "Telomere_start_mismatch", "Telomere_end_mismatch", "Telomere_length_mismatch",
    "telo_density_mismatch_tvr", "Telomere_start_mismatch_tvr", "Telomere_end_mismatch_tvr",
    "Telomere_length_mismatch_tvr"};

static SEXP named_list(int n, const char** names) {
  SEXP out = PROTECT(Rf_allocVector(VECSXP, n));
  SEXP nm = PROTECT(Rf_allocVector(STRSXP, n));
  for (int k = 0; k < n; ++k) SET_STRING_ELT(nm, k, Rf_mkChar(names[k]));
  Rf_setAttrib(out, R_NamesSymbol, nm);
  UNPROTECT(2);
  return out;
}

/* The window table of one read and pass as analyze_subtelos builds it
 * (NanoTel.R:717-766, split_telo 199-227, get_sub_density 449-468): window k
 * = [1 + kL, 1 + (k + 1)L - 1], the last one ending at n; density = covered
 * bases / width in fp64 (IEEE division, as R's); class -5 when density >=
 * min_density, 0 when < 0.1, else 1.  From the scan's window counts. */
static SEXP window_table(const uint8_t* cnt8, const uint16_t* cnt16, int64_t nw, int64_t n, int L, double md) {
  static const char* cols[] = {"ID", "start_index", "end_index", "density", "class"};
  SEXP df = PROTECT(named_list(5, cols));
  SEXP id = Rf_allocVector(INTSXP, nw);      SET_VECTOR_ELT(df, 0, id);
  SEXP s = Rf_allocVector(INTSXP, nw);       SET_VECTOR_ELT(df, 1, s);
  SEXP e = Rf_allocVector(INTSXP, nw);       SET_VECTOR_ELT(df, 2, e);
  SEXP d = Rf_allocVector(REALSXP, nw);      SET_VECTOR_ELT(df, 3, d);
  SEXP c = Rf_allocVector(REALSXP, nw);      SET_VECTOR_ELT(df, 4, c);
  for (int64_t k = 0; k < nw; ++k) {
    const int64_t a = 1 + k * (int64_t)L, b = k + 1 == nw ? n : (k + 1) * (int64_t)L;
    const double cov = cnt8 ? (double)cnt8[k] : (double)cnt16[k];
    const double den = cov / (double)(b - a + 1);
    INTEGER(id)[k] = (int)(k + 1);
    INTEGER(s)[k] = (int)a;
    INTEGER(e)[k] = (int)b;
    REAL(d)[k] = den;
    REAL(c)[k] = den < md ? (den < 0.1 ? 0.0 : 1.0) : -5.0;
  }
  SEXP rn = PROTECT(Rf_allocVector(INTSXP, 2));
  INTEGER(rn)[0] = NA_INTEGER;
  INTEGER(rn)[1] = -(int)nw;
  Rf_setAttrib(df, R_RowNamesSymbol, rn);
  Rf_setAttrib(df, R_ClassSymbol, Rf_mkString("data.frame"));
  UNPROTECT(2);
  return df;
}

/* One chunk: reads (character, scan orientation), ids (character),
 * serial_start (double), max_serial (double, -Inf before the first row),
 * want_windows (logical).  Returns list(rows = data.frame, next_serial_start,
 * max_serial, windows): the block NanoTel.R:2234-2258 computes -- the rows of
 * search_patterns over the 8 groups (NanoTel.R:2001-2078) joined by
 * Reduce(union_all) in group order, serial_start <- max(df_summary$Serial) + 1
 * -- and, when want_windows, for every row the read's index in the chunk
 * (1-based), its called start/end per pass (-1 when the pass found none, as
 * telo_position holds it) and its per-pass window tables (analyze_list[[1]]
 * of analyze_read), which the plots take (NanoTel.R:1876-1918). */
SEXP R_nt_analyze_chunk(SEXP ptr, SEXP reads, SEXP ids, SEXP serial_start, SEXP max_serial, SEXP want_windows) {
  nt_ctx* ctx = nt_of(ptr);
  const R_xlen_t n = XLENGTH(reads);
  if (XLENGTH(ids) != n) Rf_error("nanotel: %d reads but %d ids", (int)n, (int)XLENGTH(ids));
  const int np = Rf_asInteger(Rf_getAttrib(ptr, Rf_install("n_pass")));
  const int cb = Rf_asInteger(Rf_getAttrib(ptr, Rf_install("count_bytes")));
  const int L = Rf_asInteger(Rf_getAttrib(ptr, Rf_install("subseq_length")));
  const double md = Rf_asReal(Rf_getAttrib(ptr, Rf_install("min_density")));
  const int ww = Rf_asLogical(want_windows) == 1;
  const R_xlen_t n1 = n > 0 ? n : 1;
  const char** seqs = (const char**)R_alloc(n1, sizeof(char*));
  uint64_t* lens = (uint64_t*)R_alloc(n1, sizeof(uint64_t));
  uint64_t* woff = (uint64_t*)R_alloc(n1 + 1, sizeof(uint64_t)); /* the reads' window rows, prefix sum */
  woff[0] = 0;
  for (R_xlen_t i = 0; i < n; ++i) {
    seqs[i] = CHAR(STRING_ELT(reads, i));
    lens[i] = (uint64_t)LENGTH(STRING_ELT(reads, i));
    woff[i + 1] = woff[i] + nt_window_rows(nt_window_count((int64_t)lens[i], L));
  }
  /* the calling kernel's per-read outputs (R_alloc: freed by R on return or error) */
  int32_t* st = (int32_t*)R_alloc(3 * n1, sizeof(int32_t));
  int32_t* en = (int32_t*)R_alloc(3 * n1, sizeof(int32_t));
  double* de = (double*)R_alloc(3 * n1, sizeof(double));
  uint8_t* fl = (uint8_t*)R_alloc(n1, 1);
  void* wc = ww ? (void*)R_alloc(woff[n] * np + 1, cb) : NULL;
  int e = nt_analyze_host(ctx, seqs, lens, (uint64_t)n, st, en, de, fl, wc, NULL);
  if (e) nt_stop(ctx, e); /* same failures as the reference (NT_E_*) */
  /* A15: serials and the group-major row order (NanoTel.R:2050-2070, 2234-2254) */
  uint8_t* telo = (uint8_t*)R_alloc(n1, 1);
  for (R_xlen_t i = 0; i < n; ++i) telo[i] = (fl[i] & NT_ROW_TELOMERIC) != 0;
  double ss = Rf_asReal(serial_start), mx = Rf_asReal(max_serial);
  double* serial = (double*)R_alloc(n1, sizeof(double));
  int64_t* order = (int64_t*)R_alloc(n1, sizeof(int64_t));
  const int64_t rows = nt_assign_serials(telo, (uint64_t)n, &ss, &mx, serial, order);
  if (rows < 0) nt_stop(ctx, (int)rows);
  /* the columns of analyze_read's data.frame (NanoTel.R:1820-1837): the library
   * writes R's NA_integer_ / NA_real_ itself, so it fills the vectors in place */
  const int ncol = 3 + 4 * np; /* 11 columns, 15 with --tvr_patterns */
  SEXP df = PROTECT(Rf_allocVector(VECSXP, ncol));
  SEXP c_serial = Rf_allocVector(REALSXP, rows);  SET_VECTOR_ELT(df, 0, c_serial);
  SEXP c_id = Rf_allocVector(STRSXP, rows);       SET_VECTOR_ELT(df, 1, c_id);
  SEXP c_len = Rf_allocVector(INTSXP, rows);      SET_VECTOR_ELT(df, 2, c_len);
  /* per pass p: density (double), start, end, width (integer) -- one block of
   * rows per pass, as nt_rows_columns lays them out */
  const int64_t r1 = rows > 0 ? rows : 1;
  double* dens = (double*)R_alloc(np * r1, sizeof(double));
  int32_t* cs = (int32_t*)R_alloc(np * r1, sizeof(int32_t));
  int32_t* ce = (int32_t*)R_alloc(np * r1, sizeof(int32_t));
  int32_t* cw = (int32_t*)R_alloc(np * r1, sizeof(int32_t));
  const int64_t got = nt_rows_columns(st, en, de, lens, (uint64_t)n, np, serial, order, rows,
                                      REAL(c_serial), INTEGER(c_len), dens, cs, ce, cw);
  if (got != rows) {
    UNPROTECT(1);
    nt_stop(ctx, (int)(got < 0 ? got : NT_E_ARG));
  }
  for (int64_t i = 0; i < rows; ++i) /* sequence_ID = names(dna_reads)[j] */
    SET_STRING_ELT(c_id, i, STRING_ELT(ids, (R_xlen_t)order[i]));
  for (int p = 0; p < np; ++p) {
    SEXP d = Rf_allocVector(REALSXP, rows);  SET_VECTOR_ELT(df, 3 + 4 * p, d);
    SEXP s = Rf_allocVector(INTSXP, rows);   SET_VECTOR_ELT(df, 4 + 4 * p, s);
    SEXP t = Rf_allocVector(INTSXP, rows);   SET_VECTOR_ELT(df, 5 + 4 * p, t);
    SEXP w = Rf_allocVector(INTSXP, rows);   SET_VECTOR_ELT(df, 6 + 4 * p, w);
    if (rows > 0) {
      memcpy(REAL(d), dens + p * rows, rows * sizeof(double));
      memcpy(INTEGER(s), cs + p * rows, rows * sizeof(int32_t));
      memcpy(INTEGER(t), ce + p * rows, rows * sizeof(int32_t));
      memcpy(INTEGER(w), cw + p * rows, rows * sizeof(int32_t));
    }
  }
  /* a data.frame: names, compact row names, class */
  SEXP nm = PROTECT(Rf_allocVector(STRSXP, ncol));
  for (int k = 0; k < ncol; ++k) SET_STRING_ELT(nm, k, Rf_mkChar(kCols[k]));
  Rf_setAttrib(df, R_NamesSymbol, nm);
  SEXP rn = PROTECT(Rf_allocVector(INTSXP, 2));
  INTEGER(rn)[0] = NA_INTEGER;
  INTEGER(rn)[1] = -(int)rows;
  Rf_setAttrib(df, R_RowNamesSymbol, rn);
  Rf_setAttrib(df, R_ClassSymbol, Rf_mkString("data.frame"));
  /* the rows' window tables and called positions (plots) */
  SEXP win = PROTECT(Rf_allocVector(VECSXP, ww ? rows : 0));
  for (int64_t i = 0; ww && i < rows; ++i) {
    static const char* wcols[] = {"read", "start", "end", "tables"};
    const int64_t j = order[i];
    SEXP w = PROTECT(named_list(4, wcols));
    SET_VECTOR_ELT(w, 0, Rf_ScalarInteger((int)j + 1));
    SEXP ps = Rf_allocVector(INTSXP, np);  SET_VECTOR_ELT(w, 1, ps);
    SEXP pe = Rf_allocVector(INTSXP, np);  SET_VECTOR_ELT(w, 2, pe);
    SEXP tb = Rf_allocVector(VECSXP, np);  SET_VECTOR_ELT(w, 3, tb);
    const int64_t nw = nt_window_count((int64_t)lens[j], L);
    const uint64_t rws = nt_window_rows(nw);
    for (int p = 0; p < np; ++p) {
      INTEGER(ps)[p] = st[3 * j + p];
      INTEGER(pe)[p] = en[3 * j + p];
      const uint64_t o = woff[j] * np + p * rws; /* [win_off * np + p * rows + k] */
      SET_VECTOR_ELT(tb, p, window_table(cb == 1 ? (const uint8_t*)wc + o : NULL,
                                         cb == 2 ? (const uint16_t*)wc + o : NULL, nw, (int64_t)lens[j], L, md));
    }
    SET_VECTOR_ELT(win, i, w);
    UNPROTECT(1);
  }
  static const char* onames[] = {"rows", "next_serial_start", "max_serial", "windows"};
  SEXP out = PROTECT(named_list(4, onames));
  SET_VECTOR_ELT(out, 0, df);
  SET_VECTOR_ELT(out, 1, Rf_ScalarReal(ss)); /* next serial_start = max(Serial) + 1 */
  SET_VECTOR_ELT(out, 2, Rf_ScalarReal(mx)); /* running max(Serial) */
  SET_VECTOR_ELT(out, 3, win);
  UNPROTECT(5);
  return out;
}

/* --use_filter: keep[i] = filter_reads / filter_density's decision for read i
 * (reads >= 1 kb whose 200-base edge sub-read is >= 0.8 min_density covered;
 * NanoTel.R:2083-2163, called per chunk at 2227-2232). */
SEXP R_nt_filter_chunk(SEXP ptr, SEXP reads) {
  nt_ctx* ctx = nt_of(ptr);
  const R_xlen_t n = XLENGTH(reads);
  const R_xlen_t n1 = n > 0 ? n : 1;
  const char** seqs = (const char**)R_alloc(n1, sizeof(char*));
  uint64_t* lens = (uint64_t*)R_alloc(n1, sizeof(uint64_t));
  for (R_xlen_t i = 0; i < n; ++i) {
    seqs[i] = CHAR(STRING_ELT(reads, i));
    lens[i] = (uint64_t)LENGTH(STRING_ELT(reads, i));
  }
  uint8_t* keep = (uint8_t*)R_alloc(n1, 1);
  int e = nt_filter_host(ctx, seqs, lens, (uint64_t)n, keep);
  if (e) nt_stop(ctx, e);
  SEXP out = PROTECT(Rf_allocVector(LGLSXP, n));
  for (R_xlen_t i = 0; i < n; ++i) LOGICAL(out)[i] = keep[i] != 0;
  UNPROTECT(1);
  return out;
}

static const R_CallMethodDef kCalls[] = {
    {"R_nt_create", (DL_FUNC)&R_nt_create, 7},
    {"R_nt_destroy", (DL_FUNC)&R_nt_destroy, 1},
    {"R_nt_analyze_chunk", (DL_FUNC)&R_nt_analyze_chunk, 6},
    {"R_nt_filter_chunk", (DL_FUNC)&R_nt_filter_chunk, 2},
    {NULL, NULL, 0}};

void R_init_libnanotel_r(DllInfo* dll) {
  R_registerRoutines(dll, NULL, kCalls, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
