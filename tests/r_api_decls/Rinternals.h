/* Declarations of the public R C API subset that r/nanotel_r.c (the .Call shim)
 * uses (R is not installed in this image).  Test scaffolding only: it lets
 * tests/test_integration_shim.py type-check the documented shim against
 * include/nanotel.h with gcc -fsyntax-only; nothing is linked or run. */
#pragma once
#include <stddef.h>
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef unsigned int SEXPTYPE;
typedef enum { FALSE = 0, TRUE } Rboolean;
#define LGLSXP 10
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
extern SEXP R_NilValue, R_NamesSymbol, R_RowNamesSymbol, R_ClassSymbol;
extern double R_NegInf;
extern int R_NaInt;
#define NA_INTEGER R_NaInt
typedef void (*R_CFinalizer_t)(SEXP);
void Rf_error(const char*, ...) __attribute__((noreturn));
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
void* R_ExternalPtrAddr(SEXP);
void R_ClearExternalPtr(SEXP);
SEXP R_MakeExternalPtr(void*, SEXP, SEXP);
void R_RegisterCFinalizerEx(SEXP, R_CFinalizer_t, Rboolean);
int Rf_asInteger(SEXP);
double Rf_asReal(SEXP);
int Rf_asLogical(SEXP);
Rboolean Rf_isNull(SEXP);
SEXP Rf_install(const char*);
SEXP Rf_allocVector(SEXPTYPE, R_xlen_t);
SEXP Rf_getAttrib(SEXP, SEXP);
SEXP Rf_setAttrib(SEXP, SEXP, SEXP);
SEXP Rf_ScalarInteger(int);
SEXP Rf_ScalarReal(double);
SEXP Rf_mkChar(const char*);
SEXP Rf_mkString(const char*);
R_xlen_t XLENGTH(SEXP);
int LENGTH(SEXP);
SEXP STRING_ELT(SEXP, R_xlen_t);
void SET_STRING_ELT(SEXP, R_xlen_t, SEXP);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
const char* CHAR(SEXP);
double* REAL(SEXP);
int* INTEGER(SEXP);
int* LOGICAL(SEXP);
char* R_alloc(size_t, int);
