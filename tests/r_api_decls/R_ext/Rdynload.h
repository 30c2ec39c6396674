/* Declarations of the public R C API subset that r/nanotel_r.c uses (R is
 * not installed in this image); see ../Rinternals.h.  Test scaffolding only. */
#pragma once
#include "../Rinternals.h"
typedef void* (*DL_FUNC)(void);
typedef struct _DllInfo DllInfo;
typedef struct {
  const char* name;
  DL_FUNC fun;
  int numArgs;
} R_CallMethodDef;
int R_registerRoutines(DllInfo*, const void*, const R_CallMethodDef*, const void*, const void*);
Rboolean R_useDynamicSymbols(DllInfo*, Rboolean);
