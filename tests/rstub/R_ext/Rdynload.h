/* TEST STUB (tests/test_rpkg.py), not R's header; see tests/rstub/R.h. */
#ifndef MK_RSTUB_RDYNLOAD_H
#define MK_RSTUB_RDYNLOAD_H
#include "../R.h"
typedef void* (*DL_FUNC)(void);
typedef struct {
  const char* name;
  DL_FUNC fun;
  int numArgs;
} R_CallMethodDef;
typedef struct _DllInfo DllInfo;
int R_registerRoutines(DllInfo* info, const void* croutines, const R_CallMethodDef* callRoutines,
                       const void* fortranRoutines, const void* externalRoutines);
Rboolean R_useDynamicSymbols(DllInfo* info, Rboolean value);
#endif
