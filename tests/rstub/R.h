/* TEST STUB (tests/test_rpkg.py), not R's header: R is not installed in this image.  Declares only
 * what mkgpu/src/mk_r.c uses, with R's own types and signatures, so that the glue can be compiled for
 * a type check against include/mk.h.  Nothing here is linked or run. */
#ifndef MK_RSTUB_R_H
#define MK_RSTUB_R_H
#include <stddef.h>
typedef enum { FALSE = 0, TRUE } Rboolean;
void Rprintf(const char*, ...);
void R_FlushConsole(void);
void R_CheckUserInterrupt(void);
#endif
