/* TEST STUB (tests/test_rpkg.py), not R's header; see tests/rstub/R.h. */
#ifndef MK_RSTUB_RINTERNALS_H
#define MK_RSTUB_RINTERNALS_H
#include "R.h"
typedef struct SEXPREC* SEXP;
typedef ptrdiff_t R_xlen_t;
typedef int R_len_t;
typedef unsigned int SEXPTYPE;
#define NILSXP 0
#define LGLSXP 10
#define INTSXP 13
#define REALSXP 14
#define STRSXP 16
#define VECSXP 19
extern SEXP R_NilValue;
double* REAL(SEXP);
int* INTEGER(SEXP);
int* LOGICAL(SEXP);
SEXP VECTOR_ELT(SEXP, R_xlen_t);
SEXP SET_VECTOR_ELT(SEXP, R_xlen_t, SEXP);
int LENGTH(SEXP);
SEXP Rf_protect(SEXP);
void Rf_unprotect(int);
#define PROTECT(s) Rf_protect(s)
#define UNPROTECT(n) Rf_unprotect(n)
int asInteger(SEXP);
double asReal(SEXP);
int asLogical(SEXP);
SEXP allocMatrix(SEXPTYPE, int, int);
SEXP allocVector(SEXPTYPE, R_xlen_t);
int nrows(SEXP);
int ncols(SEXP);
R_len_t length(SEXP);
Rboolean isNull(SEXP);
SEXP ScalarInteger(int);
SEXP ScalarLogical(int);
SEXP ScalarReal(double);
SEXP install(const char*);
void Rf_error(const char*, ...) __attribute__((noreturn));
void error(const char*, ...) __attribute__((noreturn));
Rboolean R_ToplevelExec(void (*fun)(void*), void* data);
typedef void (*R_CFinalizer_t)(SEXP);
void* R_ExternalPtrAddr(SEXP);
SEXP R_MakeExternalPtr(void* p, SEXP tag, SEXP prot);
void R_ClearExternalPtr(SEXP);
void R_RegisterCFinalizerEx(SEXP s, R_CFinalizer_t fun, Rboolean onexit);
#endif
