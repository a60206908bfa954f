/* .Call glue between R and libmk (include/mk.h).  Uncompiled in the build image (R is not
 * installed there); see INTEGRATION.md for how each entry replaces a reference line.
 *
 *   mk_r_fit      -> mk_fit_predict_batched   MK.R:102-111 (foreach %dopar% partitioned_spMvGLM)
 *   mk_r_combine  -> mk_combine               MK.R:123-133 (quantile-average combine)
 *   mk_r_summary  -> mk_posterior_summary_ex  MK.R:136-165 (resample, p(y = 1), quantiles)
 *   mk_r_glm      -> mk_glm_binomial_link     MK.R:53-55   (glm start values, on the device)
 *
 * Only array marshalling happens here: R owns the statistics that stay on the host (the
 * partition, the seed, R's own sample() index for MK.R:141).  Errors become Rf_error() with
 * mk_last_error()'s text after every PROTECT is released; no C++ frames are crossed. */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <string.h>
#include "mk.h"

static double* dp(SEXP x) { return isNull(x) ? NULL : REAL(x); }

static void fail(int nprot) {
  UNPROTECT(nprot);
  Rf_error("libmk: %s", mk_last_error());
}

/* cfg: list(cov.model (0/1), n.batch, batch.length, accept.rate, burn.in (1-based first kept),
 *           beta.starting, beta.tuning, phi.starting, phi.tuning, A.starting, A.tuning,
 *           w.starting, w.tuning, phi.Unif a, phi.Unif b, K.IW df, K.IW S,
 *           nu.starting, nu.tuning, nu.Unif a, nu.Unif b, link (0 logit / 1 probit),
 *           predict.tile, device)                         -- MK.R:56-64, 80-85
 * Returns list(parameters = S x 200 x P, w.predict = S x 200 x q n_test, acceptance). */
SEXP mk_r_fit(SEXP n_part, SEXP coords, SEXP y, SEXP weights, SEXP x, SEXP coords_test, SEXP q, SEXP p,
              SEXP cfg, SEXP seed) {
  mk_problem pr;
  memset(&pr, 0, sizeof pr);
  pr.n_subsets = LENGTH(n_part);
  pr.subset_base = 0;
  pr.q = asInteger(q);
  pr.p = asInteger(p);
  pr.n_part = INTEGER(n_part);
  pr.coords = REAL(coords);
  pr.y = REAL(y);
  pr.weights = REAL(weights);
  pr.x = REAL(x);
  pr.n_test = isNull(coords_test) ? 0 : nrows(coords_test);
  pr.coords_test = dp(coords_test);

  mk_config c;
  memset(&c, 0, sizeof c);
  c.cov_model = asInteger(VECTOR_ELT(cfg, 0));
  c.n_batch = asInteger(VECTOR_ELT(cfg, 1));
  c.batch_length = asInteger(VECTOR_ELT(cfg, 2));
  c.accept_rate = asReal(VECTOR_ELT(cfg, 3));
  c.burn_in = asInteger(VECTOR_ELT(cfg, 4));
  c.beta_starting = REAL(VECTOR_ELT(cfg, 5));
  c.beta_tuning = REAL(VECTOR_ELT(cfg, 6));
  c.phi_starting = REAL(VECTOR_ELT(cfg, 7));
  c.phi_tuning = REAL(VECTOR_ELT(cfg, 8));
  c.A_starting = REAL(VECTOR_ELT(cfg, 9));
  c.A_tuning = REAL(VECTOR_ELT(cfg, 10));
  c.w_starting = asReal(VECTOR_ELT(cfg, 11));
  c.w_tuning = asReal(VECTOR_ELT(cfg, 12));
  c.phi_unif_a = REAL(VECTOR_ELT(cfg, 13));
  c.phi_unif_b = REAL(VECTOR_ELT(cfg, 14));
  c.K_IW_df = asReal(VECTOR_ELT(cfg, 15));
  c.K_IW_S = REAL(VECTOR_ELT(cfg, 16));
  c.nu_starting = dp(VECTOR_ELT(cfg, 17));
  c.nu_tuning = dp(VECTOR_ELT(cfg, 18));
  c.nu_unif_a = dp(VECTOR_ELT(cfg, 19));
  c.nu_unif_b = dp(VECTOR_ELT(cfg, 20));
  c.link = asInteger(VECTOR_ELT(cfg, 21));
  c.predict_tile = asInteger(VECTOR_ELT(cfg, 22));
  c.device = asInteger(VECTOR_ELT(cfg, 23));
  c.seed = (uint64_t)asReal(seed); /* drawn from R's RNG by the caller: honours set.seed */
  c.record_samples = 1;
  c.record_w = 0;
  c.n_streams = 0;

  const int S = pr.n_subsets, np = LENGTH(VECTOR_ELT(cfg, 5));
  const int P = np + pr.q * (pr.q + 1) / 2 + pr.q * (c.cov_model == MK_COV_MATERN ? 2 : 1);
  const int n_acc = P + 1; /* per batch: the p betas, the covariance parameters, the latent w */
  SEXP par = PROTECT(allocVector(REALSXP, (R_xlen_t)S * MK_N_LEVELS * P));
  SEXP wpr = PROTECT(allocVector(REALSXP, (R_xlen_t)S * MK_N_LEVELS * pr.q * pr.n_test));
  SEXP acc = PROTECT(allocVector(REALSXP, (R_xlen_t)S * c.n_batch * n_acc));
  mk_outputs o;
  memset(&o, 0, sizeof o);
  o.parameters = REAL(par);
  o.w_predict = pr.n_test ? REAL(wpr) : NULL;
  o.acceptance = REAL(acc);
  if (mk_fit_predict_batched(&pr, &c, &o) != MK_OK) fail(3);
  SEXP res = PROTECT(allocVector(VECSXP, 3));
  SET_VECTOR_ELT(res, 0, par);
  SET_VECTOR_ELT(res, 1, wpr);
  SET_VECTOR_ELT(res, 2, acc);
  UNPROTECT(4);
  return res;
}

/* grids: K x len doubles (the K subset grids back to back, each column-major as R holds it).
 * Returns (grid_1 + ... + grid_K) / K in the sequential order of MK.R:129-132. */
SEXP mk_r_combine(SEXP grids, SEXP K, SEXP len, SEXP device) {
  const int k = asInteger(K);
  const R_xlen_t n = (R_xlen_t)asReal(len);
  SEXP out = PROTECT(allocVector(REALSXP, n));
  if (mk_combine(REAL(grids), k, (int64_t)n, REAL(out), asInteger(device)) != MK_OK) fail(1);
  UNPROTECT(1);
  return out;
}

/* MK.R:136-165 on the combined grids: result 200 x P, result2 200 x C, x_test C x p,
 * index = R's sample(seq(1, length(Xout), 1), samplesize, replace = TRUE) (MK.R:141, 1-based).
 * Returns list(SamplePar, Samplew, p.sample, w.quant, param.quant). */
SEXP mk_r_summary(SEXP result, SEXP result2, SEXP x_test, SEXP index, SEXP link, SEXP device) {
  const int P = ncols(result), p = ncols(x_test), ss = LENGTH(index);
  const int64_t C = ncols(result2);
  SEXP sp = PROTECT(allocMatrix(REALSXP, ss, P));
  SEXP sw = PROTECT(allocMatrix(REALSXP, ss, (int)C));
  SEXP ps = PROTECT(allocMatrix(REALSXP, ss, (int)C));
  SEXP wq = PROTECT(allocMatrix(REALSXP, 3, (int)C));
  SEXP pq = PROTECT(allocMatrix(REALSXP, 3, P));
  mk_summary o;
  memset(&o, 0, sizeof o);
  o.sample_par = REAL(sp);
  o.sample_w = REAL(sw);
  o.p_sample = REAL(ps);
  o.w_quant = REAL(wq);
  o.param_quant = REAL(pq);
  if (mk_posterior_summary_ex(REAL(result), P, REAL(result2), C, REAL(x_test), p, ss, 0, INTEGER(index),
                              asInteger(link), &o, asInteger(device)) != MK_OK)
    fail(5);
  SEXP res = PROTECT(allocVector(VECSXP, 5));
  SET_VECTOR_ELT(res, 0, sp);
  SET_VECTOR_ELT(res, 1, sw);
  SET_VECTOR_ELT(res, 2, ps);
  SET_VECTOR_ELT(res, 3, wq);
  SET_VECTOR_ELT(res, 4, pq);
  UNPROTECT(6);
  return res;
}

/* glm((y / weight) ~ x - 1, weights, family = binomial(link)) on the device: list(coef, vcov). */
SEXP mk_r_glm(SEXP y, SEXP weights, SEXP x, SEXP link, SEXP device) {
  const int64_t n = nrows(x);
  const int p = ncols(x);
  SEXP coef = PROTECT(allocVector(REALSXP, p));
  SEXP vc = PROTECT(allocMatrix(REALSXP, p, p));
  if (mk_glm_binomial_link(REAL(y), REAL(weights), REAL(x), n, p, asInteger(link), 1e-8, 25, REAL(coef), REAL(vc),
                           NULL, asInteger(device)) != MK_OK)
    fail(2);
  SEXP res = PROTECT(allocVector(VECSXP, 2));
  SET_VECTOR_ELT(res, 0, coef);
  SET_VECTOR_ELT(res, 1, vc);
  UNPROTECT(3);
  return res;
}

static const R_CallMethodDef call_methods[] = {
    {"mk_r_fit", (DL_FUNC)&mk_r_fit, 10},
    {"mk_r_combine", (DL_FUNC)&mk_r_combine, 4},
    {"mk_r_summary", (DL_FUNC)&mk_r_summary, 6},
    {"mk_r_glm", (DL_FUNC)&mk_r_glm, 5},
    {NULL, NULL, 0}};

void R_init_mkgpu(DllInfo* dll) {
  R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
