/* .Call glue between R and libmk (include/mk.h).  Uncompiled in the build image (R is not
 * installed there); see INTEGRATION.md for how each entry replaces a reference line.
 *
 *   mk_r_fit        -> mk_meta_fit               MK.R:100-133 (makeCluster + foreach %dopar%
 *                                                partitioned_spMvGLM over the node's GPUs, and the
 *                                                quantile-average combine, device to device)
 *   mk_r_spmvglm    -> mk_session_create / _run  MK.R:80-84 (spMvGLM of one subset; the session
 *                      / _outputs                stays alive for spPredict, owned by an external
 *                                                pointer whose finalizer destroys it)
 *   mk_r_sppredict  -> mk_session_set_test_sites MK.R:87 (spPredict(m.1, coords.test, x.test,
 *                      / _set_kept_window        start, end): kriging replayed from the recorded
 *                      / _outputs                chain states, no refit)
 *   mk_r_combine    -> mk_combine                MK.R:123-133 (quantile-average combine)
 *   mk_r_summary    -> mk_posterior_summary_ex   MK.R:136-165 (resample, p(y = 1), quantiles)
 *   mk_r_glm        -> mk_glm_binomial_link      MK.R:53-55   (glm start values, on the device)
 *
 * The MCMC runs one amcmc batch at a time: between batches the glue prints spBayes's n.report
 * line and checks for a user interrupt (R_CheckUserInterrupt inside R_ToplevelExec, so the
 * long jump never crosses libmk's frames); an interrupt stops the fit, frees every device buffer
 * and raises an R error.  Only array marshalling happens here otherwise: R owns the statistics
 * that stay on the host (the partition, the seed, R's own sample() index for MK.R:141).  Errors
 * become Rf_error() with mk_last_error()'s text after every PROTECT is released. */
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

/* ---- amcmc progress between batches: spBayes's n.report line + R's interrupt check ---- */
typedef struct {
  int report, n_batch, batch_length, interrupted;
} progress_t;

static void check_interrupt(void* unused) {
  (void)unused;
  R_CheckUserInterrupt();
}

static int r_progress(void* user, int32_t it, int32_t n_samples) {
  progress_t* pg = (progress_t*)user;
  const int b = it / pg->batch_length;
  if (pg->report > 0 && (b % pg->report == 0 || it == n_samples)) {
    Rprintf("Batch: %i of %i, %3.2f%%\n", b, pg->n_batch, 100.0 * it / n_samples);
    R_FlushConsole();
  }
  if (!R_ToplevelExec(check_interrupt, NULL)) {   /* FALSE: the check jumped (an interrupt) */
    pg->interrupted = 1;
    return 1;
  }
  return 0;
}

/* cfg: list(cov.model (0/1), n.batch, batch.length, accept.rate, burn.in (1-based first kept),
 *           beta.starting, beta.tuning, phi.starting, phi.tuning, A.starting, A.tuning,
 *           w.starting, w.tuning, phi.Unif a, phi.Unif b, K.IW df, K.IW S,
 *           nu.starting, nu.tuning, nu.Unif a, nu.Unif b, link (0 logit / 1 probit),
 *           predict.tile, device)                         -- MK.R:56-64, 80-85 */
static void read_config(SEXP cfg, SEXP seed, mk_config* c) {
  memset(c, 0, sizeof *c);
  c->cov_model = asInteger(VECTOR_ELT(cfg, 0));
  c->n_batch = asInteger(VECTOR_ELT(cfg, 1));
  c->batch_length = asInteger(VECTOR_ELT(cfg, 2));
  c->accept_rate = asReal(VECTOR_ELT(cfg, 3));
  c->burn_in = asInteger(VECTOR_ELT(cfg, 4));
  c->beta_starting = REAL(VECTOR_ELT(cfg, 5));
  c->beta_tuning = REAL(VECTOR_ELT(cfg, 6));
  c->phi_starting = REAL(VECTOR_ELT(cfg, 7));
  c->phi_tuning = REAL(VECTOR_ELT(cfg, 8));
  c->A_starting = REAL(VECTOR_ELT(cfg, 9));
  c->A_tuning = REAL(VECTOR_ELT(cfg, 10));
  c->w_starting = asReal(VECTOR_ELT(cfg, 11));
  c->w_tuning = asReal(VECTOR_ELT(cfg, 12));
  c->phi_unif_a = REAL(VECTOR_ELT(cfg, 13));
  c->phi_unif_b = REAL(VECTOR_ELT(cfg, 14));
  c->K_IW_df = asReal(VECTOR_ELT(cfg, 15));
  c->K_IW_S = REAL(VECTOR_ELT(cfg, 16));
  c->nu_starting = dp(VECTOR_ELT(cfg, 17));
  c->nu_tuning = dp(VECTOR_ELT(cfg, 18));
  c->nu_unif_a = dp(VECTOR_ELT(cfg, 19));
  c->nu_unif_b = dp(VECTOR_ELT(cfg, 20));
  c->link = asInteger(VECTOR_ELT(cfg, 21));
  c->predict_tile = asInteger(VECTOR_ELT(cfg, 22));
  c->device = asInteger(VECTOR_ELT(cfg, 23));
  c->seed = (uint64_t)asReal(seed); /* drawn from R's RNG by the caller: honours set.seed */
  c->record_samples = 1;
  c->record_w = 0;
  c->n_streams = 0;
}

/* subsets back to back: coords n_s x 2 column-major, y / weights location-major, x (n_s q) x p */
static void read_problem(SEXP n_part, SEXP coords, SEXP y, SEXP weights, SEXP x, SEXP coords_test, SEXP q, SEXP p,
                         mk_problem* pr) {
  memset(pr, 0, sizeof *pr);
  pr->n_subsets = LENGTH(n_part);
  pr->subset_base = 0;
  pr->q = asInteger(q);
  pr->p = asInteger(p);
  pr->n_part = INTEGER(n_part);
  pr->coords = REAL(coords);
  pr->y = REAL(y);
  pr->weights = REAL(weights);
  pr->x = REAL(x);
  pr->n_test = isNull(coords_test) ? 0 : nrows(coords_test);
  pr->coords_test = dp(coords_test);
}

static int n_params(const mk_config* c, int np, int q) {
  return np + q * (q + 1) / 2 + q * (c->cov_model == MK_COV_MATERN ? 2 : 1);
}

/* MK.R:100-133 over the GPUs in `devices`: every subset's grids plus the combined grids.
 * combine: 0 = the reference's mean (MK.R:123-133), 1 = Weiszfeld W2 median.
 * Returns list(parameters = S x 200 x P, w.predict = S x 200 x q n_test, acceptance,
 *              result = 200 x P, result2 = 200 x q n_test). */
SEXP mk_r_fit(SEXP n_part, SEXP coords, SEXP y, SEXP weights, SEXP x, SEXP coords_test, SEXP q, SEXP p,
              SEXP cfg, SEXP seed, SEXP devices, SEXP report, SEXP combine) {
  mk_problem pr;
  mk_config c;
  read_problem(n_part, coords, y, weights, x, coords_test, q, p, &pr);
  read_config(cfg, seed, &c);
  const int S = pr.n_subsets, np = LENGTH(VECTOR_ELT(cfg, 5));
  const int P = n_params(&c, np, pr.q);
  const R_xlen_t C = (R_xlen_t)pr.q * pr.n_test;
  const int n_acc = P + 1; /* per batch: the p betas, the covariance parameters, the latent w */
  SEXP par = PROTECT(allocVector(REALSXP, (R_xlen_t)S * MK_N_LEVELS * P));
  SEXP wpr = PROTECT(allocVector(REALSXP, (R_xlen_t)S * MK_N_LEVELS * C));
  SEXP acc = PROTECT(allocVector(REALSXP, (R_xlen_t)S * c.n_batch * n_acc));
  SEXP r1 = PROTECT(allocMatrix(REALSXP, MK_N_LEVELS, P));
  SEXP r2 = PROTECT(allocMatrix(REALSXP, MK_N_LEVELS, (int)C));
  mk_outputs o;
  memset(&o, 0, sizeof o);
  o.parameters = REAL(par);
  o.w_predict = pr.n_test ? REAL(wpr) : NULL;
  o.acceptance = REAL(acc);
  mk_combined cb;
  memset(&cb, 0, sizeof cb);
  cb.result = REAL(r1);
  cb.result2 = pr.n_test ? REAL(r2) : NULL;
  cb.method = asInteger(combine);
  cb.max_iter = 100;
  cb.tol = 1e-12;
  progress_t pg = {asInteger(report), c.n_batch, c.batch_length, 0};
  if (mk_meta_fit(&pr, &c, INTEGER(devices), LENGTH(devices), r_progress, &pg, &o, &cb) != MK_OK) fail(5);
  SEXP res = PROTECT(allocVector(VECSXP, 5));
  SET_VECTOR_ELT(res, 0, par);
  SET_VECTOR_ELT(res, 1, wpr);
  SET_VECTOR_ELT(res, 2, acc);
  SET_VECTOR_ELT(res, 3, r1);
  SET_VECTOR_ELT(res, 4, r2);
  UNPROTECT(6);
  return res;
}

/* ---- spMvGLM / spPredict of one subset (MK.R:80-87) through a session kept alive between them */
static void session_finalizer(SEXP ptr) {
  mk_session* s = (mk_session*)R_ExternalPtrAddr(ptr);
  if (s) mk_session_destroy(s);
  R_ClearExternalPtr(ptr);
}

/* One subset: coords n x 2, y / weights location-major (n q), x (n q) x p; every chain state is
 * recorded (predict.tile > 0, burn.in = 1) for spPredict.  Returns list(p.beta.theta.samples
 * (n.samples x P), p.w.samples ((n q) x n.samples), acceptance (n.batch x (P + 1)), session). */
SEXP mk_r_spmvglm(SEXP coords, SEXP y, SEXP weights, SEXP x, SEXP q, SEXP cfg, SEXP seed, SEXP report) {
  mk_problem pr;
  mk_config c;
  SEXP n_part = PROTECT(ScalarInteger(nrows(coords)));
  read_problem(n_part, coords, y, weights, x, R_NilValue, q, ScalarInteger(ncols(x)), &pr);
  read_config(cfg, seed, &c);
  c.burn_in = 1;                         /* record every iteration's state: spPredict picks start..end */
  if (c.predict_tile <= 0) c.predict_tile = 65536;
  c.record_w = 1;
  const int n_samples = c.n_batch * c.batch_length;
  const int P = n_params(&c, pr.p, pr.q);
  const R_xlen_t N = (R_xlen_t)nrows(coords) * pr.q;
  mk_session* s = NULL;
  if (mk_session_create(&pr, &c, &s) != MK_OK) fail(1);
  SEXP ptr = PROTECT(R_MakeExternalPtr(s, install("mk_session"), R_NilValue));
  R_RegisterCFinalizerEx(ptr, session_finalizer, TRUE);   /* frees the device state on gc / exit */
  progress_t pg = {asInteger(report), c.n_batch, c.batch_length, 0};
  for (int it = 0; it < n_samples; it += c.batch_length) {
    if (mk_session_run(s, c.batch_length) != MK_OK) fail(2);
    if (r_progress(&pg, it + c.batch_length, n_samples)) {
      session_finalizer(ptr);
      UNPROTECT(2);
      Rf_error("spMvGLM interrupted after %d of %d iterations", it + c.batch_length, n_samples);
    }
  }
  SEXP smp = PROTECT(allocMatrix(REALSXP, n_samples, P));
  SEXP wsm = PROTECT(allocMatrix(REALSXP, (int)N, n_samples));
  SEXP acc = PROTECT(allocMatrix(REALSXP, c.n_batch, P + 1));
  mk_outputs o;
  memset(&o, 0, sizeof o);
  o.samples = REAL(smp);
  o.w_samples = REAL(wsm);
  o.acceptance = REAL(acc);
  if (mk_session_outputs(s, &o) != MK_OK) fail(5);
  SEXP res = PROTECT(allocVector(VECSXP, 4));
  SET_VECTOR_ELT(res, 0, smp);
  SET_VECTOR_ELT(res, 1, wsm);
  SET_VECTOR_ELT(res, 2, acc);
  SET_VECTOR_ELT(res, 3, ptr);
  UNPROTECT(6);
  return res;
}

/* spPredict(sp.obj, pred.coords, start, end): p.w.predictive.samples ((q n_test) x (end - start + 1)),
 * kriged from the recorded states of iterations start..end (1-based) of the spMvGLM session. */
SEXP mk_r_sppredict(SEXP session, SEXP coords_test, SEXP start, SEXP end, SEXP q) {
  mk_session* s = (mk_session*)R_ExternalPtrAddr(session);
  if (!s) Rf_error("libmk: the spMvGLM session was freed");
  const int n_test = nrows(coords_test), first = asInteger(start), last = asInteger(end);
  if (mk_session_set_test_sites(s, n_test, REAL(coords_test)) != MK_OK ||
      mk_session_set_kept_window(s, first, last) != MK_OK)
    fail(0);
  SEXP wp = PROTECT(allocMatrix(REALSXP, asInteger(q) * n_test, last - first + 1));
  mk_outputs o;
  memset(&o, 0, sizeof o);
  o.w_pred_samples = REAL(wp);
  if (mk_session_outputs(s, &o) != MK_OK) fail(1);
  UNPROTECT(1);
  return wp;
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

/* The process's HIP hardware queues: n > 0 the count HIP started with (another package started HIP
 * before .onLoad ran), n < 0 libmk reads GPU_MAX_HW_QUEUES itself (HIP starts after .onLoad set it). */
SEXP mk_r_hw_queues(SEXP n) {
  mk_set_hw_queues(asInteger(n));
  return R_NilValue;
}

/* TRUE when this process's HIP runtime already runs (it holds /dev/kfd open), checked without
 * starting it: .onLoad's GPU_MAX_HW_QUEUES can then no longer take effect. */
SEXP mk_r_hip_started(void) { return ScalarLogical(mk_hip_initialized() != 0); }

/* libmk's pooled HIP streams go while the runtime is alive (.onUnload, and R's exit finalizer). */
SEXP mk_r_shutdown(void) {
  mk_shutdown();
  return R_NilValue;
}

static const R_CallMethodDef call_methods[] = {
    {"mk_r_fit", (DL_FUNC)&mk_r_fit, 13},
    {"mk_r_spmvglm", (DL_FUNC)&mk_r_spmvglm, 8},
    {"mk_r_sppredict", (DL_FUNC)&mk_r_sppredict, 5},
    {"mk_r_combine", (DL_FUNC)&mk_r_combine, 4},
    {"mk_r_summary", (DL_FUNC)&mk_r_summary, 6},
    {"mk_r_glm", (DL_FUNC)&mk_r_glm, 5},
    {"mk_r_hw_queues", (DL_FUNC)&mk_r_hw_queues, 1},
    {"mk_r_hip_started", (DL_FUNC)&mk_r_hip_started, 0},
    {"mk_r_shutdown", (DL_FUNC)&mk_r_shutdown, 0},
    {NULL, NULL, 0}};

void R_init_mkgpu(DllInfo* dll) {
  R_registerRoutines(dll, NULL, call_methods, NULL, NULL);
  R_useDynamicSymbols(dll, FALSE);
}
