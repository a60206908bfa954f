/* libmk -- MI355X-native meta-kriging hot path (C ABI, no torch / R types).
 *
 * Drop-in boundary for the data-parallel core of MetaKriging_BinaryResponse.R:
 * the per-subset spMvGLM fits + spPredict kriging + 200-level quantile
 * summaries (the `foreach(i=1:n.core) %dopar% partitioned_spMvGLM(...)` at
 * MK.R:108, whose body is MK.R:46-96) and the quantile-average combine
 * (MK.R:119-133).  Conventions are R's: column-major fp64 matrices, int32
 * counts, location-major multivariate vectors (site i, outcome a at i*q + a),
 * caller-allocated outputs.  Every call returns 0 on success or a negative
 * MK_E* code; mk_last_error() gives the thread-local message.
 * See INTEGRATION.md for the R .Call glue that binds these entry points.
 */
#ifndef MK_H
#define MK_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MK_OK 0
#define MK_E_ARG (-1)      /* invalid argument (R: stop()) */
#define MK_E_HIP (-2)      /* HIP runtime failure */
#define MK_E_NOMEM (-3)    /* device allocation failed */
#define MK_E_NODEV (-4)    /* no HIP device */
#define MK_E_INTERRUPT (-5) /* the progress callback asked to stop (R: a user interrupt) */

#define MK_COV_EXPONENTIAL 0
#define MK_COV_MATERN 1
#define MK_LINK_LOGIT 0    /* spMvGLM's binomial family (MK.R:80-84), logistic p(y=1) (MK.R:160) */
#define MK_LINK_PROBIT 1   /* north-star extension: Phi link (no reference parity target)        */
#define MK_N_LEVELS 200    /* quantile(x, probs = seq(0.005, 1, 0.005)), MK.R:88 */

/* Subset data.  Replaces the globals Y*.part / X*.part / coords.part the
 * worker reads (MK.R:67-75) plus coords.test (MK.R:87, 108). */
typedef struct mk_problem {
  int32_t n_subsets;          /* subsets in this call (this GPU's shard)              */
  int32_t subset_base;        /* global index of subset 0 (selects its RNG stream)    */
  int32_t q;                  /* outcomes (MK.R:80: length of the formula list)       */
  int32_t p;                  /* regression coefficients, sum over outcomes           */
  const int32_t* n_part;      /* [n_subsets] sites per subset (MK.R:18)               */
  const double* coords;       /* concatenated per subset: n_s x 2 column-major        */
  const double* y;            /* concatenated per subset: n_s*q responses (counts)    */
  const double* weights;      /* concatenated per subset: n_s*q binomial trials       */
  const double* x;            /* concatenated per subset: (n_s*q) x p column-major    */
  int32_t n_test;             /* held-out sites (coords.test rows)                    */
  const double* coords_test;  /* n_test x 2 column-major                              */
} mk_problem;

/* spMvGLM arguments (MK.R:56-64, 80-85).  Tuning values are proposal
 * VARIANCES (spBayes amcmc semantics); beta_tuning is length p (the diagonal
 * of the t(chol(vcov)) matrix MK.R:55 builds). */
typedef struct mk_config {
  int32_t cov_model;          /* MK_COV_EXPONENTIAL (MK.R:84) or MK_COV_MATERN        */
  int32_t n_batch;            /* MK.R:57 */
  int32_t batch_length;       /* MK.R:58 */
  double accept_rate;         /* MK.R:83 */
  int32_t burn_in;            /* first kept sample, 1-based (MK.R:85-89: start = burn.in) */
  const double* beta_starting;  /* [p]  MK.R:54 */
  const double* beta_tuning;    /* [p]  MK.R:55 (diagonal) */
  const double* phi_starting;   /* [q]  MK.R:60 */
  const double* phi_tuning;     /* [q]  MK.R:61 */
  const double* A_starting;     /* [q(q+1)/2] lower triangle of A, col-major (MK.R:56) */
  const double* A_tuning;       /* [q(q+1)/2] MK.R:61 */
  const double* nu_starting;    /* [q] Matern only, else NULL */
  const double* nu_tuning;      /* [q] Matern only, else NULL */
  double w_starting;            /* MK.R:60 */
  double w_tuning;              /* MK.R:62 */
  const double* phi_unif_a;     /* [q] MK.R:63 */
  const double* phi_unif_b;     /* [q] */
  const double* nu_unif_a;      /* [q] Matern only */
  const double* nu_unif_b;      /* [q] Matern only */
  double K_IW_df;               /* MK.R:64 */
  const double* K_IW_S;         /* [q*q] col-major, MK.R:64 */
  uint64_t seed;                /* Philox stream seed (the R glue draws it from R's RNG) */
  int32_t record_samples;       /* keep p.beta.theta.samples (n_samples x P)            */
  int32_t record_w;             /* keep p.w.samples ((n_s*q) x n_samples)               */
  int32_t device;               /* HIP device ordinal                                    */
  int32_t n_streams;            /* subset groups run on this many HIP streams (0: default 1);
                                   results do not depend on it                          */
  int32_t predict_tile;         /* 0 (or >= n_test): spPredict fused into the kept iterations.
                                   Else the kept chain states are recorded and the kriging
                                   runs after the fit over tiles of this many test sites, so
                                   (q*n_test) x kept draws per subset never coexist (cfg5:
                                   1M sites); results are identical either way            */
  int32_t link;                 /* MK_LINK_LOGIT (the reference) or MK_LINK_PROBIT              */
} mk_config;

/* Caller-allocated outputs; any pointer may be NULL to skip it.
 * P = p + q(q+1)/2 + q (+ q for Matern); kept = n_batch*batch_length - burn_in + 1. */
typedef struct mk_outputs {
  double* parameters;   /* [n_subsets] x (200 x P) column-major: obj[[i]]$parameters (MK.R:89)  */
  double* w_predict;    /* [n_subsets] x (200 x q*n_test) column-major: obj[[i]]$w.predict      */
  double* samples;      /* [n_subsets] x (n_samples x P) column-major: m.1$p.beta.theta.samples  */
  double* w_samples;    /* [n_subsets] x ((n_s*q) x n_samples) column-major: m.1$p.w.samples    */
  double* w_pred_samples; /* [n_subsets] x ((q*n_test) x kept): m.s.pred$p.w.predictive.samples */
  double* acceptance;   /* [n_subsets] x (n_batch x (p + n_theta + 1)): per-batch accept rates,
                           last column = mean over the latent w                                  */
  double* w_predict_sum; /* 200 x (q*n_test): w_predict summed over this call's subsets in subset
                           order -- this shard's term of the combine (MK.R:129-132) without the
                           per-subset grids on the host                                          */
} mk_outputs;

typedef struct mk_session mk_session;

/* ---- batched meta-kriging path (replaces foreach %dopar% at MK.R:108) ---- */
/* Upload the shard to HBM and initialise every chain (no MCMC yet). */
int mk_session_create(const mk_problem* prob, const mk_config* cfg, mk_session** out);
/* Advance every chain by n_iter iterations (returns after the device is idle). */
int mk_session_run(mk_session* s, int32_t n_iter);
/* Iterations done so far. */
int32_t mk_session_iteration(const mk_session* s);
/* Test sites per kriging tile in use (0: fused kriging).  A tiled session takes the configured
 * predict_tile, or the largest tile (halved in 256-site steps) whose kriging buffers fit in HBM;
 * hosts replaying tile by tile (mk_session_tile_grids) step by this value. */
int32_t mk_session_predict_tile(const mk_session* s);
/* One subset's chain state after the iterations done so far, in spMvGLM's MH parameter order:
 * beta [p]; theta [n_theta] (A lower-tri col-major with log diagonal | logit phi | logit nu);
 * w [n_s q] location-major; tune [p + n_theta + n_s q] log proposal sds; accept [same] accept counts
 * of the current amcmc batch.  Any pointer may be NULL.  (Resuming the chain on another host: the CPU
 * baseline of bench.py times the oracle over the window the device timed.) */
int mk_session_chain_state(mk_session* s, int32_t subset, double* beta, double* theta, double* w, double* tune,
                           double* accept);
/* Launch schedule (results are the same chain either way): mode 1 = lookahead
 * (the next iteration's phi candidates are factored while this iteration's inverse and latent
 * sweep run; Matern: the nu step follows the phi decision; n_streams <= 1), 0 = sequential, -1 = default (lookahead where
 * eligible; env MK_LOOKAHEAD=0/1 overrides the default).  Before the first mk_session_run only.
 * mk_session_lookahead returns 1 when the lookahead schedule is in use. */
int mk_session_set_lookahead(mk_session* s, int32_t mode);
int32_t mk_session_lookahead(const mk_session* s);
/* Quantile summaries + optional sample copies (requires all iterations done
 * for parameters / w_predict). */
int mk_session_outputs(mk_session* s, mk_outputs* out);
/* spPredict after spMvGLM without refitting (spPredict(m.1, coords.test, ...), MK.R:87): a session
 * created with predict_tile > 0 keeps every kept chain state (burn_in = 1 keeps all of them);
 * mk_session_set_test_sites replaces its test sites (n_test x 2 column-major) and
 * mk_session_set_kept_window(first, last) restricts the kriging replay of the next
 * mk_session_outputs to iterations first..last (1-based, burn_in <= first <= last <= n.samples;
 * spPredict's start / end).  The draws are those a session with burn_in = first would make. */
int mk_session_set_test_sites(mk_session* s, int32_t n_test, const double* coords_test);
int mk_session_set_kept_window(mk_session* s, int32_t first, int32_t last);
/* After all iterations: the shard's 200-level grids, [n_subsets] x (200 x C) column-major -- which 0:
 * obj[[i]]$parameters (C = P), which 1: obj[[i]]$w.predict (C = q*n_test; fused sessions, tiled ones
 * use mk_session_tile_grids) -- into out: host memory, or HBM of the session's device when
 * device_out != 0 (e.g. the send buffer of a device-resident combine; no host round trip). */
int mk_session_grids(mk_session* s, int32_t which, double* out, int32_t device_out);
/* Tiled sessions (predict_tile > 0), after all iterations: the 200-level w.predict grids of the test
 * sites of tile [t0, t0 + Tc) (Tc = min(predict_tile, n_test - t0), t0 a multiple of predict_tile),
 * every subset: [n_subsets] x (200 x q*Tc) column-major, into out -- host memory, or HBM of the
 * session's device when device_out != 0 (e.g. an RCCL send buffer).  Replays that tile's kriging
 * only (spPredict, MK.R:87-89), so a host can combine tile by tile: at configs[4] the per-subset
 * grids of all 1M sites never coexist. */
int mk_session_tile_grids(mk_session* s, int32_t t0, double* out, int32_t device_out);
/* Per-kernel timing (HIP events on the launching streams): launches, total ms and
 * algorithmic flops per kernel kind.  0: the 128-tile column-update launches -- k_chol_update_trsm
 * (column k's update of tiles k+1.. with the panel solve fused in its epilogue, plus the next diagonal
 * tile's update by panels < k; the default schedule) and k_chol_update<128> (unfused and split
 * schedules); 1 diagonal tile k_chol_diag (in the fused schedule it also applies the rank-128
 * diagonal correction by panel k-1, priced here); 2 panel trsm k_chol_trsm (panel 0, and the unfused
 * schedules); 3 latent sweep; 4 R^-1 diagonal tiles; 5 whole iterations; 6 inverse levels
 * k_inv_level (flops per level over the accepted factors, n_s^3/3 per factor with kind 1's diagonal
 * inverses); 7 kind 0's 64/32-sub-tile instances; 8 kinds 0 + 7 with overlapping launches counted
 * once; 9 kriging GEMM k_pred_var; 10 candidate covariance assembly; 11 latent sweeps the
 * multi-workgroup kernel refused admission and its fallback ran -- launches = (subset, iteration)
 * count, no timing; 12 tiles of a tiled session kriged by phi interpolation -- launches = tiles, flops
 * = exact kriging-variance evaluations, total_ms = the largest per-tile check difference (not a time);
 * 13 tiles whose check failed and were replayed exactly -- launches, total_ms = the largest failing
 * difference).  Flops are algorithmic, not executed: GEMM tiles 2 m n k, the diagonal tile's
 * update as a SYRK, solves and inverse products over their triangles.  mk_session_profile(s, enable)
 * before mk_session_run: enable 0 = off, 1 = every kind, otherwise a mask with bit (1 + kind) per kind
 * bracketed (e.g. 2 << 0 = the panel update only; fewer events, less overhead). */
int mk_session_profile(mk_session* s, int32_t enable);
/* Bracket only the launches of every `every`-th iteration (iteration index % every == 0; default 1:
 * all).  At small shards per-launch events cost measurably (32 subsets: ~4 % of the rate, 250: 0.5 %);
 * a sample keeps the per-launch averages and costs a fraction of that. */
int mk_session_profile_every(mk_session* s, int32_t every);
int mk_session_kernel_stats(const mk_session* s, int32_t which, int64_t* launches, double* total_ms, double* flops);
void mk_session_destroy(mk_session* s);
/* Sessions alive in this process (a failed mk_session_create leaves none behind). */
int32_t mk_session_count(void);

/* One-shot convenience: create, run n_batch*batch_length iterations, outputs, destroy. */
int mk_fit_predict_batched(const mk_problem* prob, const mk_config* cfg, mk_outputs* out);

/* ---- the whole node (replaces makeCluster + foreach %dopar% + the combine, MK.R:100-133) ----
 * The K subsets of prob are cut into n_devices balanced contiguous blocks [floor(rK/G),
 * floor((r+1)K/G)); block r runs as one session on devices[r], one host thread per block, with
 * global subset indices (prob->subset_base + its first subset), so every chain equals the
 * one-device chain.  The chains advance one amcmc batch at a time on every device; between
 * batches the calling thread calls progress (if not NULL) -- spBayes's n.report output and R's
 * interrupt check -- and stops the fit (MK_E_INTERRUPT, every device freed) when it returns
 * nonzero.  cfg->device is ignored.
 * The combine is device to device: every block's 200-level grids stay in HBM; an all-to-all hands
 * device j all K subsets' grids for its block of columns (RCCL send/recv over xGMI when the devices
 * are distinct; device copies when a device is listed more than once -- several shards on one GPU),
 * device j combines them in global subset order -- MK.R:123-133's sequential mean, bit-identical
 * to one device, or the Weiszfeld W2 median -- and its combined columns go to the host.  Tiled
 * kriging (predict_tile) exchanges the grids of one test-site tile at a time, so the configs[4]
 * combine of 1M sites needs K x 200 x q*tile doubles per device, not K x 200 x q*n_test.
 * out (optional, any field NULL): the per-subset outputs of all K subsets as mk_session_outputs
 * lays them out; out->w_predict_sum = the sequential sum of all K w.predict grids. */
#define MK_COMBINE_MEAN 0     /* MK.R:123-133 */
#define MK_COMBINE_MEDIAN 1   /* north-star extension: per column Weiszfeld geometric median in W2 */
typedef struct mk_combined {
  double* result;     /* 200 x P: the combined parameter grid (MK.R:127 result), or NULL            */
  double* result2;    /* 200 x (q*n_test): the combined w.predict grid (MK.R:133 result2), or NULL  */
  int32_t method;     /* MK_COMBINE_MEAN or MK_COMBINE_MEDIAN                                      */
  int32_t max_iter;   /* MEDIAN: Weiszfeld iterations (<= 0: 100)                                   */
  double tol;         /* MEDIAN: convergence tolerance (< 0: 1e-12)                                 */
  int32_t exchange;   /* out: 1 = RCCL, 0 = device copies                                           */
  int32_t comm_ranks; /* out: ranks of the exchange (RCCL: ncclCommCount of the communicators; copies:
                       * the number of device blocks)                                               */
} mk_combined;
/* Progress between batches: iterations done so far (a multiple of batch_length) of n_samples. */
typedef int (*mk_progress_fn)(void* user, int32_t iterations, int32_t n_samples);
int mk_meta_fit(const mk_problem* prob, const mk_config* cfg, const int32_t* devices, int32_t n_devices,
                mk_progress_fn progress, void* user, mk_outputs* out, mk_combined* comb);

/* ---- combine (MK.R:123-133): out = (grid_1 + ... + grid_K) / K, sequential order ---- */
int mk_combine(const double* grids, int32_t K, int64_t grid_len, double* out, int32_t device);

/* The sum only (no 1/K): one shard's term of the combine, or the rank-ordered sum of shard terms. */
int mk_combine_sum(const double* grids, int32_t K, int64_t grid_len, double* out, int32_t device);
/* Device-resident form for the multi-GPU combine (grids already in HBM, e.g. RCCL receive
 * buffers): d_out[e] = sum_k d_grids[k*grid_len + e] in k order, divided by K when mean != 0.
 * stream: a hipStream_t (NULL = the legacy default stream); returns after the kernel is queued. */
int mk_combine_device(const double* d_grids, int32_t K, int64_t grid_len, double* d_out, int32_t mean,
                      int32_t device, void* stream);

/* ---- combine extension (north star; not in the reference, which averages at MK.R:123-133):
 * per column, the Weiszfeld geometric median of the K subset quantile functions in the
 * Wasserstein-2 metric, started from the mean.  grids: K x (n_levels x n_cols) column-major;
 * out: n_levels x n_cols; iters (optional): [n_cols] iterations used.  n_levels <= 256. ---- */
int mk_combine_median(const double* grids, int32_t K, int32_t n_levels, int64_t n_cols, int32_t max_iter,
                      double tol, double* out, int32_t* iters, int32_t device);
/* Device-resident form (grids, out, iters in HBM; stream as in mk_combine_device). */
int mk_combine_median_device(const double* d_grids, int32_t K, int32_t n_levels, int64_t n_cols, int32_t max_iter,
                             double tol, double* d_out, int32_t* d_iters, int32_t device, void* stream);

/* ---- post-combine steps (MK.R:136-165) ---- */
typedef struct mk_summary {
  double* sample_par;    /* samplesize x P   SamplePar  (MK.R:145)                 */
  double* sample_w;      /* samplesize x C   Samplew    (MK.R:146)                 */
  double* p_sample;      /* samplesize x C   p.sample   (MK.R:156-161)             */
  double* w_quant;       /* 3 x C            w.quant    (MK.R:164)                 */
  double* param_quant;   /* 3 x P            param.quant (MK.R:165)                */
  double* p_quant;       /* 3 x C            quantiles of p.sample (extension)     */
  int32_t* index;        /* samplesize       sampleparIndex - 1 (MK.R:141)         */
} mk_summary;
/* result: 200 x P combined parameter grid (betas first, MK.R:159); result2: 200 x C combined
 * w.predict grid; x_test: C x p (p <= P).  Any output pointer may be NULL. */
int mk_posterior_summary(const double* result, int32_t P, const double* result2, int64_t C,
                         const double* x_test, int32_t p, int32_t samplesize, uint64_t seed,
                         mk_summary* out, int32_t device);
/* As mk_posterior_summary, plus: index (optional, [samplesize], 1-based) is sampleparIndex drawn
 * by the caller -- the R glue passes R's own sample(seq(1, length(Xout), 1), samplesize,
 * replace=TRUE) (MK.R:141), so the draws follow R's RNG stream; NULL draws it from Philox(seed).
 * link: MK_LINK_LOGIT (MK.R:160) or MK_LINK_PROBIT for p.sample. */
int mk_posterior_summary_ex(const double* result, int32_t P, const double* result2, int64_t C,
                            const double* x_test, int32_t p, int32_t samplesize, uint64_t seed,
                            const int32_t* index, int32_t link, mk_summary* out, int32_t device);

/* ---- glm start values (MK.R:53-55), once on the full data: binomial-logit IRLS with
 * glm.fit's rules (mustart init, |dev - devold|/(|dev| + 0.1) < epsilon, maxit).
 * y: counts, weights: trials (n each), x: n x p column-major (p <= 8).
 * coef: [p]; vcov: p x p (dispersion 1); iters (optional). ---- */
int mk_glm_binomial(const double* y, const double* weights, const double* x, int64_t n, int32_t p,
                    double epsilon, int32_t maxit, double* coef, double* vcov, int32_t* iters,
                    int32_t device);
/* binomial(link = "probit") too: R's make.link("probit") (eta clamped to +-qnorm(eps) in linkinv,
 * mu.eta = max(dnorm(eta), eps), linkfun = qnorm). link = MK_LINK_LOGIT is mk_glm_binomial. */
int mk_glm_binomial_link(const double* y, const double* weights, const double* x, int64_t n, int32_t p,
                         int32_t link, double epsilon, int32_t maxit, double* coef, double* vcov,
                         int32_t* iters, int32_t device);

/* ---- partition (MK.R:15-41) with R's own RNG stream, host side ----
 * After `set.seed(seed)` under R >= 3.6.0 defaults (Mersenne-Twister, Rejection sampling),
 * the reference's loop `index.part[[i]] <- sample(a, n.part[i]); a <- setdiff(a, ...)`.
 * n_part: [n_core] out (MK.R:17-18); index_out: [n] out, subset i's 1-based indices at offset
 * n_part[0] + ... + n_part[i-1], in R's draw order.  Replaces nothing on the R side (R keeps
 * its own partition); it lets a non-R host fit exactly the subsets an R session fits. */
int mk_partition_r(int32_t n, int32_t n_core, int32_t seed, int32_t* n_part, int32_t* index_out);
/* sample.int(n, size) (without replacement, 1-based) right after set.seed(seed). */
int mk_r_sample(int32_t seed, int32_t n, int32_t size, int32_t* out);
/* sample.int(n, size, replace = TRUE) right after set.seed(seed): MK.R:141's sampleparIndex
 * (n = length(Xout) = 996) as an R session that set the seed just before would draw it. */
int mk_r_sample_replace(int32_t seed, int32_t n, int32_t size, int32_t* out);

/* ---- exposed kernels for parity tests ---- */
/* R_k = correlation(coords_k) (n x n column-major) for S point sets of n sites, computed by
 * the sampler's own candidate kernel (k_cov_candidate: exponential, or Matern with the binned
 * Temme/CF2 Bessel-K evaluation) -- the covariance-assembly arithmetic the chains use. */
int mk_correlation_batched(const double* coords, int32_t S, int32_t n, const double* phi, const double* nu,
                           int32_t cov_model, double* R_out, int32_t device);
/* Cholesky (lower) + log-determinant (+ optional inverse) of S SPD n x n matrices. */
int mk_cholesky_batched(const double* A, int32_t S, int32_t n, double* L_out, double* logdet_out,
                        double* inv_out, int32_t device);

/* Hardware queues the process's HIP runtime was started with (GPU_MAX_HW_QUEUES when HIP first
 * initialised; HIP's default is 4).  The lookahead schedule adds a kriging stream and a CU-masked
 * main stream only when there are >= 8 (streams beyond the queue count share queues and serialise,
 * DESIGN.md 4.2).  A host that knows HIP started before its own setting took effect (e.g. torch
 * first) passes the real count; n < 0 restores the default: GPU_MAX_HW_QUEUES from the environment. */
int mk_set_hw_queues(int32_t n);

/* Whether this process's HIP runtime has already started (the process holds /dev/kfd open), without
 * starting it: a host that sets GPU_MAX_HW_QUEUES first checks whether the setting can still take
 * effect (the R package's .onLoad; libmk itself has not touched HIP when this is called). */
int mk_hip_initialized(void);

/* Drains and destroys libmk's idle pooled HIP streams (CU-masked and priority queues included) while
 * the runtime is alive; streams of sessions still open are destroyed with them.  libmk registers it
 * with atexit after its first stream; hosts call it from their own exit hooks too (Python atexit,
 * R .onUnload).  Idempotent; libmk stays usable afterwards (new streams are no longer pooled). */
void mk_shutdown(void);

/* Stall watchdog: when seconds > 0 every launch is followed by a progress-word store into pinned host
 * memory, and a C-ABI call still running after `seconds` prints (stderr, and MK_WATCHDOG_LOG=<path>
 * if set) every stream with work outstanding and the kernel it is on.  0 = off (default; the
 * environment variable MK_WATCHDOG=<seconds> sets it at load). */
int mk_set_watchdog(int32_t seconds);

const char* mk_last_error(void);
int mk_device_count(void);
/* Free and total HBM of a device (hipMemGetInfo), e.g. to size shards or check for leaks. */
int mk_device_memory(int32_t device, int64_t* free_bytes, int64_t* total_bytes);

#ifdef __cplusplus
}
#endif
#endif /* MK_H */
