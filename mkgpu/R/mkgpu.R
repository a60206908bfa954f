# R side of the mkgpu package: the reference's worker loop and combine, run by libmk.
# Uncompiled in the build image (R is not installed there); INTEGRATION.md walks through it.
#
# MetaKriging_BinaryResponse.R (MK.R) lines this replaces:
#   MK.R:80-84    m.1 <- spMvGLM(formula = list(...), coords, weights, starting, tuning, priors,
#                                amcmc, cov.model, n.report)          -> mk_spMvGLM(same arguments)
#   MK.R:87       m.s.pred <- spPredict(m.1, coords.test, x.test, start, end)
#                                                                     -> mk_spPredict(same arguments)
#   MK.R:100-114  cl <- makeCluster(n.core); obj <- foreach(i = 1:n.core, ...) %dopar%
#                 partitioned_spMvGLM(i, ...)
#                 -> obj <- mk_meta_fit(y, x, weight, q, n.part, index.part, coords, coords.test,
#                                       devices = 0:7)    (every GPU of the node, one call)
#   MK.R:123-133  result / result2 as the mean of the subset grids -> mk_combine(obj)
#   MK.R:136-165  resampling, p(y = 1) and quantiles              -> mk_posterior_summary(...)
# The worker's statistics that R computes before spMvGLM stay in R (MK.R:53-64): glm start
# values (or mk_glm_start on the device), starting / tuning / priors, n.batch, batch.length.
# The MCMC runs one amcmc batch at a time: spBayes's "Batch: b of n.batch" line every n.report
# batches, and Ctrl-C between batches stops the fit and frees the GPUs.

# Location-major rows of subset idx: site i, outcome a at (i - 1) * q + a (MK.R:67-75 layout).
.mk_rows <- function(idx, q) as.vector(t(outer((idx - 1) * q, 1:q, "+")))

# Coordinates as libmk reads them: a numeric n x 2 matrix (a data.frame is coerced, not trusted).
.mk_coords <- function(coords, what) {
  m <- as.matrix(coords)
  if (ncol(m) != 2L) stop(sprintf("%s must have 2 columns", what))
  storage.mode(m) <- "double"
  m
}

# glm((y / weight) ~ x - 1, weights = rep(weight, n q), family = "binomial") (MK.R:53) and the
# diagonal of t(chol(vcov(fit))) (MK.R:55).  device = NULL: R's own glm; else libmk's IRLS.
mk_glm_start <- function(y, x, weight, link = c("logit", "probit"), device = NULL) {
  link <- match.arg(link)
  if (is.null(device)) {
    fit <- glm((y / weight) ~ x - 1, weights = rep(weight, length(y)), family = binomial(link = link))
    return(list(beta = coefficients(fit), tuning = diag(t(chol(vcov(fit))))))
  }
  res <- .Call("mk_r_glm", as.double(y), as.double(rep(weight, length(y))), as.matrix(x) * 1.0,
               as.integer(link == "probit"), as.integer(device))
  list(beta = res[[1]], tuning = diag(t(chol(res[[2]]))))
}

# The sampler settings list the glue reads (MK.R:56-64, 80-85), in mk_r.c's read_config order.
.mk_cfg <- function(q, beta, beta.tuning, n.batch, batch.length, accept.rate, burn.in, cov.model, link,
                    predict.tile, device, phi.starting = rep(3 / 0.5, q), phi.tuning = rep(1, q),
                    A.starting = diag(1, q)[lower.tri(diag(1, q), TRUE)], A.tuning = rep(0.1, length(A.starting)),
                    w.starting = 0, w.tuning = 0.5, phi.a = rep(3 / 0.75, q), phi.b = rep(3 / 0.25, q),
                    K.df = q, K.S = diag(0.1, q), nu.starting = 0.5, nu.tuning = 0.1, nu.a = 0.1, nu.b = 2) {
  matern <- cov.model == "matern"
  cfg <- list(as.integer(matern), as.integer(n.batch), as.integer(batch.length), as.double(accept.rate),
              as.integer(burn.in), as.double(beta), as.double(beta.tuning),
              as.double(rep_len(phi.starting, q)), as.double(rep_len(phi.tuning, q)), as.double(A.starting),
              as.double(rep_len(A.tuning, length(A.starting))), as.double(w.starting), as.double(w.tuning),
              as.double(rep_len(phi.a, q)), as.double(rep_len(phi.b, q)), as.double(K.df), as.matrix(K.S) * 1.0,
              if (matern) as.double(rep_len(nu.starting, q)) else NULL,
              if (matern) as.double(rep_len(nu.tuning, q)) else NULL,
              if (matern) as.double(rep_len(nu.a, q)) else NULL, if (matern) as.double(rep_len(nu.b, q)) else NULL,
              as.integer(link == "probit"), as.integer(predict.tile), as.integer(device))
  cfg
}

# spMvGLM's amcmc tuning is one scalar per beta: the diagonal of a tuning matrix (MK.R:55 passes
# t(chol(vcov))).
.mk_diag <- function(t) if (is.matrix(t)) diag(t) else as.double(t)

# The foreach / partitioned_spMvGLM loop of MK.R:100-114 for every subset at once over the GPUs in
# `devices` (libmk shards the subsets, one host thread per GPU, and combines the grids device to
# device: RCCL over xGMI).  Returns a list of K list(parameters = 200 x P, w.predict =
# 200 x q n_test, acceptance) -- the shape partitioned_spMvGLM returns (MK.R:89) -- with the
# combined grids (MK.R:127, 133; combine = "median": the Weiszfeld extension) as attribute
# "combined", which mk_combine(obj) returns without recomputing.
mk_meta_fit <- function(y, x, weight, q, n.part, index.part, coords, coords.test,
                        n.batch = 100, batch.length = 50, accept.rate = 0.43,
                        cov.model = c("exponential", "matern"), link = c("logit", "probit"),
                        predict.tile = 0L, devices = 0L, glm.on.device = FALSE, n.report = 10,
                        combine = c("mean", "median")) {
  cov.model <- match.arg(cov.model)
  link <- match.arg(link)
  combine <- match.arg(combine)
  coords <- .mk_coords(coords, "coords")
  coords.test <- .mk_coords(coords.test, "coords.test")
  st <- mk_glm_start(y, x, weight, link, if (glm.on.device) devices[1] else NULL)   # MK.R:53-55
  n.samples <- n.batch * batch.length
  cfg <- .mk_cfg(q, st$beta, st$tuning, n.batch, batch.length, accept.rate,
                 as.integer(0.75 * n.samples),                                       # MK.R:85 burn.in
                 cov.model, link, predict.tile, devices[1])
  S <- length(n.part)
  res <- .Call("mk_r_fit", as.integer(n.part),
               unlist(lapply(index.part, function(i) as.vector(coords[i, ]))),
               unlist(lapply(index.part, function(i) as.double(y[.mk_rows(i, q)]))),
               unlist(lapply(index.part, function(i) rep(as.double(weight), length(i) * q))),
               unlist(lapply(index.part, function(i) as.vector(x[.mk_rows(i, q), , drop = FALSE] * 1.0))),
               coords.test, as.integer(q), ncol(x), cfg,
               floor(runif(1) * 2^52),                                               # honours set.seed
               as.integer(devices), as.integer(n.report), as.integer(combine == "median"))
  P <- length(res[[1]]) / (S * 200)
  C <- length(res[[2]]) / (S * 200)
  obj <- lapply(seq_len(S), function(k) list(
    parameters = matrix(res[[1]][(k - 1) * 200 * P + 1:(200 * P)], 200, P),
    w.predict = matrix(res[[2]][(k - 1) * 200 * C + seq_len(200 * C)], 200, C),
    acceptance = matrix(res[[3]][(k - 1) * n.batch * (P + 1) + 1:(n.batch * (P + 1))], n.batch, P + 1)))
  attr(obj, "combined") <- list(result = res[[4]], result2 = res[[5]], method = combine)
  obj
}

# MK.R:123-133: result = mean of obj[[k]]$parameters, result2 = mean of obj[[k]]$w.predict, in
# the same sequential summation order (bit-identical to the R loop).  An obj from mk_meta_fit
# already carries them (combined on the GPUs).
mk_combine <- function(obj, device = 0L) {
  cb <- attr(obj, "combined")
  if (!is.null(cb) && identical(cb$method, "mean")) return(list(result = cb$result, result2 = cb$result2))
  K <- length(obj)
  one <- function(field) {
    g <- unlist(lapply(obj, function(o) as.vector(o[[field]])))
    m <- .Call("mk_r_combine", g, as.integer(K), as.double(length(obj[[1]][[field]])), as.integer(device))
    matrix(m, nrow(obj[[1]][[field]]))
  }
  list(result = one("parameters"), result2 = one("w.predict"))
}

# spMvGLM(formula, coords, weights, starting, tuning, priors, amcmc, cov.model, n.report) of one
# subset, as MK.R:80-84 calls it: formula is a list of `Y ~ X - 1` formulas (one per outcome,
# evaluated where they were written), weights an n x q matrix of binomial trials, starting /
# tuning / priors / amcmc spBayes's lists.  Returns spBayes's fields p.beta.theta.samples
# (n.samples x P, the reported columns beta | K lower triangle | phi [| nu]), p.w.samples
# ((n q) x n.samples) and acceptance, plus the device session spPredict krigs from (every
# iteration's chain state is kept in HBM; it is freed with the object).
mk_spMvGLM <- function(formula, coords, weights, starting, tuning, priors, amcmc,
                       cov.model = c("exponential", "matern"), family = "binomial", n.report = 100,
                       link = c("logit", "probit"), device = 0L) {
  cov.model <- match.arg(cov.model)
  link <- match.arg(link)
  if (family != "binomial") stop("error: family must be binomial")
  if (is.null(amcmc)) stop("error: this build implements the amcmc (adaptive) sampler, as MK.R:83 uses")
  if (!is.list(formula)) formula <- list(formula)
  q <- length(formula)
  coords <- .mk_coords(coords, "coords")
  n <- nrow(coords)
  Y <- lapply(formula, function(f) {
    mf <- model.frame(f, environment(f))
    list(y = as.double(model.response(mf)), x = model.matrix(attr(mf, "terms"), mf))
  })
  p.a <- vapply(Y, function(o) ncol(o$x), 1L)
  p <- sum(p.a)
  y <- numeric(n * q)
  X <- matrix(0, n * q, p)
  off <- 0
  for (a in seq_len(q)) {
    if (length(Y[[a]]$y) != n) stop("error: every outcome needs the same number of locations")
    y[seq(a, n * q, by = q)] <- Y[[a]]$y                           # location-major (site i, outcome a)
    X[seq(a, n * q, by = q), off + seq_len(p.a[a])] <- Y[[a]]$x
    off <- off + p.a[a]
  }
  wt <- as.double(t(matrix(weights, n, q)))                         # location-major
  if (is.null(starting$beta) || is.null(tuning$beta)) stop("error: beta must be specified in starting and tuning")
  if (is.null(priors$phi.Unif) || is.null(priors$K.IW)) stop("error: phi.Unif and K.IW must be specified in priors")
  n.batch <- amcmc$n.batch
  batch.length <- amcmc$batch.length
  accept.rate <- if (is.null(amcmc$accept.rate)) 0.43 else amcmc$accept.rate
  cfg <- .mk_cfg(q, starting$beta, .mk_diag(tuning$beta), n.batch, batch.length, accept.rate, 1L, cov.model, link,
                 0L, device, phi.starting = starting$phi, phi.tuning = tuning$phi, A.starting = starting$A,
                 A.tuning = tuning$A, w.starting = starting$w[1], w.tuning = tuning$w[1],
                 phi.a = priors$phi.Unif[[1]], phi.b = priors$phi.Unif[[2]], K.df = priors$K.IW[[1]],
                 K.S = priors$K.IW[[2]], nu.starting = starting$nu, nu.tuning = tuning$nu,
                 nu.a = priors$nu.Unif[[1]], nu.b = priors$nu.Unif[[2]])
  res <- .Call("mk_r_spmvglm", coords, y, wt, X, as.integer(q), cfg, floor(runif(1) * 2^52),
               as.integer(n.report))
  ntri <- q * (q + 1) / 2
  cn <- c(paste0("beta.", seq_len(p)), paste0("K[", seq_len(ntri), "]"), paste0("phi[", seq_len(q), "]"),
          if (cov.model == "matern") paste0("nu[", seq_len(q), "]"))
  colnames(res[[1]]) <- cn
  structure(list(p.beta.theta.samples = res[[1]], p.w.samples = res[[2]], acceptance = res[[3]],
                 n.samples = n.batch * batch.length, q = q, session = res[[4]]), class = "mk_spMvGLM")
}

# spPredict(sp.obj, pred.coords, pred.covars, start, end, thin) as MK.R:87 calls it:
# p.w.predictive.samples ((q n_test) x kept, location-major rows) kriged from the recorded chain
# states of iterations start..end (no refit).  pred.covars is accepted for the reference's
# signature; the latent field's predictive draws (the only output MK.R:89 uses) do not need it.
mk_spPredict <- function(sp.obj, pred.coords, pred.covars = NULL, start = 1, end = sp.obj$n.samples, thin = 1) {
  if (!inherits(sp.obj, "mk_spMvGLM")) stop("error: sp.obj must come from mk_spMvGLM")
  start <- as.integer(start)
  end <- as.integer(end)
  if (start < 1L || end < start || end > sp.obj$n.samples) stop("error: invalid start/end")
  wp <- .Call("mk_r_sppredict", sp.obj$session, .mk_coords(pred.coords, "pred.coords"), start, end,
              as.integer(sp.obj$q))
  list(p.w.predictive.samples = wp[, seq(1, ncol(wp), by = thin), drop = FALSE])
}

# MK.R:136-165 on the combined grids.  The resample index is drawn here by R itself, exactly as
# MK.R:141 does (sample(seq(1, length(Xout), 1), samplesize, replace = TRUE)), so a session that
# called set.seed gets the reference's draws; the device does the linear interpolation, the
# logistic (or probit) transform and the 2.5 / 50 / 97.5 % quantiles.
mk_posterior_summary <- function(result, result2, x.test, samplesize = 1000, n.out = 996,
                                 link = c("logit", "probit"), device = 0L) {
  link <- match.arg(link)
  index <- sample(seq(1, n.out, 1), samplesize, replace = TRUE)                  # MK.R:141
  res <- .Call("mk_r_summary", result, result2, as.matrix(x.test) * 1.0, as.integer(index),
               as.integer(link == "probit"), as.integer(device))
  names(res) <- c("SamplePar", "Samplew", "p.sample", "w.quant", "param.quant")
  res
}

# libmk's lookahead schedule runs up to five HIP streams; HIP reads its hardware-queue count
# (default 4, streams beyond it share queues) once, when it starts.  If HIP has not started yet
# (libmk has not touched it; mk_hip_initialized checks /dev/kfd without starting it) the variable
# is raised to 8 here and libmk reads it itself.  If another package started HIP first, the
# setting comes too late: libmk is told the count HIP started with -- the variable as it was, or
# HIP's default 4 -- and runs three streams instead of five rather than share queues.
.onLoad <- function(libname, pkgname) {
  q <- suppressWarnings(as.integer(Sys.getenv("GPU_MAX_HW_QUEUES", "0")))
  if (is.na(q)) q <- 0L
  if (.Call("mk_r_hip_started")) {
    .Call("mk_r_hw_queues", if (q > 0L) q else 4L)
  } else {
    if (q < 8L) Sys.setenv(GPU_MAX_HW_QUEUES = "8")
    .Call("mk_r_hw_queues", -1L)
  }
  # libmk's pooled streams are destroyed while the HIP runtime is still alive at R's exit
  reg.finalizer(.mk_exit, function(e) .Call("mk_r_shutdown"), onexit = TRUE)
}

.mk_exit <- new.env()

.onUnload <- function(libpath) {
  .Call("mk_r_shutdown")
  library.dynam.unload("mkgpu", libpath)
}
