# R side of the mkgpu package: the reference's worker loop and combine, run by libmk.
# Uncompiled in the build image (R is not installed there); INTEGRATION.md walks through it.
#
# MetaKriging_BinaryResponse.R (MK.R) lines this replaces:
#   MK.R:102-111  obj <- foreach(i = 1:n.core, ...) %dopar% partitioned_spMvGLM(i, ...)
#                 -> obj <- mk_meta_fit(y, x, weight, q, n.part, index.part, coords, coords.test)
#   MK.R:123-133  result / result2 as the mean of the subset grids -> mk_combine(obj)
#   MK.R:136-165  resampling, p(y = 1) and quantiles              -> mk_posterior_summary(...)
# The worker's statistics that R computes before spMvGLM stay in R (MK.R:53-64): glm start
# values (or mk_glm_start on the device), starting / tuning / priors, n.batch, batch.length.

# Location-major rows of subset idx: site i, outcome a at (i - 1) * q + a (MK.R:67-75 layout).
.mk_rows <- function(idx, q) as.vector(t(outer((idx - 1) * q, 1:q, "+")))

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

# The foreach / partitioned_spMvGLM loop of MK.R:102-111 for every subset at once on one GPU.
# Returns a list of K list(parameters = 200 x P, w.predict = 200 x q n_test), the shape
# partitioned_spMvGLM returns (MK.R:89), plus per-batch acceptance rates.
mk_meta_fit <- function(y, x, weight, q, n.part, index.part, coords, coords.test,
                        n.batch = 100, batch.length = 50, accept.rate = 0.43,
                        cov.model = c("exponential", "matern"), link = c("logit", "probit"),
                        predict.tile = 0L, device = 0L, glm.on.device = FALSE) {
  cov.model <- match.arg(cov.model)
  link <- match.arg(link)
  st <- mk_glm_start(y, x, weight, link, if (glm.on.device) device else NULL)   # MK.R:53-55
  n.samples <- n.batch * batch.length
  A.starting <- diag(1, q)[lower.tri(diag(1, q), TRUE)]                          # MK.R:56
  matern <- cov.model == "matern"
  cfg <- list(as.integer(matern), as.integer(n.batch), as.integer(batch.length), accept.rate,
              as.integer(0.75 * n.samples),                                      # MK.R:85 burn.in
              as.double(st$beta), as.double(st$tuning),
              rep(3 / 0.5, q), rep(1, q), A.starting, rep(0.1, length(A.starting)),
              0, 0.5,                                                            # MK.R:60-62
              rep(3 / 0.75, q), rep(3 / 0.25, q), as.double(q), diag(0.1, q),    # MK.R:63-64
              if (matern) rep(0.5, q) else NULL, if (matern) rep(0.1, q) else NULL,
              if (matern) rep(0.1, q) else NULL, if (matern) rep(2, q) else NULL,
              as.integer(link == "probit"), as.integer(predict.tile), as.integer(device))
  S <- length(n.part)
  res <- .Call("mk_r_fit", as.integer(n.part),
               unlist(lapply(index.part, function(i) as.vector(coords[i, ]))),
               unlist(lapply(index.part, function(i) y[.mk_rows(i, q)])),
               unlist(lapply(index.part, function(i) rep(weight, length(i) * q))),
               unlist(lapply(index.part, function(i) as.vector(x[.mk_rows(i, q), , drop = FALSE]))),  # per subset
               coords.test, as.integer(q), ncol(x), cfg,
               floor(runif(1) * 2^52))                                           # honours set.seed
  P <- length(res[[1]]) / (S * 200)
  C <- length(res[[2]]) / (S * 200)
  lapply(seq_len(S), function(k) list(
    parameters = matrix(res[[1]][(k - 1) * 200 * P + 1:(200 * P)], 200, P),
    w.predict = matrix(res[[2]][(k - 1) * 200 * C + seq_len(200 * C)], 200, C),
    acceptance = matrix(res[[3]][(k - 1) * n.batch * (P + 1) + 1:(n.batch * (P + 1))], n.batch, P + 1)))
}

# MK.R:123-133: result = mean of obj[[k]]$parameters, result2 = mean of obj[[k]]$w.predict, in
# the same sequential summation order (bit-identical to the R loop).
mk_combine <- function(obj, device = 0L) {
  K <- length(obj)
  one <- function(field) {
    g <- unlist(lapply(obj, function(o) as.vector(o[[field]])))
    m <- .Call("mk_r_combine", g, as.integer(K), as.double(length(obj[[1]][[field]])), as.integer(device))
    matrix(m, nrow(obj[[1]][[field]]))
  }
  list(result = one("parameters"), result2 = one("w.predict"))
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
# (default 4, streams beyond it share queues) when it starts, which is after this hook.
.onLoad <- function(libname, pkgname) {
  q <- suppressWarnings(as.integer(Sys.getenv("GPU_MAX_HW_QUEUES", "0")))
  if (is.na(q) || q < 8L) Sys.setenv(GPU_MAX_HW_QUEUES = "8")
}
