"""Combine extensions and post-processing, NumPy restatement (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

  posterior_summary  -- MetaKriging_BinaryResponse.R:136-165: interpolate both combined
                        200-level grids to Xout = seq(0.005, 1, 0.001) (996 levels, MK.R:140-144),
                        one shared resample index vector (MK.R:141, 145-146), p(y=1) =
                        1/(1+exp(-(x.test %*% B.s + Samplew[j,]))) (MK.R:156-161), and the
                        (0.5, 0.025, 0.975) type-7 summaries (MK.R:163-165).
  weiszfeld_median   -- the north-star "Weiszfeld geometric-median" combine.
                        NOT in the reference (which averages, MK.R:123-133): parity unpinned, this
                        restatement is the spec the device kernel is checked against.

Resample index (MK.R:141, sample(seq(1, length(Xout), 1), samplesize, replace=TRUE)): either
R's own draws -- a caller-given 1-based index, e.g. rrng.RRng(seed).sample_int_replace(996, S)
for an R session that called set.seed(seed) just before -- or, by default, Philox: draw j uses
key (seed, 0), counter (j, 0, TAG_RESAMPLE, 0), idx_j = min(floor(u_j * 996), 995), uniform
over the 996 Xout levels with replacement like R's.
"""
import numpy as np

from . import philox
from .rstats import PROBS200, XOUT996, r_approx, r_quantile7
from .spmvglm import combine_mean

SUMMARY_PROBS = np.array([0.5, 0.025, 0.975])      # quant.pred, MK.R:163


def resample_index(samplesize, seed, n_levels=len(XOUT996)):
    """0-based rows of the interpolated grids, shared by every column (MK.R:141)."""
    u = philox.resample_uniform(philox.make_key(seed, 0), np.arange(samplesize))
    return np.minimum(np.floor(u * n_levels).astype(np.int64), n_levels - 1)


def posterior_summary(result, result2, x_test, samplesize=1000, seed=20250114, index=None, link="logit"):
    """MK.R:136-165.  result: 200 x P combined parameter grid (betas first, MK.R:159);
    result2: 200 x C combined w.predict grid; x_test: C x p.  Returns the reference's
    SamplePar, Samplew, p.sample, w.quant (3 x C), param.quant (3 x P), plus p.quant (3 x C)."""
    result = np.asarray(result, dtype=np.float64)
    result2 = np.asarray(result2, dtype=np.float64)
    x_test = np.asarray(x_test, dtype=np.float64)
    # index: caller-drawn 1-based sampleparIndex (e.g. R's stream, rrng.RRng(seed).sample_int_replace)
    idx = resample_index(samplesize, seed) if index is None else np.asarray(index, dtype=np.int64) - 1
    sample_par = r_approx(PROBS200, result, XOUT996)[idx]          # Result.Inter[sampleparIndex,]
    sample_w = r_approx(PROBS200, result2, XOUT996)[idx]           # Result.Inter2[sampleparIndex,]
    p = x_test.shape[1]
    # x.test %*% B.s, summed in column order m = 0..p-1 (the device's order)
    xb = np.zeros((samplesize, x_test.shape[0]))
    for m in range(p):
        xb = xb + sample_par[:, m:m + 1] * x_test[:, m][None, :]
    eta = xb + sample_w
    if link == "probit":                      # extension: Phi(eta) = erfc(-eta/sqrt2)/2 (device formula)
        from scipy.special import erfc
        p_sample = 0.5 * erfc(-eta * 0.7071067811865476)
    else:
        p_sample = 1.0 / (1.0 + np.exp(-eta))
    return dict(index=idx, SamplePar=sample_par, Samplew=sample_w, p_sample=p_sample,
                w_quant=r_quantile7(sample_w, SUMMARY_PROBS, axis=0),
                param_quant=r_quantile7(sample_par, SUMMARY_PROBS, axis=0),
                p_quant=r_quantile7(p_sample, SUMMARY_PROBS, axis=0))


def weiszfeld_median(grids, max_iter=100, tol=1e-12):
    """Geometric median of the K subset quantile functions, column by column.

    grids: (K, L, C) -- K subsets' L-level quantile grids (obj[[k]]$parameters or $w.predict).
    Each column c is one marginal; its K quantile functions Q_k are points of L2(0,1), whose
    metric on 1-D laws is the Wasserstein-2 distance, discretised on the L levels:
        d(y, Q_k) = sqrt(mean_l (y_l - Q_k,l)^2).
    Weiszfeld iteration from the barycenter (the reference's mean, MK.R:123-133):
        y <- sum_k Q_k / d_k  /  sum_k 1 / d_k,    d_k floored at eps = 1e-14 (1 + rms(y)),
    stopped when d(y_new, y) <= tol (1 + rms(y_new)) or after max_iter steps.  A convex
    combination of quantile functions is a quantile function, so every iterate is monotone.
    Returns (median (L, C), iterations (C,))."""
    g = np.asarray(grids, dtype=np.float64)
    K, L, C = g.shape
    y = combine_mean(list(g))
    iters = np.zeros(C, dtype=np.int64)
    active = np.ones(C, dtype=bool)
    for t in range(max_iter):
        if not active.any():
            break
        cols = np.nonzero(active)[0]
        ya = y[:, cols]
        ga = g[:, :, cols]
        scale = 1.0 + np.sqrt(np.mean(ya * ya, axis=0))
        d = np.sqrt(np.mean((ga - ya[None]) ** 2, axis=1))          # (K, Ca)
        d = np.maximum(d, 1e-14 * scale[None])
        w = 1.0 / d
        num = np.zeros_like(ya)
        den = np.zeros(len(cols))
        for k in range(K):                                          # sequential over subsets
            num = num + ga[k] * w[k][None]
            den = den + w[k]
        ynew = num / den[None]
        step = np.sqrt(np.mean((ynew - ya) ** 2, axis=0))
        y[:, cols] = ynew
        iters[cols] = t + 1
        done = step <= tol * (1.0 + np.sqrt(np.mean(ynew * ynew, axis=0)))
        active[cols[done]] = False
    return y, iters
