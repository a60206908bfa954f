"""Binomial-logit IRLS start values (MK.R:53-55).

``fit <- glm((y/weight) ~ x - 1, weights = rep(weight, n*q), family = "binomial")``;
``beta.starting <- coefficients(fit)``; ``beta.tuning <- t(chol(vcov(fit)))``.
The R worker runs this above the spBayes boundary on the FULL data in every
worker; here it runs once per call.  glm.fit rules:
binomial()$initialize mustart, logit link with R's eta thresholds, relative
deviance convergence |dev - devold| / (|dev| + 0.1) < 1e-8, maxit 25, vcov
from the final weighted QR (dispersion 1).
"""
import numpy as np

_EPS = np.finfo(np.float64).eps


def _linkinv(eta):
    t = np.exp(np.clip(eta, -30.0, 30.0))
    t = np.where(eta < -30.0, _EPS, np.where(eta > 30.0, 1.0 / _EPS, t))
    return t / (1.0 + t)


def _mu_eta(eta):
    e = np.exp(np.clip(eta, -30.0, 30.0))
    return np.where(np.abs(eta) > 30.0, _EPS, e / ((1.0 + e) * (1.0 + e)))


def _dev(y, mu, wt):
    with np.errstate(divide="ignore", invalid="ignore"):
        a = np.where(y > 0, y * np.log(np.where(y > 0, y, 1.0) / mu), 0.0)
        b = np.where(y < 1, (1 - y) * np.log(np.where(y < 1, 1 - y, 1.0) / (1 - mu)), 0.0)
    return float(np.sum(2.0 * wt * (a + b)))


def glm_binomial(y, x, weights, epsilon=1e-8, maxit=25):
    """Returns (coefficients, vcov, beta_tuning = t(chol(vcov)))."""
    x = np.asarray(x, dtype=np.float64)
    wt = np.asarray(weights, dtype=np.float64)
    yp = np.asarray(y, dtype=np.float64) / wt
    mu = (wt * yp + 0.5) / (wt + 1.0)
    eta = np.log(mu / (1.0 - mu))
    devold = _dev(yp, mu, wt)
    R = None
    coef = np.zeros(x.shape[1])
    for _ in range(maxit):
        me = _mu_eta(eta)
        var = mu * (1.0 - mu)
        good = (wt > 0) & (me != 0)
        z = eta[good] + (yp[good] - mu[good]) / me[good]
        w = np.sqrt(wt[good] * me[good] ** 2 / var[good])
        Qm, R = np.linalg.qr(x[good] * w[:, None])
        coef = np.linalg.solve(R, Qm.T @ (z * w))
        eta = x @ coef
        mu = _linkinv(eta)
        dev = _dev(yp, mu, wt)
        if abs(dev - devold) / (abs(dev) + 0.1) < epsilon:
            break
        devold = dev
    Ri = np.linalg.inv(R)
    vcov = Ri @ Ri.T
    return coef, vcov, np.linalg.cholesky(vcov)
