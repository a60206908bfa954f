"""R semantics needed on the hot path, restated in NumPy (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

Each function restates the R behaviour the reference script relies on:
  r_seq          -- seq(from, to, by)               MK.R:88 (probs), MK.R:140 (Xout), MK.R:142
  r_quantile7    -- quantile(x, probs) (type 7)     MK.R:88, MK.R:163
  r_approx       -- approx(x, y, xout)$y (linear)   MK.R:142
  glm_binomial   -- glm(y/weight ~ x - 1, weights, family=binomial)   MK.R:53-55
These are R's published algorithms (R 4.x: seq.default, quantile.default,
stats/src/approx.c, glm.fit + family.c); R is not installed here (SURVEY.md
section 8c), so they are pinned against independent numpy/scipy
implementations in tests/test_oracle_rstats.py.
"""
import numpy as np


def r_seq(frm, to, by):
    """seq.default(from, to, by): from + (0:n)*by, n = as.integer(del/by + 1e-10), pmin(x, to)."""
    dl = to - frm
    n = int(dl / by + 1e-10)
    x = frm + np.arange(n + 1, dtype=np.float64) * by
    return np.minimum(x, to) if by > 0 else np.maximum(x, to)


PROBS200 = r_seq(0.005, 1.0, 0.005)   # MK.R:88 allquant levels (200)
XOUT996 = r_seq(0.005, 1.0, 0.001)    # MK.R:140 interpolation grid (996)


def r_quantile7(x, probs, axis=0):
    """quantile.default(x, probs, type=7) along `axis` (names dropped).

    index <- 1 + (n-1)*probs; lo <- floor(index); hi <- ceiling(index)
    qs <- x[lo]; i <- index > lo & x[hi] != qs; qs[i] <- (1-h)*qs[i] + h*x[hi[i]]
    """
    x = np.moveaxis(np.asarray(x, dtype=np.float64), axis, 0)
    n = x.shape[0]
    xs = np.sort(x, axis=0)
    probs = np.asarray(probs, dtype=np.float64)
    index = 1.0 + max(n - 1, 0) * probs
    lo = np.floor(index).astype(np.int64)
    hi = np.ceil(index).astype(np.int64)
    qlo = xs[lo - 1]
    qhi = xs[hi - 1]
    h = (index - lo).reshape((-1,) + (1,) * (x.ndim - 1))
    interp = (index > lo).reshape(h.shape) & (qhi != qlo)
    out = np.where(interp, (1.0 - h) * qlo + h * qhi, qlo)
    return np.moveaxis(out, 0, axis)


def r_approx(x, y, xout):
    """stats::approx(x, y, xout, method='linear', rule=1)$y for strictly increasing x.

    approx1(): bisection for i < j with x[i] <= v <= x[j]; exact hits return y;
    otherwise y[i] + (y[j]-y[i]) * ((v-x[i])/(x[j]-x[i])); out-of-range -> NA.
    Vectorised over trailing dims of y (each column interpolated independently).
    """
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xout = np.asarray(xout, dtype=np.float64)
    n = x.shape[0]
    out = np.empty((xout.shape[0],) + y.shape[1:], dtype=np.float64)
    for k, v in enumerate(xout):
        if v < x[0] or v > x[n - 1]:
            out[k] = np.nan
            continue
        i, j = 0, n - 1
        while i < j - 1:
            ij = (i + j) // 2
            if v < x[ij]:
                j = ij
            else:
                i = ij
        if v == x[j]:
            out[k] = y[j]
        elif v == x[i]:
            out[k] = y[i]
        else:
            out[k] = y[i] + (y[j] - y[i]) * ((v - x[i]) / (x[j] - x[i]))
    return out


# ---------------------------------------------------------------- glm (binomial, logit)
_THRESH = 30.0
_MTHRESH = -30.0
_INVEPS = 1.0 / np.finfo(np.float64).eps
_DBL_EPS = np.finfo(np.float64).eps


def _logit_linkinv(eta):
    tmp = np.where(eta < _MTHRESH, _DBL_EPS, np.where(eta > _THRESH, _INVEPS, np.exp(eta)))
    return tmp / (1.0 + tmp)


def _logit_mu_eta(eta):
    opexp = 1.0 + np.exp(eta)
    return np.where((eta > _THRESH) | (eta < _MTHRESH), _DBL_EPS, np.exp(eta) / (opexp * opexp))


def _y_log_y(y, mu):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(y != 0.0, y * np.log(np.where(y != 0.0, y, 1.0) / mu), 0.0)


def _binom_dev(y, mu, wt):
    return np.sum(2.0 * wt * (_y_log_y(y, mu) + _y_log_y(1.0 - y, 1.0 - mu)))


_PROBIT_THRESH = 8.125890664701906     # -qnorm(.Machine$double.eps)


def _probit_linkinv(eta):
    from scipy.special import ndtr
    return ndtr(np.clip(eta, -_PROBIT_THRESH, _PROBIT_THRESH))


def _probit_mu_eta(eta):
    return np.maximum(np.exp(-0.5 * eta * eta) / np.sqrt(2.0 * np.pi), _DBL_EPS)


def glm_binomial(yprop, X, prior_w, epsilon=1e-8, maxit=25, link="logit"):
    """glm.fit IRLS for family=binomial(logit); returns (coef, vcov).

    vcov = chol2inv(R) of the final weighted QR (dispersion 1), as summary.glm.
    MK.R:53-55 then uses coef as beta.starting and t(chol(vcov)) as beta.tuning.
    link="probit": make.link("probit") (linkinv pnorm of eta clamped to +-qnorm(eps),
    mu.eta max(dnorm, eps), linkfun qnorm) -- the extension's start values.
    """
    from scipy.special import ndtri
    linkinv, mu_eta_f = (_logit_linkinv, _logit_mu_eta) if link == "logit" else (_probit_linkinv, _probit_mu_eta)
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(yprop, dtype=np.float64)
    wt = np.asarray(prior_w, dtype=np.float64)
    mu = (wt * y + 0.5) / (wt + 1.0)                  # binomial()$initialize
    eta = np.log(mu / (1.0 - mu)) if link == "logit" else ndtri(mu)
    devold = _binom_dev(y, mu, wt)
    coef = None
    R = None
    for _ in range(maxit):
        mu_eta = mu_eta_f(eta)
        varmu = mu * (1.0 - mu)
        good = (wt > 0) & (mu_eta != 0)
        z = eta[good] + (y[good] - mu[good]) / mu_eta[good]
        w = np.sqrt(wt[good] * mu_eta[good] ** 2 / varmu[good])
        Xw = X[good] * w[:, None]
        Qm, R = np.linalg.qr(Xw)
        coef = np.linalg.solve(R, Qm.T @ (z * w))
        eta = X @ coef
        mu = linkinv(eta)
        dev = _binom_dev(y, mu, wt)
        if abs(dev - devold) / (abs(dev) + 0.1) < epsilon:
            break
        devold = dev
    Rinv = np.linalg.inv(R)
    vcov = Rinv @ Rinv.T
    return coef, vcov
