"""Binomial-logit IRLS start values (MK.R:53-55), on device.

``fit <- glm((y/weight) ~ x - 1, weights = rep(weight, n*q), family = "binomial")``;
``beta.starting <- coefficients(fit)``; ``beta.tuning <- t(chol(vcov(fit)))``.
The R worker runs this above the spBayes boundary on the FULL data in every worker;
here it runs once per call through mk_glm_binomial:
each IRLS step is one HBM pass over the data (deviance of the current fit + the weighted
normal equations of the next), glm.fit's rules throughout -- binomial()$initialize mustart,
R's logit eta thresholds, |dev - devold| / (|dev| + 0.1) < epsilon, maxit 25, vcov =
(X'WX)^-1 at the weights that produced the final coefficients (dispersion 1).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, dptr, iptr


def glm_binomial(y, x, weights, epsilon=1e-8, maxit=25, device=0, link="logit"):
    """Returns (coefficients, vcov, beta_tuning = t(chol(vcov))) -- y are counts, weights trials.
    link="probit": binomial(link = "probit") (north-star extension; the reference fits logit)."""
    from .session import LINKS
    if link not in LINKS:
        raise ValueError(f"error: link must be 'logit' or 'probit', not '{link}'")
    lib = _lib.load()
    x = np.asarray(x, dtype=np.float64)
    n, p = x.shape
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float64).reshape(n))
    wt = np.ascontiguousarray(np.broadcast_to(np.asarray(weights, dtype=np.float64), (n,)))
    xf = np.ascontiguousarray(x.ravel(order="F"))
    coef = np.zeros(p)
    vcov = np.zeros(p * p)
    it = np.zeros(1, dtype=np.int32)
    check(lib.mk_glm_binomial_link(dptr(y), dptr(wt), dptr(xf), n, p, LINKS[link], float(epsilon), int(maxit),
                                   dptr(coef), dptr(vcov), iptr(it), int(device)))
    vcov = vcov.reshape(p, p, order="F")
    return coef, vcov, np.linalg.cholesky(vcov)
