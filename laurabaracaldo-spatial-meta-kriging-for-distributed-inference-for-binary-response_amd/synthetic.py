"""Deterministic synthetic binary spatial data (the driver the reference lacks).

MetaKriging_BinaryResponse.R reads globals it never defines -- n, y, x, weight,
coords, coords.test, x.test, n.extra (MK.R:15, 33-39, 108, 156); they come
from the spBayes ``spMvGLM`` help-page recipe.  This module is that driver
(SURVEY.md section 8d):

  coords ~ U[0,1]^2; per outcome X_a = [1, N(0,1)]; block-diagonal design
  beta = (1,-1) | (1,-1,-1,1) | (1,-1,-1,1,0.5,-0.5); phi = 6; K = A A'
  w ~ GP(0, LMC(exponential|Matern)); exact Cholesky draw for n_total <= 6000,
  random Fourier features (M = 4096) above; y ~ Binomial(weight, logistic(X beta + w)).

Layout produced (R conventions): y, weight location-major (site i, outcome a at
i*q + a); x (n*q, p) block-diagonal; coords (n, 2).  Test sites: coords_test
(n_test, 2), x_test (q*n_test, p).
"""
import numpy as np

TRUE_BETA = {1: [1.0, -1.0], 2: [1.0, -1.0, -1.0, 1.0], 3: [1.0, -1.0, -1.0, 1.0, 0.5, -0.5],
             4: [1.0, -1.0, -1.0, 1.0, 0.5, -0.5, -0.5, 0.5]}   # q = 4: the library's maximum (MK_QMAX)
TRUE_A = {1: [[1.0]],
          2: [[1.0, 0.0], [-0.5, 1.0]],
          3: [[1.0, 0.0, 0.0], [-0.5, 1.0, 0.0], [0.25, 0.3, 0.8]],
          4: [[1.0, 0.0, 0.0, 0.0], [-0.5, 1.0, 0.0, 0.0], [0.25, 0.3, 0.8, 0.0], [0.1, -0.2, 0.3, 0.7]]}


def block_design(xcov, q):
    """xcov (n, q) covariate per outcome -> (n*q, 2q) design with [1, x] blocks (spBayes mkMvX)."""
    n = xcov.shape[0]
    X = np.zeros((n * q, 2 * q))
    for a in range(q):
        X[a::q, 2 * a] = 1.0
        X[a::q, 2 * a + 1] = xcov[:, a]
    return X


def _exact_field(coords, A, phi, nu, cov_model, rng):
    from scipy.special import gamma, kv
    n = coords.shape[0]
    q = A.shape[0]
    d = np.sqrt(((coords[:, None, :] - coords[None, :, :]) ** 2).sum(-1))
    W = np.zeros((n, q))
    for h in range(q):
        if cov_model == 0:
            R = np.exp(-phi * d)
        else:
            x = phi * d
            R = np.ones_like(x)
            m = x > 0
            R[m] = x[m] ** nu / (2 ** (nu - 1) * gamma(nu)) * kv(nu, x[m])
        Lr = np.linalg.cholesky(R + 1e-12 * np.eye(n))
        W[:, h] = Lr @ rng.standard_normal(n)
    return W @ A.T


def _rff_field(coords, A, phi, nu, cov_model, rng, M=4096, chunk=8192):
    """Random Fourier features: exponential -> omega = phi*z/sqrt(u), u~chi2_1 (Cauchy-type);
    Matern -> multivariate-t(2 nu) frequencies scaled by phi.  M = 4096 features;
    the n x M cosines (2e9 at configs[2]) in row chunks with NumPy.  (Not torch: a host that loads
    torch after libmk maps torch's bundled HIP runtime beside libmk's -- two HIP runtimes in one
    process)"""
    import os
    from concurrent.futures import ThreadPoolExecutor
    n = coords.shape[0]
    q = A.shape[0]
    W = np.zeros((n, q))
    n_thr = max(1, min(16, os.cpu_count() or 1, (n + chunk - 1) // chunk))

    def rows(s, om_t, b, c, h):     # NumPy releases the GIL in matmul / cos: chunks run in parallel
        m = min(chunk, n - s)
        p_ = coords[s:s + m] @ om_t
        p_ += b
        np.cos(p_, out=p_)
        W[s:s + m, h] = np.sqrt(2.0 / M) * (p_ @ c)

    with ThreadPoolExecutor(n_thr) as ex:
        for h in range(q):
            z = rng.standard_normal((M, 2))
            dof = 1.0 if cov_model == 0 else 2.0 * nu
            u = rng.chisquare(dof, size=M) / dof
            omega = phi * z / np.sqrt(u)[:, None]
            b = rng.uniform(0, 2 * np.pi, size=M)
            c = rng.standard_normal(M)
            om_t = np.ascontiguousarray(omega.T)
            list(ex.map(lambda s: rows(s, om_t, b, c, h), range(0, n, chunk)))
    return W @ A.T


def generate(n, q=1, n_test=1000, weight=1, cov_model=0, phi=6.0, nu=0.5, seed=20250114,
             exact_max=6000, link="logit"):
    rng = np.random.default_rng(seed)
    A = np.array(TRUE_A[q])
    beta = np.array(TRUE_BETA[q])
    coords_all = rng.uniform(size=(n + n_test, 2))
    if n + n_test <= exact_max:
        W = _exact_field(coords_all, A, phi, nu, cov_model, rng)
    else:
        W = _rff_field(coords_all, A, phi, nu, cov_model, rng)
    xcov = rng.standard_normal((n + n_test, q))
    X_all = block_design(xcov, q)
    eta = X_all @ beta + W.reshape(-1)
    if link == "probit":      # extension: y ~ Binomial(weight, Phi(eta))
        from scipy.special import ndtr
        prob = ndtr(eta)
    else:
        prob = 1.0 / (1.0 + np.exp(-eta))
    y_all = rng.binomial(weight, prob).astype(np.float64)
    N = n * q
    return dict(
        n=n, q=q, p=2 * q, weight=weight,
        coords=coords_all[:n].copy(), y=y_all[:N].copy(), x=X_all[:N].copy(),
        w_true=W[:n].reshape(-1).copy(),
        coords_test=coords_all[n:].copy(), x_test=X_all[N:].copy(),
        y_test=y_all[N:].copy(), w_test_true=W[n:].reshape(-1).copy(),
        beta_true=beta, A_true=A, phi_true=phi, nu_true=nu, cov_model=cov_model,
        n_extra=n + n_test)
