"""Literal restatement of spBayes' amcmc loop for spMvGLM (TEST INFRASTRUCTURE ONLY).

spBayes (spMvGLM, MK.R:80-84) evaluates, for EVERY single-parameter proposal
(each beta_j, each A entry, each phi_h / nu_h and each of the N latent w_k),
the full log posterior from scratch: it rebuilds the dense N x N LMC
covariance, Cholesky-factors it (dpotrf), takes the log-determinant, forms
w' C^-1 w, adds the IW(K) prior with its Jacobian, the logit-uniform
Jacobians and the binomial log-likelihood, and accepts if
runif <= exp(cand - current).  That is O(N^3) per proposal, O(N^4) per
iteration -- usable only for tiny N.

This file does exactly that, on the same Philox draws as spmvglm.fit_subset,
so tests can show that the incremental O(N^2)-per-iteration algorithm used by
the oracle and the HIP library reproduces the literal algorithm's chain.
"""
import numpy as np

from . import philox
from .spmvglm import (COV_MATERN, A_to_tri_start, correlation, distance_matrix,
                      iw_logprior_A, lmc_covariance, logit, logit_inv, loglik_terms,
                      lower_tri_vec, n_tri, tri_to_A, unif_jacobian)


def log_posterior(params, coords, y, wt, X, cfg):
    q, p = cfg.q, cfg.p
    n = coords.shape[0]
    ntri = n_tri(q)
    matern = cfg.cov_model == COV_MATERN
    beta = params[:p]
    A = tri_to_A(params[p:p + ntri], q)
    o_phi = p + ntri
    phi = logit_inv(params[o_phi:o_phi + q], cfg.phi_a, cfg.phi_b)
    nu = logit_inv(params[o_phi + q:o_phi + 2 * q], cfg.nu_a, cfg.nu_b) if matern else [0.0] * q
    w = params[o_phi + q * (2 if matern else 1):]
    C = lmc_covariance(coords, A, phi, nu, cfg.cov_model)
    Lc = np.linalg.cholesky(C)
    logdet = 2.0 * np.sum(np.log(np.diag(Lc)))
    z = np.linalg.solve(Lc, w)
    out = -0.5 * logdet - 0.5 * (z @ z)
    lp, _ = iw_logprior_A(A, cfg.K_IW_df, cfg.K_IW_S)
    out += lp
    out += np.sum(unif_jacobian(phi, cfg.phi_a, cfg.phi_b))
    if matern:
        out += np.sum(unif_jacobian(np.asarray(nu), cfg.nu_a, cfg.nu_b))
    eta = X @ beta + w
    out += np.sum(loglik_terms(y, wt, eta, getattr(cfg, "link", 0)))
    return out


def fit_subset_literal(coords, y, wt, X, cfg, subset=0, n_iter=None):
    q, p = cfg.q, cfg.p
    n = coords.shape[0]
    N = n * q
    matern = cfg.cov_model == COV_MATERN
    key = philox.make_key(cfg.seed, subset)
    params = np.concatenate([
        cfg.beta_starting, A_to_tri_start(cfg.A_starting, q),
        logit(cfg.phi_starting, cfg.phi_a, cfg.phi_b),
        logit(cfg.nu_starting, cfg.nu_a, cfg.nu_b) if matern else np.zeros(0),
        np.full(N, cfg.w_starting)])
    n_mh = params.size
    tune = np.concatenate([
        np.log(np.sqrt(cfg.beta_tuning)), np.log(np.sqrt(cfg.A_tuning)),
        np.log(np.sqrt(cfg.phi_tuning)),
        np.log(np.sqrt(cfg.nu_tuning)) if matern else np.zeros(0),
        np.full(N, np.log(np.sqrt(cfg.w_tuning)))])
    n_iter = cfg.n_samples if n_iter is None else n_iter
    cur = log_posterior(params, coords, y, wt, X, cfg)
    accept = np.zeros(n_mh)
    samples = np.zeros((n_iter, cfg.n_report))
    decisions = np.zeros((n_iter, n_mh), dtype=bool)
    ntri = n_tri(q)
    for s in range(n_iter):
        js = np.arange(n_mh)
        zs = philox.proposal_normal(key, js, s)
        logus = philox.accept_log_uniform(key, js, s)
        for j in range(n_mh):
            old = params[j]
            params[j] = old + np.exp(tune[j]) * zs[j]
            cand = log_posterior(params, coords, y, wt, X, cfg)
            if logus[j] <= cand - cur:
                cur = cand
                accept[j] += 1
                decisions[s, j] = True
            else:
                params[j] = old
        A = tri_to_A(params[p:p + ntri], q)
        o_phi = p + ntri
        samples[s, :p] = params[:p]
        samples[s, p:p + ntri] = lower_tri_vec(A @ A.T)
        samples[s, o_phi:o_phi + q] = logit_inv(params[o_phi:o_phi + q], cfg.phi_a, cfg.phi_b)
        if matern:
            samples[s, o_phi + q:o_phi + 2 * q] = logit_inv(params[o_phi + q:o_phi + 2 * q], cfg.nu_a, cfg.nu_b)
        if (s + 1) % cfg.batch_length == 0:
            b = s // cfg.batch_length
            rate = accept / cfg.batch_length
            step = min(0.01, 1.0 / np.sqrt(b)) if b > 0 else 0.01
            tune = np.where(rate > cfg.accept_rate, tune + step, tune - step)
            accept[:] = 0.0
    return dict(samples=samples, params=params, decisions=decisions)
