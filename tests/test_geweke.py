"""Geweke's "getting it right" test of the oracle sampler (CPU).

The device replays the oracle on identical Philox draws (tests/test_gpu_sampler.py,
tests/test_stat_cfg2_cfg4.py), and the oracle is pinned against oracle/literal.py -- but both
restate the same spec, so a spec error they share (the IW / A Jacobian, the logit
phi and nu Jacobians, the LMC quadratic form, the single-site w ratio) would pass every one of
those tests.  This test checks the oracle's transition kernel against the MODEL it claims to
sample (MK.R:60-64, 80-84) by Geweke's two simulators of the joint
p(theta, w, y) (Geweke 2004, JASA 99:799):

  marginal-conditional   theta ~ prior, w | theta ~ N(0, C(theta)), y | w ~ Binomial -- exact,
                         independent draws;
  successive-conditional one oracle amcmc iteration on (theta, w) given y (fit_subset resumed from
                         the chain's state: the A, phi, nu and single-site w steps, the code the
                         device replays), then y | w redrawn -- a Markov chain whose stationary law
                         is the same joint iff every MH step leaves p(theta, w | y) invariant.

Each successive-conditional chain starts from a marginal-conditional draw, so it is stationary
from its first iteration and its mean is unbiased; chains are independent (their own Philox key:
the subset index), so the standard error comes from the spread of the chain means -- no
autocorrelation estimate.  Test functions: log K_hh and its square, the LMC correlation
K_21 / sqrt(K_11 K_22), phi_h and nu_h (Matern) with their squared distances from the prior's
midpoint (a Jacobian error piles mass at both edges of the support), the standardised latent field
mean(w_h) / sqrt(K_hh) and mean(w_h^2) / K_hh, and mean(y).  Every |z| <= 4.5.

Proper priors are required, so: beta is held at its true value in the covariance cases (MK.R:63's
beta.Flat is improper), and the case exp_q1_beta moves it under a TEST-ONLY proper prior
beta_j ~ N(0, 1) (oracle Config.beta_prior: the flat-prior step -- the likelihood ratio over eta,
the code the device replays -- plus the prior's log ratio); the IW
hyperparameters are K.IW = (q + 5, 4 I) -- the same IW code as the reference's (q, 0.1 I), whose
q = 1 form (inverse-gamma(0.5, 0.05): log K has sd 2.2, w's scale spans orders of magnitude) mixes
too slowly for a test of this length.  No adaptation (one batch longer than the run): adaptation
changes the proposal scale, not the target.

Power: the same test with the phi Jacobian or the IW Jacobian's A -> K terms deleted from the
oracle (monkeypatched inside the workers), or with the beta prior's term dropped from the beta step
(the chain then samples beta under a flat prior while the marginal-conditional side draws it from
N(0, 1)), must fail (max |z| > 6): the negative controls below.
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

N_SITES = 10
CHAINS = 32
ITERS = 250
MC_DRAWS = 20000
WORKERS = min(4, os.cpu_count() or 1)

CASES = {
    "exp_q1": dict(q=1, cov_model=0),
    "matern_q1": dict(q=1, cov_model=1),
    "lmc_q2": dict(q=2, cov_model=0),
    "exp_q1_beta": dict(q=1, cov_model=0, beta=True),
}


def _setup(case):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import spmvglm as om
    c = CASES[case]
    q, cov = c["q"], c["cov_model"]
    rng = np.random.default_rng(20250114 + q + 7 * cov)
    coords = rng.uniform(size=(N_SITES, 2))
    p = 2 * q
    X = np.zeros((N_SITES * q, p))
    for a in range(q):
        X[a::q, 2 * a] = 1.0
        X[a::q, 2 * a + 1] = rng.normal(size=N_SITES)
    beta = np.array([0.3, -0.5, -0.2, 0.4][:p])
    cfg = om.Config(q, p, beta, np.full(p, 0.5), cov_model=cov, n_batch=1, batch_length=10 ** 7, burn_in=10 ** 7,
                    K_IW_df=q + 5.0, K_IW_S=4.0 * np.eye(q),
                    beta_prior=(np.zeros(p), np.ones(p)) if c.get("beta") else None)
    return om, coords, X, beta, cfg


def _joint(om, rng, coords, X, beta, cfg):
    """One marginal-conditional draw: (beta, A, phi, nu, w, y); beta from its prior when it moves."""
    from scipy.stats import invwishart
    q = cfg.q
    if cfg.beta_prior is not None:
        beta = rng.normal(cfg.beta_prior[0], cfg.beta_prior[1])
    K = np.atleast_2d(invwishart.rvs(cfg.K_IW_df, cfg.K_IW_S, random_state=rng))
    A = np.linalg.cholesky(K)
    phi = rng.uniform(cfg.phi_a, cfg.phi_b)
    nu = rng.uniform(cfg.nu_a, cfg.nu_b) if cfg.cov_model == om.COV_MATERN else None
    C = om.lmc_covariance(coords, A, phi, nu, cfg.cov_model)
    w = np.linalg.cholesky(C + 1e-12 * np.eye(C.shape[0])) @ rng.normal(size=C.shape[0])
    y = rng.binomial(1, 1.0 / (1.0 + np.exp(-(X @ beta + w)))).astype(float)
    return beta, A, phi, nu, w, y


def _features(beta, A, phi, nu, w, y, q, cfg):
    K = A @ A.T
    f = []
    if cfg.beta_prior is not None:
        for b in beta:
            f += [b, b * b]
    for h in range(q):
        lk = np.log(K[h, h])
        # phi and nu: the mean and the spread about the prior's midpoint (a Jacobian error moves mass
        # toward both edges of the support and barely moves the mean)
        pm = 0.5 * (cfg.phi_a[h] + cfg.phi_b[h])
        f += [lk, lk * lk, phi[h], (phi[h] - pm) ** 2]
        if nu is not None:
            nm = 0.5 * (cfg.nu_a[h] + cfg.nu_b[h])
            f += [nu[h], (nu[h] - nm) ** 2]
        wh = w[h::q]
        f += [np.mean(wh) / np.sqrt(K[h, h]), np.mean(wh * wh) / K[h, h]]
    if q == 2:
        f.append(K[1, 0] / np.sqrt(K[0, 0] * K[1, 1]))
    f.append(np.mean(y))
    return np.array(f)


def _feature_names(q, matern, beta_p=0):
    names = []
    for j in range(beta_p):
        names += [f"beta{j}", f"beta{j}^2"]
    for h in range(q):
        names += [f"logK{h}", f"logK{h}^2", f"phi{h}", f"(phi{h}-mid)^2"]
        if matern:
            names += [f"nu{h}", f"(nu{h}-mid)^2"]
        names += [f"w{h}/sdK", f"w{h}^2/K"]
    if q == 2:
        names.append("corrK")
    return names + ["y"]


def _bug(om, which):
    """Negative controls: delete a Jacobian from the oracle's log posterior."""
    if which == "phi_jacobian":
        om.unif_jacobian = lambda v, a, b: 0.0
    elif which == "iw_jacobian":
        import scipy.linalg as sla

        def iw_no_jac(A, df, S):
            q = A.shape[0]
            logdetK = 2.0 * np.sum(np.log(np.diag(A)))
            Ainv = sla.solve_triangular(A, np.eye(q), lower=True)
            Kinv = Ainv.T @ Ainv
            return -0.5 * (df + q + 1.0) * logdetK - 0.5 * np.sum(S * Kinv.T), logdetK
        om.iw_logprior_A = iw_no_jac
    elif which == "beta_prior":
        om.beta_logprior = lambda b, j, cfg: 0.0


def _chain(args):
    """One successive-conditional chain: ITERS (oracle iteration, y redraw) pairs from a joint draw;
    returns the chain mean of the test functions."""
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    case, k, bug = args
    om, coords, X, beta, cfg = _setup(case)
    if bug:
        _bug(om, bug)
    q, matern = cfg.q, cfg.cov_model == om.COV_MATERN
    rng = np.random.default_rng([7, k, len(bug or "")])
    beta, A, phi, nu, w, y = _joint(om, rng, coords, X, beta, cfg)
    n_mh = cfg.p + cfg.n_theta + N_SITES * q
    moves = cfg.beta_prior is not None
    tune = np.concatenate([np.log(np.sqrt(cfg.beta_tuning)) if moves else np.full(cfg.p, -np.inf),  # held: sd 0
                           np.log(np.sqrt(cfg.A_tuning)), np.log(np.sqrt(cfg.phi_tuning)),
                           np.log(np.sqrt(cfg.nu_tuning)) if matern else np.zeros(0),
                           np.full(N_SITES * q, np.log(np.sqrt(cfg.w_tuning)))])
    theta = [om.A_to_tri(A), om.logit(phi, cfg.phi_a, cfg.phi_b)]
    if matern:
        theta.append(om.logit(nu, cfg.nu_a, cfg.nu_b))
    state = dict(iteration=0, beta=beta.copy(), theta=np.concatenate(theta), w=w, tune=tune, accept=np.zeros(n_mh))
    ntri = q * (q + 1) // 2
    acc = np.zeros_like(_features(beta, A, phi, nu, w, y, q, cfg))
    for s in range(ITERS):
        r = om.fit_subset(coords, y, np.ones(N_SITES * q), X, cfg, subset=k, start=state, max_iter=s + 1,
                          quantiles=False)
        state = r["state"]
        th = state["theta"]
        A = om.tri_to_A(th[:ntri], q)
        phi = om.logit_inv(th[ntri:ntri + q], cfg.phi_a, cfg.phi_b)
        nu = om.logit_inv(th[ntri + q:ntri + 2 * q], cfg.nu_a, cfg.nu_b) if matern else None
        w = state["w"]
        beta = state["beta"]
        y = rng.binomial(1, 1.0 / (1.0 + np.exp(-(X @ beta + w)))).astype(float)
        acc += _features(beta, A, phi, nu, w, y, q, cfg)
    return acc / ITERS


def _mc(case):
    om, coords, X, beta, cfg = _setup(case)
    rng = np.random.default_rng(99)
    f = np.stack([_features(*_joint(om, rng, coords, X, beta, cfg), cfg.q, cfg) for _ in range(MC_DRAWS)])
    return f.mean(axis=0), f.std(axis=0, ddof=1) / np.sqrt(MC_DRAWS)


def _z(case, bug=None):
    with mp.get_context("spawn").Pool(WORKERS) as pool:
        means = np.stack(pool.map(_chain, [(case, k, bug) for k in range(CHAINS)]))
    m_mc, se_mc = _mc(case)
    m_sc, se_sc = means.mean(axis=0), means.std(axis=0, ddof=1) / np.sqrt(CHAINS)
    return (m_sc - m_mc) / np.sqrt(se_sc ** 2 + se_mc ** 2), m_sc, m_mc


@pytest.mark.parametrize("case", sorted(CASES))
def test_geweke_successive_conditional_matches_marginal_conditional(case):
    z, m_sc, m_mc = _z(case)
    c = CASES[case]
    names = _feature_names(c["q"], c["cov_model"] == 1, 2 * c["q"] if c.get("beta") else 0)
    report = {n: (round(float(a), 4), round(float(b), 4), round(float(c), 2)) for n, a, b, c in zip(names, m_sc, m_mc, z)}
    assert np.all(np.abs(z) <= 4.5), report


@pytest.mark.parametrize("bug", ["phi_jacobian", "iw_jacobian"])
def test_geweke_detects_a_deleted_jacobian(bug):
    z, _, _ = _z("exp_q1", bug)
    assert np.max(np.abs(z)) > 6.0, (bug, np.round(z, 2))


def test_geweke_detects_a_dropped_beta_prior():
    z, _, _ = _z("exp_q1_beta", "beta_prior")
    assert np.max(np.abs(z)) > 6.0, np.round(z, 2)
