"""CPU restatement of the per-subset hot path (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import,
call or execute this module, and only as the checker / timed CPU baseline.  The
product path (the HIP library) never routes through it.

What it restates
----------------
The reference worker ``partitioned_spMvGLM`` (MetaKriging_BinaryResponse.R:46-96)
fits ``spMvGLM`` (MK.R:80-84, binomial-logit, exponential or Matern LMC
covariance, adaptive Metropolis-within-Gibbs ``amcmc`` MK.R:83), krige with
``spPredict`` (MK.R:87) and summarise each column with 200 type-7 quantiles
(MK.R:88-89).  spBayes (a CRAN package, version unpinned, absent from this
container -- SURVEY.md section 8c) holds the arithmetic; its documented model
 is restated here and every internal choice is fixed
explicitly (DESIGN.md "Sampler specification").

PARITY STATUS: parity unpinned against spBayes itself (no R, no spBayes, no
reference fixtures).  Deterministic pieces (covariance, Cholesky, quantiles,
approx) are pinned against independent scipy/numpy implementations; the
incremental sampler is pinned against ``literal.py`` -- a restatement of
spBayes' own amcmc structure that recomputes the full log posterior
(covariance, dense Cholesky, quadratic form) for every single-parameter
proposal -- on identical Philox draws.

Algorithm (identical to the HIP library; see DESIGN.md for the derivation)
---------------------------------------------------------------------------
MH parameter vector, spBayes order: beta (p) | A lower-tri col-major, log-diag
(q(q+1)/2) | logit phi (q) | logit nu (q, Matern) | w (N = n*q, location major).
One-at-a-time Gaussian random-walk proposals, sd = exp(l_j), accept iff
log(U) <= log-posterior(candidate) - log-posterior(current).  The LMC
covariance C = (I_n (x) A) Rtilde (I_n (x) A') is never formed: every ratio is
computed from per-outcome correlation factors R_h = L_h L_h', Q_h = R_h^-1,
u = (I (x) A^-1) w and g_h = Q_h u_h, which gives the same ratios as spBayes'
dense recompute at O(N^2) instead of O(N^4) per iteration.
"""
import numpy as np
import scipy.linalg as sla
import scipy.special as ssp

from . import philox
from .rstats import PROBS200, r_quantile7

COV_EXPONENTIAL = 0
COV_MATERN = 1


# ----------------------------------------------------------------- small helpers
def logit_inv(z, a, b):
    """spBayes util logitInv(z, a, b) = b - (b - a) / (1 + exp(z))."""
    return b - (b - a) / (1.0 + np.exp(z))


def logit(theta, a, b):
    return np.log((theta - a) / (b - theta))


def softplus(x):
    """log(1 + exp(x)), stable form used by host and device alike."""
    return np.maximum(x, 0.0) + np.log1p(np.exp(-np.abs(x)))


LINK_LOGIT, LINK_PROBIT = 0, 1


def log_ndtr(x):
    """log Phi(x), the device's formula (csrc/mk_common.hpp log_norm_cdf): log1p(-erfc(x/sqrt2)/2)
    for x >= 0, log(erfcx(-x/sqrt2)/2) - x^2/2 below (no underflow)."""
    x = np.asarray(x, dtype=np.float64)
    r = 0.7071067811865476
    pos = x >= 0.0
    out = np.empty_like(x)
    out[pos] = np.log1p(-0.5 * ssp.erfc(x[pos] * r))
    xn = x[~pos]
    out[~pos] = np.log(0.5 * ssp.erfcx(-xn * r)) - 0.5 * xn * xn
    return out


def loglik_terms(y, wt, eta, link=LINK_LOGIT):
    """Binomial log-likelihood per observation (constants dropped).  logit (spMvGLM's binomial
    family, MK.R:80-84): y*eta - wt*log(1+exp(eta)); probit (north-star extension, no reference
    parity target): y log Phi(eta) + (wt - y) log Phi(-eta)."""
    if link == LINK_PROBIT:
        return y * log_ndtr(eta) + (wt - y) * log_ndtr(-eta)
    return y * eta - wt * softplus(eta)


def n_tri(q):
    return q * (q + 1) // 2


def tri_to_A(tri, q):
    """spBayes covTransInvExpand: lower-tri col-major vector (log diagonal) -> A."""
    A = np.zeros((q, q))
    k = 0
    for j in range(q):
        for i in range(j, q):
            A[i, j] = np.exp(tri[k]) if i == j else tri[k]
            k += 1
    return A


def A_to_tri(A):
    q = A.shape[0]
    out = []
    for j in range(q):
        for i in range(j, q):
            out.append(np.log(A[i, j]) if i == j else A[i, j])
    return np.array(out)


def lower_tri_vec(M):
    q = M.shape[0]
    return np.array([M[i, j] for j in range(q) for i in range(j, q)])


# ----------------------------------------------------------------- covariance
def correlation(d, phi, nu, cov_model):
    """spBayes spCor: exponential exp(-phi d); Matern (phi d)^nu/(2^(nu-1) Gamma(nu)) K_nu(phi d), 1 at d=0."""
    d = np.asarray(d, dtype=np.float64)
    if cov_model == COV_EXPONENTIAL:
        return np.exp(-phi * d)
    x = phi * d
    out = np.ones_like(x)
    pos = x > 0.0
    xp = x[pos]
    out[pos] = np.power(xp, nu) / (np.power(2.0, nu - 1.0) * ssp.gamma(nu)) * ssp.kv(nu, xp)
    return out


def distance_matrix(c1, c2):
    dx = c1[:, 0][:, None] - c2[:, 0][None, :]
    dy = c1[:, 1][:, None] - c2[:, 1][None, :]
    return np.sqrt(dx * dx + dy * dy)


def lmc_covariance(coords, A, phi, nu, cov_model):
    """Dense LMC covariance in spBayes' location-major order (used by literal.py and tests):
    C[(i,a),(j,b)] = sum_h A[a,h] A[b,h] rho_h(d_ij)."""
    n = coords.shape[0]
    q = A.shape[0]
    D = distance_matrix(coords, coords)
    C = np.zeros((n * q, n * q))
    for h in range(q):
        Rh = correlation(D, phi[h], nu[h] if nu is not None else 0.0, cov_model)
        C += np.kron(Rh, np.outer(A[:, h], A[:, h]))
    return C


def iw_logprior_A(A, df, S):
    """IW(df, S) log density of K = A A' (up to const) plus the Jacobian of
    (lower-tri A, log diagonal) -> K, exactly as spBayes spMvGLM accumulates it."""
    q = A.shape[0]
    dA = np.diag(A)
    logdetK = 2.0 * np.sum(np.log(dA))
    Ainv = sla.solve_triangular(A, np.eye(q), lower=True)
    Kinv = Ainv.T @ Ainv
    out = -0.5 * (df + q + 1.0) * logdetK - 0.5 * np.sum(S * Kinv.T)
    for k in range(q):
        out += (q - k) * np.log(dA[k]) + np.log(dA[k])
    return out, logdetK


def unif_jacobian(v, a, b):
    return np.log(v - a) + np.log(b - v)


# ----------------------------------------------------------------- configuration
class Config:
    """Mirrors the spMvGLM arguments the reference passes (MK.R:56-64, 83-85).

    Tuning values are proposal VARIANCES (spBayes amcmc semantics); the
    initial log proposal sd is log(sqrt(tuning)).  beta tuning is the diagonal
    of the matrix MK.R:55 builds (build decision)."""

    def __init__(self, q, p, beta_starting, beta_tuning, cov_model=COV_EXPONENTIAL,
                 n_batch=100, batch_length=50, accept_rate=0.43,
                 phi_starting=None, phi_tuning=None, phi_unif=None,
                 A_starting=None, A_tuning=None, w_starting=0.0, w_tuning=0.5,
                 nu_starting=None, nu_tuning=None, nu_unif=None,
                 K_IW_df=None, K_IW_S=None, burn_in=None, seed=20250114, link=LINK_LOGIT, beta_prior=None):
        self.q, self.p = q, p
        # TEST-ONLY (tests/test_geweke.py): a proper N(mean, sd^2) prior per beta_j as (mean, sd) arrays.
        # None is the reference's beta.Flat (MK.R:63) -- the sampler the device implements.
        self.beta_prior = None if beta_prior is None else (np.asarray(beta_prior[0], float),
                                                           np.asarray(beta_prior[1], float))
        self.link = int(link)
        self.cov_model = cov_model
        self.n_batch, self.batch_length = n_batch, batch_length
        self.n_samples = n_batch * batch_length
        self.accept_rate = accept_rate
        self.beta_starting = np.asarray(beta_starting, dtype=np.float64)
        bt = np.asarray(beta_tuning, dtype=np.float64)
        self.beta_tuning = np.diag(bt).copy() if bt.ndim == 2 else bt
        self.phi_starting = np.full(q, 3.0 / 0.5) if phi_starting is None else np.asarray(phi_starting, float)
        self.phi_tuning = np.ones(q) if phi_tuning is None else np.asarray(phi_tuning, float)
        if phi_unif is None:
            phi_unif = (np.full(q, 3.0 / 0.75), np.full(q, 3.0 / 0.25))
        self.phi_a, self.phi_b = (np.asarray(phi_unif[0], float), np.asarray(phi_unif[1], float))
        self.A_starting = lower_tri_vec(np.eye(q)) if A_starting is None else np.asarray(A_starting, float)
        self.A_tuning = np.full(n_tri(q), 0.1) if A_tuning is None else np.asarray(A_tuning, float)
        self.w_starting = float(w_starting)
        self.w_tuning = float(w_tuning)
        matern = cov_model == COV_MATERN
        self.nu_starting = (np.full(q, 0.5) if nu_starting is None else np.asarray(nu_starting, float)) if matern else None
        self.nu_tuning = (np.full(q, 0.1) if nu_tuning is None else np.asarray(nu_tuning, float)) if matern else None
        if matern:
            if nu_unif is None:
                nu_unif = (np.full(q, 0.1), np.full(q, 2.0))
            self.nu_a, self.nu_b = np.asarray(nu_unif[0], float), np.asarray(nu_unif[1], float)
        else:
            self.nu_a = self.nu_b = None
        self.K_IW_df = float(q) if K_IW_df is None else float(K_IW_df)
        self.K_IW_S = np.diag(np.full(q, 0.1)) if K_IW_S is None else np.asarray(K_IW_S, float)
        self.burn_in = int(0.75 * self.n_samples) if burn_in is None else int(burn_in)  # MK.R:85
        self.seed = int(seed)

    @property
    def n_theta(self):
        return n_tri(self.q) + self.q * (2 if self.cov_model == COV_MATERN else 1)

    @property
    def n_report(self):
        """Columns of p.beta.theta.samples: beta | K lower-tri | phi | (nu)."""
        return self.p + self.n_theta

    @property
    def kept(self):
        return self.n_samples - self.burn_in + 1


# ----------------------------------------------------------------- the sampler
def beta_logprior(b, j, cfg):
    """log N(b; mean_j, sd_j^2) up to a constant, for Config.beta_prior (test-only: the reference's beta
    prior is flat, MK.R:63, and contributes nothing to the ratio)."""
    mu, sd = cfg.beta_prior
    return -0.5 * ((b - mu[j]) / sd[j]) ** 2


_SWEEP_LIB = None


def _c_sweep():
    """ctypes handle of oracle/_sweep.so (make -C oracle), built on first use."""
    global _SWEEP_LIB
    if _SWEEP_LIB is None:
        import ctypes
        import os
        import subprocess
        here = os.path.dirname(os.path.abspath(__file__))
        so = os.path.join(here, "_sweep.so")
        if not os.path.exists(so):
            subprocess.check_call(["make", "-s", "-C", here, "_sweep.so"])
        lib = ctypes.CDLL(so)
        dp = ctypes.POINTER(ctypes.c_double)
        lib.mk_oracle_sweep.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, ctypes.POINTER(dp), dp, dp, dp,
                                        dp, dp]
        lib.mk_oracle_sweep.restype = None
        _SWEEP_LIB = lib
    return _SWEEP_LIB


def fit_subset(coords, y, wt, X, cfg, subset=0, coords_test=None, record_w=False,
               quantiles=True, max_iter=None, sweep="py", site_index=None, start=None):
    """One subset: spMvGLM amcmc fit with fused spPredict on kept iterations.

    coords (n,2); y, wt (N=n*q) location-major; X (N,p) block-diagonal design.
    Returns dict with 'samples' (n_samples,P) reported parameters, 'accept'
    (n_batch, n_mh) acceptance rates, 'tuning' final log-sd, 'w_pred' (kept,
    q*n_test) predictive draws, and (if quantiles) 'param_q' (200,P), 'w_q'
    (200, q*n_test).  max_iter truncates the chain (bounded CPU timing).  sweep="c" runs step 5
    (the latent-w sweep) in oracle/csrc/sweep.c -- the same operations in the same order -- for
    the CPU baseline's timing.  site_index (optional, [n_test] ints): the global index of each
    test site, so a sub-sample of a large kriging set (configs[4]: 1M sites) draws the same
    Philox streams as the device does for those sites (default 0..n_test-1).  start (optional):
    resume a chain -- a dict with 'iteration' (iterations already done) and the state after them in
    MH order, 'beta', 'theta' (A tri with log diagonal | logit phi | logit nu), 'w', 'tune' (log
    sds) and 'accept' (the current batch's counts), as the device's mk_session_chain_state returns
    it; the loop then runs iterations start['iteration'] .. max_iter - 1 with the same Philox
    counters (bench.py's CPU baseline times the device's window this way).  out['phase_seconds']
    splits the loop's time by step.
    """
    q, p = cfg.q, cfg.p
    n = coords.shape[0]
    N = n * q
    ntri = n_tri(q)
    matern = cfg.cov_model == COV_MATERN
    key = philox.make_key(cfg.seed, subset)
    y = np.asarray(y, float)
    wt = np.asarray(wt, float)
    X = np.asarray(X, float)

    # ---- parameter offsets (spBayes order)
    o_beta, o_A, o_phi = 0, p, p + ntri
    o_nu = o_phi + q
    o_w = o_phi + q * (2 if matern else 1)
    n_mh = o_w + N

    # ---- state
    beta = cfg.beta_starting.copy()
    A = tri_to_A(A_to_tri_start(cfg.A_starting, q), q)
    theta_phi = logit(cfg.phi_starting, cfg.phi_a, cfg.phi_b)
    theta_nu = logit(cfg.nu_starting, cfg.nu_a, cfg.nu_b) if matern else None
    w = np.full(N, cfg.w_starting)
    tune = np.concatenate([
        np.log(np.sqrt(cfg.beta_tuning)), np.log(np.sqrt(cfg.A_tuning)),
        np.log(np.sqrt(cfg.phi_tuning)),
        np.log(np.sqrt(cfg.nu_tuning)) if matern else np.zeros(0),
        np.full(N, np.log(np.sqrt(cfg.w_tuning)))])
    accept0 = None
    s_begin = 0
    if start is not None:
        s_begin = int(start["iteration"])
        beta = np.array(start["beta"], dtype=np.float64)
        th = np.asarray(start["theta"], dtype=np.float64)
        A = tri_to_A(th[:ntri], q)
        theta_phi = th[ntri:ntri + q].copy()
        if matern:
            theta_nu = th[ntri + q:ntri + 2 * q].copy()
        w = np.array(start["w"], dtype=np.float64)
        tune = np.array(start["tune"], dtype=np.float64)
        accept0 = np.array(start["accept"], dtype=np.float64)
    eta = X @ beta + w

    D = distance_matrix(coords, coords)

    def phi_of(h, th=None):
        return logit_inv(theta_phi[h] if th is None else th, cfg.phi_a[h], cfg.phi_b[h])

    def nu_of(h, th=None):
        if not matern:
            return 0.0
        return logit_inv(theta_nu[h] if th is None else th, cfg.nu_a[h], cfg.nu_b[h])

    def factor(h, phi_v, nu_v):
        R = correlation(D, phi_v, nu_v, cfg.cov_model)
        L = np.linalg.cholesky(R)
        return L, 2.0 * np.sum(np.log(np.diag(L)))

    L = [None] * q
    logdetR = np.zeros(q)
    Q = [None] * q
    for h in range(q):
        L[h], logdetR[h] = factor(h, phi_of(h), nu_of(h))
        Q[h] = cho_inverse(L[h])
    Ainv = sla.solve_triangular(A, np.eye(q), lower=True)
    U = (Ainv @ w.reshape(n, q).T).T           # u (n,q): u_i = A^-1 w_i
    G = np.stack([Q[h] @ U[:, h] for h in range(q)], axis=1)   # g_h = Q_h u_h

    if coords_test is not None:
        n_test = coords_test.shape[0]
        Dt = distance_matrix(coords_test, coords)
        P_cache = [None] * q       # (phi,nu) -> (P_h, s_h)
        site_ix = (np.arange(n_test, dtype=np.int64) if site_index is None
                   else np.asarray(site_index, dtype=np.int64).reshape(n_test))
    else:
        n_test = 0

    n_iter = cfg.n_samples if max_iter is None else min(max_iter, cfg.n_samples)
    samples = np.zeros((n_iter, cfg.n_report))
    w_samples = np.zeros((n_iter, N)) if record_w else None
    acc_hist = np.zeros((cfg.n_batch, n_mh))
    kept0 = cfg.burn_in - 1           # 0-based first kept iteration (R start=burn.in)
    w_pred = np.zeros((max(0, n_iter - kept0), q * n_test)) if n_test else None
    accept = np.zeros(n_mh) if accept0 is None else accept0

    import time as _time
    clock = _time.perf_counter
    phase = dict(beta_A=0.0, factor=0.0, inverse=0.0, sweep=0.0, krige=0.0, other=0.0)
    t_loop = clock()
    for s in range(s_begin, n_iter):
        t_ph = clock()
        b = s // cfg.batch_length
        # all proposal normals / accept draws for this iteration (one Philox call each)
        js = np.arange(n_mh)
        zs = philox.proposal_normal(key, js, s)
        logus = philox.accept_log_uniform(key, js, s)

        # ---------------- 1. beta_j (flat prior, MK.R:63): likelihood only
        for j in range(p):
            delta = np.exp(tune[o_beta + j]) * zs[o_beta + j]
            eta_c = eta + delta * X[:, j]
            ratio = np.sum(loglik_terms(y, wt, eta_c, cfg.link) - loglik_terms(y, wt, eta, cfg.link))
            if cfg.beta_prior is not None:      # test-only proper prior (Geweke test)
                ratio += beta_logprior(beta[j] + delta, j, cfg) - beta_logprior(beta[j], j, cfg)
            if logus[o_beta + j] <= ratio:
                beta[j] += delta
                eta = eta_c
                accept[o_beta + j] += 1

        # ---------------- 2. A entries: O(q^3) per proposal given T
        A_base = A.copy()
        if q == 1:
            Gc = G[:, :, None].copy()                  # G[:,h,c] = Q_h u_c
        else:
            Gc = np.stack([np.stack([Q[h] @ U[:, c] for c in range(q)], axis=1) for h in range(q)], axis=1)
        T = np.einsum('ic,ihd->hcd', U, Gc)           # T[h,c,d] = u_c . Q_h u_d

        def a_objective(Acand):
            M = sla.solve_triangular(Acand, A_base, lower=True)     # A'^-1 A_base
            quad = np.einsum('hc,hd,hcd->', M, M, T)
            lp, logdetK = iw_logprior_A(Acand, cfg.K_IW_df, cfg.K_IW_S)
            return -0.5 * n * logdetK - 0.5 * quad + lp

        tri = A_to_tri(A)
        f_cur = a_objective(A)
        for k in range(ntri):
            j = o_A + k
            cand = tri.copy()
            cand[k] += np.exp(tune[j]) * zs[j]
            Ac = tri_to_A(cand, q)
            f_c = a_objective(Ac)
            if logus[j] <= f_c - f_cur:
                tri = cand
                A = Ac
                f_cur = f_c
                accept[j] += 1
        Ainv = sla.solve_triangular(A, np.eye(q), lower=True)
        M = Ainv @ A_base
        U = (Ainv @ w.reshape(n, q).T).T
        G = np.einsum('hc,ihc->ih', M, Gc)

        # ---------------- 3. phi_h then nu_h: one Cholesky per proposal
        t_c = clock()
        phase["beta_A"] += t_c - t_ph
        t_ph = t_c
        quad_h = np.einsum('ih,ih->h', U, G)
        dirty = [False] * q
        for kind in (("phi", "nu") if matern else ("phi",)):
            for h in range(q):
                j = (o_phi if kind == "phi" else o_nu) + h
                if kind == "phi":
                    th_c = theta_phi[h] + np.exp(tune[j]) * zs[j]
                    v_c, v_cur = phi_of(h, th_c), phi_of(h)
                    a_, b_ = cfg.phi_a[h], cfg.phi_b[h]
                    Lc, ldc = factor(h, v_c, nu_of(h))
                else:
                    th_c = theta_nu[h] + np.exp(tune[j]) * zs[j]
                    v_c, v_cur = nu_of(h, th_c), nu_of(h)
                    a_, b_ = cfg.nu_a[h], cfg.nu_b[h]
                    Lc, ldc = factor(h, phi_of(h), v_c)
                zc = sla.solve_triangular(Lc, U[:, h], lower=True)
                quad_c = zc @ zc
                ratio = (-0.5 * (ldc - logdetR[h]) - 0.5 * (quad_c - quad_h[h])
                         + unif_jacobian(v_c, a_, b_) - unif_jacobian(v_cur, a_, b_))
                if logus[j] <= ratio:
                    if kind == "phi":
                        theta_phi[h] = th_c
                    else:
                        theta_nu[h] = th_c
                    L[h], logdetR[h], quad_h[h] = Lc, ldc, quad_c
                    dirty[h] = True
                    accept[j] += 1
        # ---------------- 4. refresh Q_h, g_h where R_h changed (and for every h at the
        #                     first kept iteration, where kriging needs fresh factors)
        t_c = clock()
        phase["factor"] += t_c - t_ph
        t_ph = t_c
        for h in range(q):
            if dirty[h] or s == kept0:
                Q[h] = cho_inverse(L[h])
                G[:, h] = Q[h] @ U[:, h]

        # ---------------- 5. single-site w sweep (site-major, outcome-minor)
        t_c = clock()
        phase["inverse"] += t_c - t_ph
        t_ph = t_c
        delta_w = np.exp(tune[o_w:o_w + N]) * zs[o_w:o_w + N]
        dll = loglik_terms(y, wt, eta + delta_w, cfg.link) - loglik_terms(y, wt, eta, cfg.link)
        lu = logus[o_w:o_w + N]
        Qdiag = np.stack([np.diag(Q[h]) for h in range(q)], axis=1)      # (n,q)
        if sweep == "c":
            import ctypes
            dp = ctypes.POINTER(ctypes.c_double)
            arrs = [np.ascontiguousarray(a_, dtype=np.float64) for a_ in (delta_w, dll, lu, Ainv, Qdiag)]
            G, U = np.ascontiguousarray(G), np.ascontiguousarray(U)   # updated in place below
            for a_ in (w, eta):
                assert a_.flags["C_CONTIGUOUS"] and a_.dtype == np.float64
            Qs = [np.ascontiguousarray(Q[h]) for h in range(q)]
            qptr = (dp * q)(*[a_.ctypes.data_as(dp) for a_ in Qs])
            acc_w = accept[o_w:o_w + N].copy()
            _c_sweep().mk_oracle_sweep(n, q, *[a_.ctypes.data_as(dp) for a_ in arrs], qptr, G.ctypes.data_as(dp),
                                       U.ctypes.data_as(dp), w.ctypes.data_as(dp), eta.ctypes.data_as(dp),
                                       acc_w.ctypes.data_as(dp))
            accept[o_w:o_w + N] = acc_w
        for k in (range(N) if sweep != "c" else ()):
            i, a = divmod(k, q)
            dl = delta_w[k]
            c = Ainv[:, a] @ G[i]
            d = (Ainv[:, a] ** 2) @ Qdiag[i]
            if lu[k] <= dll[k] - (dl * c + 0.5 * dl * dl * d):
                w[k] += dl
                eta[k] += dl
                coef = dl * Ainv[:, a]
                U[i] += coef
                for h in range(q):
                    G[:, h] += coef[h] * Q[h][:, i]
                accept[o_w + k] += 1

        # ---------------- 6. record
        t_c = clock()
        phase["sweep"] += t_c - t_ph
        t_ph = t_c
        K = A @ A.T
        samples[s, :p] = beta
        samples[s, p:p + ntri] = lower_tri_vec(K)
        samples[s, p + ntri:p + ntri + q] = [phi_of(h) for h in range(q)]
        if matern:
            samples[s, p + ntri + q:] = [nu_of(h) for h in range(q)]
        if record_w:
            w_samples[s] = w

        # ---------------- 7. fused spPredict on kept iterations
        t_c = clock()
        phase["other"] += t_c - t_ph
        t_ph = t_c
        if n_test and s >= kept0:
            key_s = s
            mean = np.zeros((n_test, q))
            sd = np.zeros((n_test, q))
            for h in range(q):
                ph, nh = phi_of(h), nu_of(h)
                if P_cache[h] is None or P_cache[h][0] != (ph, nh):
                    Ph = correlation(Dt, ph, nh, cfg.cov_model)            # (n_test, n)
                    Xh = sla.solve_triangular(L[h], Ph.T, lower=True)      # L^-1 P'
                    sh = np.einsum('it,it->t', Xh, Xh)
                    P_cache[h] = ((ph, nh), Ph, sh)
                _, Ph, sh = P_cache[h]
                mean[:, h] = Ph @ G[:, h]
                sd[:, h] = np.sqrt(np.maximum(1.0 - sh, 0.0))
            idx = (site_ix[:, None] * q + np.arange(q)[None, :]).reshape(-1)
            zt = philox.predict_normal(key, idx, key_s).reshape(n_test, q)
            draw = (mean + sd * zt) @ A.T                                # A(mean_h + sd_h z_h)
            w_pred[s - kept0] = draw.reshape(-1)

        # ---------------- 8. batch end: adapt log-sd toward accept_rate
        t_c = clock()
        phase["krige"] += t_c - t_ph
        t_ph = t_c
        if (s + 1) % cfg.batch_length == 0:
            rate = accept / cfg.batch_length
            acc_hist[b] = rate
            step = min(0.01, 1.0 / np.sqrt(b)) if b > 0 else 0.01
            tune = np.where(rate > cfg.accept_rate, tune + step, tune - step)
            accept[:] = 0.0
        phase["other"] += clock() - t_ph

    out = dict(samples=samples, accept=acc_hist, tuning=tune, w_pred=w_pred,
               beta=beta, A=A, w=w, n_iter=n_iter, loop_seconds=clock() - t_loop, phase_seconds=phase)
    # the state after the last iteration, in the layout `start` takes (and mk_session_chain_state returns)
    th_out = [A_to_tri(A), theta_phi] + ([theta_nu] if matern else [])
    out["state"] = dict(iteration=n_iter, beta=beta.copy(), theta=np.concatenate(th_out), w=w.copy(),
                        tune=tune.copy(), accept=accept.copy())
    if record_w:
        out["w_samples"] = w_samples
    if quantiles and n_iter >= cfg.n_samples:
        kept = samples[kept0:]
        out["param_q"] = r_quantile7(kept, PROBS200, axis=0)
        if n_test:
            out["w_q"] = r_quantile7(w_pred, PROBS200, axis=0)
    return out


def A_to_tri_start(A_start_tri, q):
    """starting$A is the lower triangle of A itself (MK.R:56); store the log of its diagonal."""
    out = np.array(A_start_tri, dtype=np.float64).copy()
    k = 0
    for j in range(q):
        for i in range(j, q):
            if i == j:
                out[k] = np.log(out[k])
            k += 1
    return out


def cho_inverse(L):
    """R^-1 from its lower Cholesky factor (LAPACK dpotri), full symmetric."""
    inv, info = sla.lapack.dpotri(L, lower=1)
    if info != 0:
        raise np.linalg.LinAlgError("dpotri failed")
    inv = np.tril(inv)
    return inv + np.tril(inv, -1).T


# ----------------------------------------------------------------- combine (MK.R:119-133)
def combine_mean(grids):
    """result <- obj[[1]]; for(k in 2:K) result <- result + obj[[k]]; result/K (sequential order)."""
    acc = np.array(grids[0], dtype=np.float64, copy=True)
    for g in grids[1:]:
        acc = acc + g
    return acc / len(grids)
