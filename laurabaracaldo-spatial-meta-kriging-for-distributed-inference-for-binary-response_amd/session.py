"""Host handle on one GPU shard of subsets (mk_session in include/mk.h).

This is the batched replacement of ``foreach(i=1:n.core) %dopar%
partitioned_spMvGLM(...)`` (MetaKriging_BinaryResponse.R:108): all subsets of
the shard live in HBM, every MCMC iteration advances all of them at once.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import Config, Outputs, Problem, check, dptr, iptr

COV_MODELS = {"exponential": _lib.MK_COV_EXPONENTIAL, "matern": _lib.MK_COV_MATERN}
LINKS = {"logit": _lib.MK_LINK_LOGIT, "probit": _lib.MK_LINK_PROBIT}

# kernel-stat ids (mk_api.hip)
(KS_CHOL_UPDATE, KS_CHOL_DIAG, KS_CHOL_TRSM, KS_SWEEP, KS_LAUUM, KS_ITER, KS_INV, KS_CHOL_UPDATE_SUB, KS_UPDATE_BUSY,
 KS_PRED_VAR, KS_COV, KS_SWEEP_FALLBACK, KS_KRIG_CHEB, KS_KRIG_FALLBACK) = range(14)


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


class SamplerConfig:
    """spMvGLM arguments of MK.R:56-64, 80-85 in one place (R names in comments)."""

    def __init__(self, q, p, beta_starting, beta_tuning, cov_model="exponential", n_batch=100, batch_length=50,
                 accept_rate=0.43, burn_in=None, phi_starting=None, phi_tuning=None, phi_unif=None,
                 A_starting=None, A_tuning=None, w_starting=0.0, w_tuning=0.5, nu_starting=None, nu_tuning=None,
                 nu_unif=None, K_IW_df=None, K_IW_S=None, seed=20250114, n_streams=0, predict_tile=0,
                 link="logit"):
        if cov_model not in COV_MODELS:
            raise ValueError(f"error: specified cov.model '{cov_model}' is not a valid option")
        if link not in LINKS:
            raise ValueError(f"error: link must be 'logit' (the reference) or 'probit', not '{link}'")
        self.link = link
        self.q, self.p = int(q), int(p)
        self.cov_model = cov_model
        self.n_batch, self.batch_length = int(n_batch), int(batch_length)
        self.n_samples = self.n_batch * self.batch_length
        self.accept_rate = float(accept_rate)
        self.burn_in = int(0.75 * self.n_samples) if burn_in is None else int(burn_in)   # MK.R:85
        bt = np.asarray(beta_tuning, dtype=np.float64)
        if bt.ndim == 2:
            bt = np.diag(bt)           # amcmc uses one scalar tuning per beta (build decision)
        if bt.shape != (self.p,):
            raise ValueError(f"error: beta tuning must be of length {self.p}")
        self.beta_starting = _f64(beta_starting).reshape(self.p)
        self.beta_tuning = _f64(bt)
        q = self.q
        self.phi_starting = _f64(np.full(q, 3.0 / 0.5) if phi_starting is None else phi_starting).reshape(q)
        self.phi_tuning = _f64(np.ones(q) if phi_tuning is None else phi_tuning).reshape(q)
        if phi_unif is None:
            phi_unif = (np.full(q, 3.0 / 0.75), np.full(q, 3.0 / 0.25))
        self.phi_a = _f64(phi_unif[0]).reshape(q)
        self.phi_b = _f64(phi_unif[1]).reshape(q)
        ntri = q * (q + 1) // 2
        if A_starting is None:   # diag(1,q)[lower.tri(diag(1,q), TRUE)]  (MK.R:56)
            A_starting = np.array([1.0 if i == j else 0.0 for j in range(q) for i in range(j, q)])
        self.A_starting = _f64(A_starting).reshape(ntri)
        self.A_tuning = _f64(np.full(ntri, 0.1) if A_tuning is None else A_tuning).reshape(ntri)
        self.w_starting, self.w_tuning = float(w_starting), float(w_tuning)
        matern = cov_model == "matern"
        if matern:
            self.nu_starting = _f64(np.full(q, 0.5) if nu_starting is None else nu_starting).reshape(q)
            self.nu_tuning = _f64(np.full(q, 0.1) if nu_tuning is None else nu_tuning).reshape(q)
            if nu_unif is None:
                nu_unif = (np.full(q, 0.1), np.full(q, 2.0))
            self.nu_a = _f64(nu_unif[0]).reshape(q)
            self.nu_b = _f64(nu_unif[1]).reshape(q)
        else:
            self.nu_starting = self.nu_tuning = self.nu_a = self.nu_b = None
        self.K_IW_df = float(q if K_IW_df is None else K_IW_df)
        self.K_IW_S = _f64(np.diag(np.full(q, 0.1)) if K_IW_S is None else K_IW_S).reshape(q, q)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.n_streams = int(n_streams)     # device execution only (0 = library default); no effect on results
        self.predict_tile = int(predict_tile)   # 0: kriging fused into kept iterations; else test sites per pass

    @property
    def n_theta(self):
        return self.q * (self.q + 1) // 2 + self.q * (2 if self.cov_model == "matern" else 1)

    @property
    def P(self):
        return self.p + self.n_theta

    @property
    def kept(self):
        return self.n_samples - self.burn_in + 1

    def to_c(self, device=0, record_w=False):
        keep = []

        def p_(a):
            if a is None:
                return None
            a = _f64(a)
            keep.append(a)
            return dptr(a)

        c = Config()
        c.cov_model = COV_MODELS[self.cov_model]
        c.n_batch, c.batch_length, c.accept_rate, c.burn_in = self.n_batch, self.batch_length, self.accept_rate, self.burn_in
        c.beta_starting, c.beta_tuning = p_(self.beta_starting), p_(self.beta_tuning)
        c.phi_starting, c.phi_tuning = p_(self.phi_starting), p_(self.phi_tuning)
        c.A_starting, c.A_tuning = p_(self.A_starting), p_(self.A_tuning)
        c.nu_starting, c.nu_tuning = p_(self.nu_starting), p_(self.nu_tuning)
        c.w_starting, c.w_tuning = self.w_starting, self.w_tuning
        c.phi_unif_a, c.phi_unif_b = p_(self.phi_a), p_(self.phi_b)
        c.nu_unif_a, c.nu_unif_b = p_(self.nu_a), p_(self.nu_b)
        c.K_IW_df = self.K_IW_df
        c.K_IW_S = p_(np.asfortranarray(self.K_IW_S).ravel(order="F"))
        c.seed = self.seed
        c.record_samples = 1
        c.record_w = 1 if record_w else 0
        c.device = int(device)
        c.n_streams = self.n_streams
        c.predict_tile = self.predict_tile
        c.link = LINKS[self.link]
        return c, keep


class PackedProblem:
    """mk_problem of a list of subsets (the R layout libmk reads: per subset column-major coords,
    location-major y / weights, (n_s q) x p design), with the arrays it points into kept alive."""

    def __init__(self, subsets, cfg, coords_test=None, subset_base=0):
        self.n_part = np.ascontiguousarray([s["coords"].shape[0] for s in subsets], dtype=np.int32)
        self.S = len(subsets)
        self.coords = _f64(np.concatenate([np.asarray(s["coords"], float).ravel(order="F") for s in subsets]))
        self.y = _f64(np.concatenate([np.asarray(s["y"], float).ravel() for s in subsets]))
        self.weights = _f64(np.concatenate([np.asarray(s["weights"], float).ravel() for s in subsets]))
        self.x = _f64(np.concatenate([np.asarray(s["x"], float).reshape(-1, cfg.p).ravel(order="F") for s in subsets]))
        for s, ns in zip(subsets, self.n_part):
            if np.asarray(s["y"]).size != ns * cfg.q or np.asarray(s["x"]).shape != (ns * cfg.q, cfg.p):
                raise ValueError("error: subset y/x sizes must be n_s*q and (n_s*q) x p")
        self.n_test = 0 if coords_test is None else int(np.asarray(coords_test).shape[0])
        self.coords_test = None if coords_test is None else _f64(np.asarray(coords_test, float).ravel(order="F"))
        pr = Problem()
        pr.n_subsets, pr.subset_base, pr.q, pr.p = self.S, int(subset_base), cfg.q, cfg.p
        pr.n_part = iptr(self.n_part)
        pr.coords, pr.y, pr.weights, pr.x = dptr(self.coords), dptr(self.y), dptr(self.weights), dptr(self.x)
        pr.n_test = self.n_test
        pr.coords_test = dptr(self.coords_test) if self.coords_test is not None else None
        self.c = pr


class Session:
    """One shard of subsets resident on one GPU.

    subsets: list of dicts with 'coords' (n_s,2), 'y' (n_s*q,), 'weights' (n_s*q,), 'x' (n_s*q, p).
    """

    def __init__(self, subsets, cfg, coords_test=None, subset_base=0, device=0, record_w=False, lookahead=None):
        lib = _lib.load()
        self.cfg = cfg
        self.q, self.p = cfg.q, cfg.p
        self._prob = PackedProblem(subsets, cfg, coords_test, subset_base)
        self.n_part, self.S = self._prob.n_part, self._prob.S
        self.n_test, self.coords_test = self._prob.n_test, self._prob.coords_test
        pr = self._prob.c
        c, self._keep = cfg.to_c(device=device, record_w=record_w)
        self.record_w = record_w
        h = ctypes.c_void_p()
        check(lib.mk_session_create(ctypes.byref(pr), ctypes.byref(c), ctypes.byref(h)))
        self._h = h
        self._lib = lib
        if lookahead is not None:
            self.set_lookahead(lookahead)

    def run(self, n_iter):
        check(self._lib.mk_session_run(self._h, int(n_iter)))

    def chain_state(self, i):
        """Subset i's chain state now (mk_session_chain_state): beta, theta (A tri with log diagonal |
        logit phi | logit nu), w (n_s q), tune (log proposal sds) and accept (this batch's counts), in
        spMvGLM's MH order -- enough to resume the chain on another host at iteration `self.iteration`."""
        cfg = self.cfg
        nq = int(self.n_part[i]) * cfg.q
        nmh = cfg.p + cfg.n_theta + nq
        st = dict(beta=np.zeros(cfg.p), theta=np.zeros(cfg.n_theta), w=np.zeros(nq), tune=np.zeros(nmh),
                  accept=np.zeros(nmh))
        check(self._lib.mk_session_chain_state(self._h, int(i), dptr(st["beta"]), dptr(st["theta"]), dptr(st["w"]),
                                               dptr(st["tune"]), dptr(st["accept"])))
        st["iteration"] = self.iteration
        return st

    def set_test_sites(self, coords_test):
        """Kriging sites for the next outputs() of a session created with predict_tile > 0
        (its kept chain states were recorded during the run): spPredict without refitting."""
        ct = np.asarray(coords_test, float).reshape(-1, 2)
        self.n_test = int(ct.shape[0])
        self.coords_test = _f64(ct.ravel(order="F"))
        check(self._lib.mk_session_set_test_sites(self._h, self.n_test, dptr(self.coords_test)))

    def grids_device(self, which, out_ptr):
        """Write the shard's (S, C, 200) grids -- which 0 parameters, 1 w.predict -- into device memory
        at out_ptr (HBM of the session's device, e.g. a torch CUDA tensor's data_ptr()): the
        device-resident combine's input, no host round trip."""
        check(self._lib.mk_session_grids(self._h, int(which), ctypes.c_void_p(int(out_ptr)), 1))

    def tile_grids(self, t0):
        """Tiled session (predict_tile > 0), after the run: (S, 200, q*Tc) w.predict grids of test
        sites [t0, t0 + Tc) -- one tile's kriging replay only (configs[4]'s per-tile combine)."""
        T = self.predict_tile
        Tc = min(T, self.n_test - int(t0))
        out = np.zeros((self.S, self.q * Tc, _lib.N_LEVELS))
        check(self._lib.mk_session_tile_grids(self._h, int(t0), out.ctypes.data_as(ctypes.c_void_p), 0))
        return np.ascontiguousarray(np.transpose(out, (0, 2, 1)))

    def set_kept_window(self, first, last):
        """Replay only iterations first..last (1-based; spPredict's start / end) in the next outputs()."""
        check(self._lib.mk_session_set_kept_window(self._h, int(first), int(last)))
        self._window = int(last) - int(first) + 1

    def set_lookahead(self, mode):
        """Launch schedule before the first run: True / 1 lookahead (the next iteration's phi
        candidates factored while this iteration's inverse and sweep run), False / 0 sequential,
        -1 the library default.  The chain is the same either way (to rounding)."""
        check(self._lib.mk_session_set_lookahead(self._h, int(mode)))

    @property
    def lookahead(self):
        return bool(self._lib.mk_session_lookahead(self._h))

    @property
    def iteration(self):
        return self._lib.mk_session_iteration(self._h)

    @property
    def predict_tile(self):
        """Test sites per kriging tile in use (0: fused): cfg.predict_tile, or smaller where the tile's
        kriging buffers would not fit in HBM (the draws do not depend on it)."""
        return int(self._lib.mk_session_predict_tile(self._h))

    def profile(self, on=True, kinds=None, every=1):
        """Per-kernel HIP-event timing from the next run on: every kind, or only `kinds`
        (KS_* constants; fewer events in the stream); every > 1 brackets only the launches of every
        every-th iteration (a sample: per-launch events cost ~4 % of the rate at 32 subsets)."""
        check(self._lib.mk_session_profile_every(self._h, int(every)))
        if not on:
            v = 0
        elif kinds is None:
            v = 1
        else:
            v = 0
            for k in kinds:
                v |= 2 << int(k)
        check(self._lib.mk_session_profile(self._h, v))

    def kernel_stats(self, which):
        n = ctypes.c_int64()
        ms = ctypes.c_double()
        fl = ctypes.c_double()
        check(self._lib.mk_session_kernel_stats(self._h, which, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(fl)))
        return dict(launches=n.value, ms=ms.value, flops=fl.value)

    def outputs(self, quantiles=True, samples=False, w_samples=False, w_pred_samples=False, acceptance=False,
                w_predict_sum=False, w_predict=True):
        """quantiles: obj[[i]]$parameters (and $w.predict unless w_predict=False -- at 1M test sites the
        per-subset grids are 1.6 GB each; w_predict_sum gives this shard's term of the combine)."""
        cfg = self.cfg
        S, P, q = self.S, cfg.P, cfg.q
        o = Outputs()
        res = {}
        if quantiles:
            res["parameters"] = np.zeros((S, P, _lib.N_LEVELS))
            o.parameters = dptr(res["parameters"])
            if self.n_test and w_predict:
                res["w_predict"] = np.zeros((S, q * self.n_test, _lib.N_LEVELS))
                o.w_predict = dptr(res["w_predict"])
        if samples:
            res["samples"] = np.zeros((S, P, cfg.n_samples))
            o.samples = dptr(res["samples"])
        if w_samples:
            tot = int(self.n_part.sum()) * q * cfg.n_samples
            res["_w_samples_flat"] = np.zeros(tot)
            o.w_samples = dptr(res["_w_samples_flat"])
        if w_pred_samples and self.n_test:
            res["w_pred_samples"] = np.zeros((S, getattr(self, "_window", cfg.kept), q * self.n_test))
            o.w_pred_samples = dptr(res["w_pred_samples"])
        if acceptance:
            nrep = cfg.p + cfg.n_theta + 1
            res["acceptance"] = np.zeros((S, nrep, cfg.n_batch))
            o.acceptance = dptr(res["acceptance"])
        if w_predict_sum and self.n_test:
            res["w_predict_sum"] = np.zeros((q * self.n_test, _lib.N_LEVELS))
            o.w_predict_sum = dptr(res["w_predict_sum"])
        check(self._lib.mk_session_outputs(self._h, ctypes.byref(o)))
        out = {}
        # device/R layout: per subset column-major (levels x cols) == row-major (cols, levels)
        if "parameters" in res:
            out["parameters"] = [res["parameters"][i].T.copy() for i in range(S)]          # 200 x P
        if "w_predict" in res:
            out["w_predict"] = [res["w_predict"][i].T.copy() for i in range(S)]            # 200 x q*n_test
        if "samples" in res:
            out["samples"] = [res["samples"][i].T.copy() for i in range(S)]                # n_samples x P
        if "_w_samples_flat" in res:
            flat, off, ws = res["_w_samples_flat"], 0, []
            for ns in self.n_part:
                N = int(ns) * q
                ws.append(flat[off:off + N * cfg.n_samples].reshape(cfg.n_samples, N).T.copy())   # N x n_samples
                off += N * cfg.n_samples
            out["w_samples"] = ws
        if "w_pred_samples" in res:
            out["w_pred_samples"] = [res["w_pred_samples"][i].T.copy() for i in range(S)]  # (q n_test) x kept
        if "w_predict_sum" in res:
            out["w_predict_sum"] = res["w_predict_sum"].T.copy()                               # 200 x q*n_test
        if "acceptance" in res:
            out["acceptance"] = [res["acceptance"][i].T.copy() for i in range(S)]          # n_batch x nrep
        return out

    def close(self):
        if getattr(self, "_h", None):
            self._lib.mk_session_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def combine(grids, device=0, mean=True):
    """MK.R:123-133 on device: (grid_1 + ... + grid_K)/K in the reference's sequential order
    (mean=False: the sum only -- a shard's term of the combine)."""
    lib = _lib.load()
    g = _f64(np.stack([np.asarray(x, float) for x in grids]))
    K = g.shape[0]
    out = np.zeros(g.shape[1:])
    fn = lib.mk_combine if mean else lib.mk_combine_sum
    check(fn(dptr(g.reshape(K, -1)), K, int(np.prod(g.shape[1:])), dptr(out), int(device)))
    return out


def correlation_batched(coords, phi, nu=None, cov_model="exponential", device=0):
    """R_k = rho(|s_i - s_j|) for a batch of point sets (coords (S, n, 2))."""
    lib = _lib.load()
    coords = np.asarray(coords, float)
    S, n, _ = coords.shape
    c = _f64(np.stack([coords[i].ravel(order="F") for i in range(S)]))
    ph = _f64(np.broadcast_to(np.asarray(phi, float), (S,)))
    nv = None if nu is None else _f64(np.broadcast_to(np.asarray(nu, float), (S,)))
    out = np.zeros((S, n, n))
    check(lib.mk_correlation_batched(dptr(c), S, n, dptr(ph), dptr(nv) if nv is not None else None,
                                     COV_MODELS[cov_model], dptr(out), int(device)))
    return np.ascontiguousarray(np.transpose(out, (0, 2, 1)))   # column-major -> (S, n, n) row-major


def cholesky_batched(A, inverse=False, device=0):
    """Lower Cholesky factors, log-determinants (and inverses) of a batch of SPD matrices (S, n, n)."""
    lib = _lib.load()
    A = np.asarray(A, float)
    S, n, _ = A.shape
    a = _f64(np.transpose(A, (0, 2, 1)))          # row-major (S,n,n) -> column-major per matrix
    L = np.zeros((S, n, n))
    ld = np.zeros(S)
    inv = np.zeros((S, n, n)) if inverse else None
    check(lib.mk_cholesky_batched(dptr(a), S, n, dptr(L), dptr(ld), dptr(inv) if inverse else None, int(device)))
    L = np.ascontiguousarray(np.transpose(L, (0, 2, 1)))
    if inverse:
        inv = np.ascontiguousarray(np.transpose(inv, (0, 2, 1)))
        return L, ld, inv
    return L, ld
