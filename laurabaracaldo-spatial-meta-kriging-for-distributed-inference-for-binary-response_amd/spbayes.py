"""spMvGLM / spPredict drop-ins (the spBayes surface MK.R:80-89 uses).

Argument names and meaning follow spBayes as called by the reference:

  spMvGLM(formula=list(Y1 ~ X1 - 1, ...), coords, weights = n x q matrix,
          starting = list(beta, phi, A, w[, nu]), tuning = list(beta, phi, A, w[, nu]),
          priors = list("beta.Flat", phi.Unif = list(a, b), K.IW = list(df, S)[, nu.Unif]),
          amcmc = list(n.batch, batch.length, accept.rate), cov.model, n.report)
  spPredict(sp.obj, pred.coords, pred.covars, start, end)

``formula`` is a list of (Y_a, X_a) pairs (Y_a: n responses, X_a: n x p_a
design without intercept handling -- the ``Y ~ X - 1`` form of MK.R:80).
Errors are raised as ValueError / MkError where spBayes would stop().

spMvGLM keeps its device session open with every chain state recorded
(predict_tile mode, burn_in = 1); spPredict then only runs the kriging: it sets
the prediction sites (mk_session_set_test_sites) and replays the kept states of
iterations start..end (mk_session_set_kept_window) -- no refit.  Every kriging
draw has its own Philox stream keyed by the iteration, so the draws equal those of
a fit that fused the kriging into iterations start..end.
"""
import numpy as np

from .session import SamplerConfig, Session

PREDICT_TILE = 65536   # test sites per kriging pass in spPredict (device buffers per pass)


def _stack(formula, weights):
    q = len(formula)
    n = np.asarray(formula[0][0]).shape[0]
    ps = [np.asarray(X, float).reshape(n, -1).shape[1] for _, X in formula]
    p = sum(ps)
    y = np.zeros(n * q)
    X = np.zeros((n * q, p))
    off = 0
    for a, (Ya, Xa) in enumerate(formula):
        Ya = np.asarray(Ya, float).reshape(-1)
        Xa = np.asarray(Xa, float).reshape(n, -1)
        if Ya.shape[0] != n:
            raise ValueError("error: every outcome needs the same number of locations")
        y[a::q] = Ya
        X[a::q, off:off + ps[a]] = Xa
        off += ps[a]
    w = np.asarray(weights, float)
    w = np.broadcast_to(w, (n, q)) if w.ndim < 2 else w
    if w.shape != (n, q):
        raise ValueError("error: weights must be a n x q matrix")
    return q, p, n, y, X, np.ascontiguousarray(w).reshape(-1)


def _config(q, p, starting, tuning, priors, amcmc, cov_model, burn_in=None, seed=20250114):
    if amcmc is None:
        raise ValueError("error: this build implements the amcmc (adaptive) sampler only, as MK.R:83 uses")
    if "beta" not in starting or "beta" not in tuning:
        raise ValueError("error: beta must be specified in starting and tuning")
    for nm in ("phi", "A", "w"):
        if nm not in starting:
            raise ValueError(f"error: {nm} must be specified in starting")
        if nm not in tuning:
            raise ValueError(f"error: {nm} must be specified in tuning")
    if "phi.Unif" not in priors or "K.IW" not in priors:
        raise ValueError("error: phi.Unif and K.IW must be specified in priors")
    phi_u = priors["phi.Unif"]
    kiw = priors["K.IW"]
    matern = cov_model == "matern"
    if matern and ("nu" not in starting or "nu" not in tuning or "nu.Unif" not in priors):
        raise ValueError("error: nu must be specified in starting, tuning and priors (nu.Unif) for matern")
    return SamplerConfig(
        q, p, beta_starting=starting["beta"], beta_tuning=tuning["beta"], cov_model=cov_model,
        n_batch=amcmc["n.batch"], batch_length=amcmc["batch.length"], accept_rate=amcmc.get("accept.rate", 0.43),
        burn_in=burn_in, phi_starting=np.broadcast_to(np.asarray(starting["phi"], float), (q,)),
        phi_tuning=np.broadcast_to(np.asarray(tuning["phi"], float), (q,)),
        phi_unif=(np.broadcast_to(np.asarray(phi_u[0], float), (q,)), np.broadcast_to(np.asarray(phi_u[1], float), (q,))),
        A_starting=starting["A"], A_tuning=np.broadcast_to(np.asarray(tuning["A"], float), (q * (q + 1) // 2,)),
        w_starting=float(np.asarray(starting["w"]).reshape(-1)[0]), w_tuning=float(np.asarray(tuning["w"]).reshape(-1)[0]),
        nu_starting=None if not matern else np.broadcast_to(np.asarray(starting["nu"], float), (q,)),
        nu_tuning=None if not matern else np.broadcast_to(np.asarray(tuning["nu"], float), (q,)),
        nu_unif=None if not matern else (np.broadcast_to(np.asarray(priors["nu.Unif"][0], float), (q,)),
                                         np.broadcast_to(np.asarray(priors["nu.Unif"][1], float), (q,))),
        K_IW_df=kiw[0], K_IW_S=np.asarray(kiw[1], float).reshape(q, q), seed=seed)


class SpMvGLMFit(dict):
    """Result of spMvGLM: keys 'p.beta.theta.samples' (n.samples x P), 'p.w.samples'
    ((n q) x n.samples), 'acceptance' (n.batch x (p + n_theta + 1)), plus the inputs
    spPredict needs.

    The fit holds its device session (every recorded chain state, for spPredict) until
    ``close()`` -- or the end of a ``with`` block, or garbage collection.  Close fits you no
    longer predict from when fitting many subsets in a loop: each holds its factors in HBM."""

    def close(self):
        ses = self.pop("_session", None)
        if ses is not None:
            ses.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def spMvGLM(formula, coords, weights, starting, tuning, priors, amcmc, cov_model="exponential",
            family="binomial", n_report=10, seed=20250114, device=0, subset_index=0):
    if family != "binomial":
        raise ValueError("error: family must be binomial (the reference's binary response)")
    q, p, n, y, X, wt = _stack(formula, weights)
    coords = np.asarray(coords, float).reshape(n, 2)
    cfg = _config(q, p, starting, tuning, priors, amcmc, cov_model, burn_in=1, seed=seed)
    cfg.predict_tile = PREDICT_TILE          # record every chain state for spPredict
    sub = dict(coords=coords, y=y, weights=wt, x=X)
    ses = Session([sub], cfg, subset_base=subset_index, device=device, record_w=True)
    try:
        ses.run(cfg.n_samples)
        out = ses.outputs(quantiles=False, samples=True, w_samples=True, acceptance=True)
    except Exception:
        ses.close()
        raise
    fit = SpMvGLMFit()
    fit["p.beta.theta.samples"] = out["samples"][0]
    fit["p.w.samples"] = out["w_samples"][0]
    fit["acceptance"] = out["acceptance"][0]
    fit["_session"] = ses                    # closed when the fit object is collected
    fit["_n_samples"] = cfg.n_samples
    return fit


def spPredict(sp_obj, pred_coords, pred_covars=None, start=1, end=None, thin=1):
    """p.w.predictive.samples ((q n_test) x kept) for kept iterations start..end (1-based,
    inclusive; every thin-th), kriged from the chain states spMvGLM recorded (no refit)."""
    ses = sp_obj.get("_session")
    if ses is None:
        raise ValueError("error: the spMvGLM fit was closed; spPredict needs its recorded chain states")
    n_samples = sp_obj["_n_samples"]
    end = n_samples if end is None else int(end)
    start = int(start)
    if not (1 <= start <= end <= n_samples):
        raise ValueError("error: invalid start/end")
    ses.set_test_sites(np.asarray(pred_coords, float).reshape(-1, 2))
    ses.set_kept_window(start, end)
    out = ses.outputs(quantiles=False, w_pred_samples=True)
    wp = out["w_pred_samples"][0]                  # (q n_test) x (end - start + 1)
    return {"p.w.predictive.samples": wp[:, ::int(thin)]}
