"""Steps either side of the fits, on device (include/mk.h).

  combine_median     Weiszfeld geometric median of the subset quantile grids (north-star combine
                     extension; the reference averages them, MK.R:123-133)
  posterior_summary  MK.R:136-165: approx() to Xout, shared resample index, p(y=1), summaries
"""
import numpy as np

from . import _lib
from ._lib import Summary, check, dptr, iptr


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def combine_median(grids, max_iter=100, tol=1e-12, device=0):
    """grids: K arrays of L x C (obj[[k]]$parameters or $w.predict).  Returns (median L x C,
    iterations per column).  Column c is the W2 geometric median of the K quantile functions."""
    lib = _lib.load()
    g = np.stack([np.asarray(x, dtype=np.float64) for x in grids])
    K, L = g.shape[:2]
    C = int(np.prod(g.shape[2:])) if g.ndim > 2 else 1
    flat = _f64(np.stack([gk.reshape(L, C).ravel(order="F") for gk in g]))
    out = np.zeros(L * C)
    it = np.zeros(C, dtype=np.int32)
    check(lib.mk_combine_median(dptr(flat), K, L, C, int(max_iter), float(tol), dptr(out), iptr(it), int(device)))
    return out.reshape(L, C, order="F").reshape(g.shape[1:]), it


def posterior_summary(result, result2, x_test, q=None, samplesize=1000, seed=20250114, device=0, p_sample=True,
                      rng="philox", index=None, link="logit"):
    """MK.R:136-165 on device.  result: 200 x P combined parameter grid (betas first, MK.R:159);
    result2: 200 x C combined w.predict grid; x_test: C x p.  Returns SamplePar, Samplew,
    p_sample (samplesize x ...), w_quant (3 x C), param_quant (3 x P), p_quant (3 x C), index
    (0-based rows of the 996-level grid).

    sampleparIndex (MK.R:141): rng="philox" draws it from Philox(seed); rng="R" replays R's
    sample(seq(1, 996, 1), samplesize, replace=TRUE) right after set.seed(seed)
    (mk_r_sample_replace); index= takes a caller-drawn 1-based vector (R's own stream).
    link="probit" evaluates p(y=1) = Phi(x.test B + w) (extension; MK.R:160 is logistic)."""
    from .session import LINKS
    lib = _lib.load()
    if link not in LINKS:
        raise ValueError(f"error: link must be 'logit' or 'probit', not '{link}'")
    if index is None and rng == "R":
        index = np.empty(int(samplesize), dtype=np.int32)
        check(lib.mk_r_sample_replace(int(seed), 996, int(samplesize), iptr(index)))
    elif index is None and rng != "philox":
        raise ValueError(f"error: rng must be 'philox' or 'R', not '{rng}'")
    idx_in = None
    if index is not None:
        idx_in = np.ascontiguousarray(np.asarray(index), dtype=np.int32)
        if idx_in.shape != (int(samplesize),):
            raise ValueError("error: index must have samplesize entries")
    result = np.asarray(result, dtype=np.float64)
    P = result.shape[1]
    res = _f64(result.ravel(order="F"))
    C = 0 if result2 is None else int(np.asarray(result2).shape[1])
    res2 = _f64(np.asarray(result2, dtype=np.float64).ravel(order="F")) if C else None
    xt = np.asarray(x_test, dtype=np.float64) if C else np.zeros((0, 0))
    p = xt.shape[1] if C else 0
    xtf = _f64(xt.ravel(order="F")) if C else None
    S = int(samplesize)
    out = dict(SamplePar=np.zeros(S * P), param_quant=np.zeros(3 * P), index=np.zeros(S, dtype=np.int32))
    o = Summary()
    o.sample_par, o.param_quant, o.index = dptr(out["SamplePar"]), dptr(out["param_quant"]), iptr(out["index"])
    if C:
        out.update(Samplew=np.zeros(S * C), w_quant=np.zeros(3 * C), p_quant=np.zeros(3 * C))
        o.sample_w, o.w_quant, o.p_quant = dptr(out["Samplew"]), dptr(out["w_quant"]), dptr(out["p_quant"])
        if p_sample:
            out["p_sample"] = np.zeros(S * C)
            o.p_sample = dptr(out["p_sample"])
    check(lib.mk_posterior_summary_ex(dptr(res), P, dptr(res2), C, dptr(xtf), p, S, int(seed) & 0xFFFFFFFFFFFFFFFF,
                                      iptr(idx_in) if idx_in is not None else None, LINKS[link], o, int(device)))
    shapes = dict(SamplePar=(S, P), param_quant=(3, P), Samplew=(S, C), w_quant=(3, C), p_quant=(3, C),
                  p_sample=(S, C))
    for k, shp in shapes.items():
        if k in out:
            out[k] = out[k].reshape(shp, order="F")
    out["index"] = out["index"].astype(np.int64)
    return out
