"""The whole node in one call: mk_meta_fit (include/mk.h) -- MK.R:100-133 without a cluster.

The K subsets are cut into len(devices) balanced contiguous blocks, one session per device on
its own host thread inside libmk, every chain keyed by its global subset index (so equal to the
one-device chain).  The chains advance one amcmc batch at a time on every device; between
batches libmk calls ``progress(iterations, n_samples)`` on this thread (spBayes's n.report lines;
return True to stop: MkError with code MK_E_INTERRUPT, every device freed).  The combine runs
device to device: an all-to-all of column blocks (RCCL over xGMI for distinct devices; device
copies when a device is listed more than once), the sequential mean (MK.R:123-133, bit-identical
to one device) or the Weiszfeld median per column on each block's owner.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import Combined, Outputs, check
from .session import PackedProblem

N_LEVELS = _lib.N_LEVELS


def meta_fit_node(subsets, cfg, coords_test=None, devices=(0,), subset_base=0, method="mean", per_subset=True,
                  samples=False, w_samples=False, w_pred_samples=False, acceptance=False, w_predict_sum=False,
                  progress=None, record_w=False, max_iter=100, tol=1e-12):
    """Fit all subsets over `devices` and combine.  Returns a dict with 'result' (200 x P, MK.R:127),
    'result2' (200 x q n_test, MK.R:133; None without test sites), 'exchange' ('rccl' / 'copy'),
    'comm_ranks' (the ranks the exchange spans: RCCL's own ncclCommCount, or the blocks for copies),
    and per subset (lists, as Session.outputs lays them out) 'parameters' / 'w_predict' when
    per_subset, plus the optional 'samples', 'w_samples', 'w_pred_samples', 'acceptance',
    'w_predict_sum' (the sequential sum of all K w.predict grids)."""
    lib = _lib.load()
    if method not in ("mean", "median"):
        raise ValueError(f"error: unknown combine method '{method}'")
    pp = PackedProblem(subsets, cfg, coords_test, subset_base)
    c, keep = cfg.to_c(device=0, record_w=record_w or w_samples)
    devs = np.ascontiguousarray(devices, dtype=np.int32)
    K, P, q, n_test = pp.S, cfg.P, cfg.q, pp.n_test
    C = q * n_test
    res = {}
    o = Outputs()
    if per_subset:
        res["parameters"] = np.zeros((K, P, N_LEVELS))
        o.parameters = _lib.dptr(res["parameters"])
        if n_test:
            res["w_predict"] = np.zeros((K, C, N_LEVELS))
            o.w_predict = _lib.dptr(res["w_predict"])
    if samples:
        res["samples"] = np.zeros((K, P, cfg.n_samples))
        o.samples = _lib.dptr(res["samples"])
    if w_samples:
        res["_w"] = np.zeros(int(pp.n_part.sum()) * q * cfg.n_samples)
        o.w_samples = _lib.dptr(res["_w"])
    if w_pred_samples and n_test:
        res["w_pred_samples"] = np.zeros((K, cfg.kept, C))
        o.w_pred_samples = _lib.dptr(res["w_pred_samples"])
    if acceptance:
        res["acceptance"] = np.zeros((K, cfg.p + cfg.n_theta + 1, cfg.n_batch))
        o.acceptance = _lib.dptr(res["acceptance"])
    if w_predict_sum and n_test:
        res["w_predict_sum"] = np.zeros((C, N_LEVELS))
        o.w_predict_sum = _lib.dptr(res["w_predict_sum"])
    cb = Combined()
    result = np.zeros((P, N_LEVELS))
    cb.result = _lib.dptr(result)
    result2 = np.zeros((C, N_LEVELS)) if n_test else None
    cb.result2 = _lib.dptr(result2) if n_test else None
    cb.method = _lib.MK_COMBINE_MEDIAN if method == "median" else _lib.MK_COMBINE_MEAN
    cb.max_iter, cb.tol = int(max_iter), float(tol)

    def _cb(user, it, n):
        try:
            return 1 if (progress is not None and progress(int(it), int(n))) else 0
        except Exception:       # an exception in the callback stops the fit as an interrupt
            return 1

    fn = _lib.PROGRESS_FN(_cb)
    check(lib.mk_meta_fit(ctypes.byref(pp.c), ctypes.byref(c), devs.ctypes.data_as(_lib._ip), len(devs), fn, None,
                          ctypes.byref(o), ctypes.byref(cb)))
    del keep
    out = {"result": result.T.copy(), "result2": None if result2 is None else result2.T.copy(),
           "exchange": "rccl" if cb.exchange else "copy", "comm_ranks": int(cb.comm_ranks)}
    if "parameters" in res:
        out["parameters"] = [res["parameters"][i].T.copy() for i in range(K)]
    if "w_predict" in res:
        out["w_predict"] = [res["w_predict"][i].T.copy() for i in range(K)]
    if "samples" in res:
        out["samples"] = [res["samples"][i].T.copy() for i in range(K)]
    if "_w" in res:
        flat, off, ws = res["_w"], 0, []
        for ns in pp.n_part:
            N = int(ns) * q
            ws.append(flat[off:off + N * cfg.n_samples].reshape(cfg.n_samples, N).T.copy())
            off += N * cfg.n_samples
        out["w_samples"] = ws
    if "w_pred_samples" in res:
        out["w_pred_samples"] = [res["w_pred_samples"][i].T.copy() for i in range(K)]
    if "acceptance" in res:
        out["acceptance"] = [res["acceptance"][i].T.copy() for i in range(K)]
    if "w_predict_sum" in res:
        out["w_predict_sum"] = res["w_predict_sum"].T.copy()
    return out
