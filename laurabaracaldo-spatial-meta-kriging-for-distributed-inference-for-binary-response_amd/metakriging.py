"""Meta-kriging workflow around the device path (MetaKriging_BinaryResponse.R).

  partition            MK.R:15-41   random split into n.core subsets (last takes the remainder);
                                    method="R" replays R's own sample()/setdiff stream
  partitioned_spMvGLM  MK.R:46-96   one subset: glm start values -> spMvGLM -> spPredict -> quantiles
  meta_fit             MK.R:100-114 every subset of a shard at once on one GPU (replaces foreach %dopar%)
  combine              MK.R:119-133 mean of the subsets' 200-quantile grids (device kernel)
  posterior_summary    MK.R:136-165 interpolate to the 996-level grid, resample, p(y=1), summaries
"""
import numpy as np

from ._lib import _ip, check, load
from .glm import glm_binomial
from .post import combine_median
from .post import posterior_summary as _post_summary
from .session import SamplerConfig, Session, combine

PROBS200 = None


def r_seq(frm, to, by):
    n = int((to - frm) / by + 1e-10)
    x = frm + np.arange(n + 1, dtype=np.float64) * by
    return np.minimum(x, to)


PROBS200 = r_seq(0.005, 1.0, 0.005)     # MK.R:88
XOUT996 = r_seq(0.005, 1.0, 0.001)      # MK.R:140


def partition(n, n_core, seed=20250114, method="permutation"):
    """MK.R:15-41: n.part = c(rep(floor(n/K), K-1), remainder); random indices without replacement.

    Returns (n_part, index_part) with 0-based index arrays.
    method="R": the index sets R itself draws after `set.seed(seed)` (R >= 3.6 defaults:
    Mersenne-Twister + rejection sampling), via libmk's mk_partition_r -- the reference's
    sample()/setdiff loop (MK.R:29-41), in R's draw order.
    method="permutation": a seeded NumPy permutation split (same distribution, not R's stream)."""
    if method == "R":
        lib = load()
        n_part = np.empty(n_core, dtype=np.int32)
        idx = np.empty(n, dtype=np.int32)
        check(lib.mk_partition_r(int(n), int(n_core), int(seed),
                                 n_part.ctypes.data_as(_ip), idx.ctypes.data_as(_ip)))
        offs = np.concatenate([[0], np.cumsum(n_part)])
        return n_part, [idx[offs[i]:offs[i + 1]].astype(np.int64) - 1 for i in range(n_core)]
    if method != "permutation":
        raise ValueError(f"error: unknown partition method '{method}'")
    per = n // n_core
    n_part = [per] * (n_core - 1) + [n - per * (n_core - 1)]
    perm = np.random.default_rng(seed).permutation(n)
    idx, off = [], 0
    for m in n_part:
        idx.append(perm[off:off + m])
        off += m
    return np.array(n_part, dtype=np.int32), idx


def subset_data(y, x, weight, coords, q, index):
    """Y*.part / X*.part / coords.part for one subset (MK.R:33-39), stacked location-major."""
    rows = (np.asarray(index)[:, None] * q + np.arange(q)[None, :]).reshape(-1)
    w = np.broadcast_to(np.asarray(weight, float), (len(y),))
    return dict(coords=np.asarray(coords, float)[index], y=np.asarray(y, float)[rows],
                weights=np.ascontiguousarray(w[rows]), x=np.asarray(x, float)[rows])


def default_config(q, p, beta_starting, beta_tuning, cov_model="exponential", n_batch=100, batch_length=50,
                   seed=20250114, **kw):
    """The worker's literal settings (MK.R:56-64, 83, 85)."""
    return SamplerConfig(q, p, beta_starting, beta_tuning, cov_model=cov_model, n_batch=n_batch,
                         batch_length=batch_length, accept_rate=0.43, seed=seed, **kw)


def start_values(y, x, weight, q, device=0, link="logit"):
    """MK.R:53-55 on the full data, once, on device: beta.starting and t(chol(vcov))."""
    n_tot = len(y)
    wt = np.broadcast_to(np.asarray(weight, float), (n_tot,))
    coef, vcov, bt = glm_binomial(y, x, wt, device=device, link=link)
    return coef, bt


def r_sample_replace(n, size, seed):
    """sample.int(n, size, replace=TRUE) as R draws it right after set.seed(seed) (1-based),
    e.g. MK.R:141's sampleparIndex with n = length(Xout) = 996."""
    lib = load()
    out = np.empty(int(size), dtype=np.int32)
    check(lib.mk_r_sample_replace(int(seed), int(n), int(size), out.ctypes.data_as(_ip)))
    return out


def meta_fit(y, x, weight, coords, q, index_part, coords_test=None, cfg=None, subset_base=0, device=0,
             cov_model="exponential", n_batch=100, batch_length=50, seed=20250114):
    """All subsets of one shard on one GPU; returns the list `obj` of MK.R:108 for those subsets:
    [{'parameters': 200 x P, 'w.predict': 200 x (q n_test)}, ...]."""
    p = np.asarray(x).shape[1]
    if cfg is None:
        beta0, bt = start_values(y, x, weight, q)
        cfg = default_config(q, p, beta0, bt, cov_model=cov_model, n_batch=n_batch, batch_length=batch_length,
                             seed=seed)
    subsets = [subset_data(y, x, weight, coords, q, idx) for idx in index_part]
    with Session(subsets, cfg, coords_test=coords_test, subset_base=subset_base, device=device) as ses:
        ses.run(cfg.n_samples)
        out = ses.outputs()
    res = []
    for i in range(len(subsets)):
        d = {"parameters": out["parameters"][i]}
        if "w_predict" in out:
            d["w.predict"] = out["w_predict"][i]
        res.append(d)
    return res


def partitioned_spMvGLM(i, y, x, weight, n, q, n_part, coords_test, x_test, index_part, coords,
                        cov_model="exponential", n_batch=100, batch_length=50, seed=20250114, device=0):
    """MK.R:46-96 for subset i (1-based, as the reference): list(parameters, w.predict)."""
    return meta_fit(y, x, weight, coords, q, [index_part[i - 1]], coords_test=coords_test, subset_base=i - 1,
                    device=device, cov_model=cov_model, n_batch=n_batch, batch_length=batch_length, seed=seed)[0]


def combine_results(obj, device=0, method="mean"):
    """MK.R:123-133: result (200 x P) and result2 (200 x q n_test).  method="median" is the
    Weiszfeld geometric-median extension (the reference averages)."""
    if method == "mean":
        comb = lambda grids: combine(grids, device=device)             # noqa: E731
    elif method == "median":
        comb = lambda grids: combine_median(grids, device=device)[0]   # noqa: E731
    else:
        raise ValueError(f"error: unknown combine method '{method}'")
    result = comb([o["parameters"] for o in obj])
    result2 = comb([o["w.predict"] for o in obj]) if "w.predict" in obj[0] else None
    return result, result2


def posterior_summary(result, result2, x_test, q=None, samplesize=1000, seed=20250114, device=0, rng="philox",
                      index=None, link="logit"):
    """MK.R:136-165 on device: interpolate both combined grids to Xout (996 levels), one shared
    resample index vector (comonotone draws, MK.R:141), p(y=1) = logistic(x.test B + w) and the
    median / 2.5% / 97.5% summaries (post.posterior_summary).  rng="R": sampleparIndex is R's
    sample(seq(1, length(Xout), 1), samplesize, replace=TRUE) right after set.seed(seed);
    index: a 1-based index vector drawn by the caller (R's own stream)."""
    return _post_summary(result, result2, x_test, samplesize=samplesize, seed=seed, device=device, rng=rng,
                         index=index, link=link)


def reference_flow(d, K, q, cov_model="exponential", n_batch=100, batch_length=50, seed=20250114, devices=(0,),
                   method="mean", predict_tile=0, partition_method="R", samplesize=1000, progress=None):
    """The reference script end to end in one process over the GPUs in `devices` (mk_meta_fit: the
    subsets sharded over them in-library, the combine device to device):

      partition                 MK.R:15-41    mk_partition_r (R's own index sets after set.seed)
      glm start values          MK.R:53-55    device IRLS on the full data, once
      foreach %dopar% worker    MK.R:100-114  every subset's spMvGLM + spPredict + 200-level grids
      combine                   MK.R:119-133  sequential mean (or Weiszfeld median), per test-site
                                              tile when predict_tile > 0 (configs[4])
      resample, p(y=1), quant.  MK.R:136-165  posterior_summary

    d: synthetic.generate output.  progress(iterations, n_samples) is called between amcmc batches
    (return True to stop).  Returns (phases, result, result2, summary, cfg) -- phases in seconds of
    wall clock: set-up (partition, glm, subset slicing), the chains (to the last batch boundary),
    quantiles + combine, post-processing, and the whole."""
    import time
    from .node import meta_fit_node
    t = {}
    n = len(d["coords"])
    t0 = time.perf_counter()
    n_part, index_part = partition(n, K, seed=seed, method=partition_method)                 # MK.R:15-41
    beta0, bt = start_values(d["y"], d["x"], 1.0, q, device=int(devices[0]))                 # MK.R:53-55
    p = d["x"].shape[1]
    cfg = SamplerConfig(q, p, beta0, bt, cov_model=cov_model, n_batch=n_batch, batch_length=batch_length, seed=seed,
                        predict_tile=predict_tile)
    subs = [subset_data(d["y"], d["x"], 1.0, d["coords"], q, index_part[i]) for i in range(K)]
    t["setup_s"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    stamp = {}

    def _progress(it, n_samples):
        if it >= n_samples:
            stamp["chains"] = time.perf_counter()
        return bool(progress(it, n_samples)) if progress is not None else False

    fit = meta_fit_node(subs, cfg, coords_test=d["coords_test"], devices=devices, method=method, per_subset=False,
                        progress=_progress)                                                  # MK.R:100-133
    t3 = time.perf_counter()
    t["chains_s"] = stamp.get("chains", t3) - t1
    t["quantiles_combine_s"] = t3 - stamp.get("chains", t3)
    t2 = time.perf_counter()
    summ = posterior_summary(fit["result"], fit["result2"], d["x_test"], samplesize=samplesize, seed=seed,
                             device=int(devices[0]))                                         # MK.R:136-165
    t["post_s"] = time.perf_counter() - t2
    t["end_to_end_s"] = time.perf_counter() - t0
    t["exchange"] = fit["exchange"]          # the combine's all-to-all: "rccl" (distinct GPUs) or "copy"
    t["comm_ranks"] = fit["comm_ranks"]      # ranks RCCL's communicators hold (copies: device blocks)
    return t, fit["result"], fit["result2"], summ, cfg
