"""Subsets sharded over ranks (one process per GPU, torch.distributed over RCCL/xGMI).

Subsets are independent during the fit and kriging (MK.R:108: foreach over subsets),
so every rank runs its contiguous block of subsets with no traffic.  The one exchange
is the combine (MK.R:119-133): an all-gather of the per-subset 200-level grids in
global subset order, after which every rank sums them in the reference's sequential
order -- the multi-GPU result is bit-identical to the single-GPU one.  The same
all-gathered grids feed the Weiszfeld / barycenter extensions.
"""
import numpy as np


def shard_range(K, world, rank):
    """Contiguous block of ceil(K/world) subsets for `rank` -> [lo, hi)."""
    per = (K + world - 1) // world
    lo = min(K, rank * per)
    return lo, min(K, lo + per)


def allgather_grids(local, K, dist, device=None):
    """local: (n_local, *G) grids of this rank's subsets; returns (K, *G) in global order."""
    import torch
    world = dist.get_world_size()
    per = (K + world - 1) // world
    local = np.asarray(local, dtype=np.float64)
    shape = local.shape[1:]
    buf = np.zeros((per,) + shape)
    buf[:local.shape[0]] = local
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    full = torch.cat(outs, dim=0)[:K]
    return full.cpu().numpy()


def meta_fit_distributed(y, x, weight, coords, q, index_part, coords_test, cfg, dist, device=0):
    """Fit this rank's shard of subsets on its GPU, all-gather the grids, combine (on device).

    Returns (obj_local, result, result2): the local `obj` entries (MK.R:108) and the
    combined grids (MK.R:127, MK.R:133), identical on every rank."""
    from .metakriging import meta_fit
    from .session import combine
    import torch
    K = len(index_part)
    lo, hi = shard_range(K, dist.get_world_size(), dist.get_rank())
    obj = meta_fit(y, x, weight, coords, q, index_part[lo:hi], coords_test=coords_test, cfg=cfg, subset_base=lo,
                   device=device)
    dev = torch.device("cuda", device) if dist.get_backend() == "nccl" else None
    P = cfg.P
    par = np.stack([o["parameters"] for o in obj]) if obj else np.zeros((0, 200, P))
    allpar = allgather_grids(par, K, dist, dev)
    result = combine(list(allpar), device=device)
    result2 = None
    if coords_test is not None:
        C = q * np.asarray(coords_test).shape[0]
        wp = np.stack([o["w.predict"] for o in obj]) if obj else np.zeros((0, 200, C))
        allw = allgather_grids(wp, K, dist, dev)
        result2 = combine(list(allw), device=device)
    return obj, result, result2
