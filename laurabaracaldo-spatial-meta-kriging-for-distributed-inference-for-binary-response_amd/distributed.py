"""Subsets sharded over ranks (one process per GPU, torch.distributed over RCCL/xGMI).

Subsets are independent during the fit and kriging (MK.R:108: foreach over subsets),
so every rank runs its contiguous block of subsets with no traffic.  The one exchange
is the combine (MK.R:119-133), column-sharded: an all-to-all hands every rank all K
subsets' grids for its block of columns, the rank combines them in global subset order
(the reference's sequential mean -- bit-identical to one GPU -- or the Weiszfeld median,
SURVEY.md 8f row 2) and the combined blocks are all-gathered.  With an RCCL group the
exchanged blocks stay in HBM: the per-column combine runs on the receive buffers through
mk_combine_device / mk_combine_median_device and only the final grid reaches the host.
allgather_grids keeps the plain all-gather of whole grids for small problems.
"""
import numpy as np


def shard_range(K, world, rank):
    """Contiguous balanced block of subsets for `rank` -> [lo, hi): sizes differ by at most one
    (250 over 8 ranks: 31 or 32), so no rank is empty while K >= world."""
    lo = (rank * K) // world
    return lo, ((rank + 1) * K) // world


def shard_capacity(K, world):
    """Largest shard (the exchange buffers' subset dimension)."""
    return max(hi - lo for lo, hi in (shard_range(K, world, r) for r in range(world)))


def allgather_grids(local, K, dist, device=None):
    """local: (n_local, *G) grids of this rank's subsets; returns (K, *G) in global order."""
    import torch
    world = dist.get_world_size()
    per = shard_capacity(K, world)
    local = np.asarray(local, dtype=np.float64)
    shape = local.shape[1:]
    buf = np.zeros((per,) + shape)
    buf[:local.shape[0]] = local
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    parts = []
    for r in range(world):
        lo, hi = shard_range(K, world, r)
        parts.append(outs[r][:hi - lo])
    return torch.cat(parts, dim=0).cpu().numpy()


def col_blocks(C, world):
    """Contiguous column blocks of ceil(C/world) columns -> [(a, b)] per rank."""
    per = (C + world - 1) // world
    return [(min(C, r * per), min(C, (r + 1) * per)) for r in range(world)]


def _exchange(send, recv, dist):
    """recv[src] <- what rank src put in its send[me]: point-to-point pairs (RCCL and gloo)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    recv[rank].copy_(send[rank])
    ops = []
    for r in range(world):
        if r != rank:
            ops.append(dist.P2POp(dist.isend, send[r], r))
            ops.append(dist.P2POp(dist.irecv, recv[r], r))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def _device_combine(grids, method, gpu):
    """grids: (K, L, c) float64 CUDA tensor, global subset order -> (L, c) CUDA tensor, combined
    in HBM by libmk on torch's current stream (mean / sum: k_combine's sequential order;
    median: k_weiszfeld per column)."""
    import torch
    from ._lib import check, load
    lib = load()
    K, L, c = grids.shape
    stream = torch.cuda.current_stream(grids.device).cuda_stream
    if method in ("mean", "sum"):
        g = grids.contiguous()
        out = torch.empty((L, c), dtype=torch.float64, device=grids.device)
        check(lib.mk_combine_device(g.data_ptr(), K, L * c, out.data_ptr(), 1 if method == "mean" else 0, gpu, stream))
        return out
    if method == "median":
        g = grids.transpose(1, 2).contiguous()                  # per grid: column c = L contiguous levels
        out = torch.empty((c, L), dtype=torch.float64, device=grids.device)
        it = torch.empty((c,), dtype=torch.int32, device=grids.device)
        check(lib.mk_combine_median_device(g.data_ptr(), K, L, c, 100, 1e-12, out.data_ptr(), it.data_ptr(), gpu,
                                           stream))
        return out.t()
    raise ValueError(f"error: unknown combine method '{method}'")


def combine_sharded(local, K, dist, method="mean", device=None, gpu=0, combine_fn=None):
    """Column-sharded combine of K subset grids held by contiguous subset blocks of the ranks.

    local: (n_local, L, C) grids of this rank's subsets (shard_range order) -- a NumPy array, or a
    torch tensor already in HBM (e.g. Session.grids_device's (n_local, C, L) buffer transposed:
    then nothing of the exchange touches the host until the combined grid).  One all-to-all
    exchange gives rank r every subset's grid for its column block; it combines them in global
    subset order -- "mean" is MK.R:123-133 in the reference's summation order (so the result is
    bit-identical to one GPU), "sum" the same without the 1/K, "median" the Weiszfeld extension
    (per column, so also independent of the sharding) -- and the combined blocks are
    all-gathered.  Per-rank memory is K x L x C / world, where a full all-gather needs
    K x L x C (400 GB at cfg5's 1M sites).

    device: a CUDA device -> the exchange runs over RCCL and the combine runs in HBM on the
    receive buffers (mk_combine_device); None -> CPU tensors (gloo) and the host entry points.
    combine_fn(list of L x c grids) -> L x c overrides the combine (CPU tests)."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cpu") if device is None else torch.device(device)
    on_gpu = dev.type == "cuda"
    if isinstance(local, torch.Tensor):
        # device-resident grids (Session.grids_device): the send buffer is packed in HBM
        local_t = local.to(dev)
    else:
        local_t = torch.from_numpy(np.ascontiguousarray(np.asarray(local, dtype=np.float64)))
    L, C = int(local_t.shape[1]), int(local_t.shape[2])
    per_k = shard_capacity(K, world)
    blocks = col_blocks(C, world)
    cmax = max(1, max(b - a for a, b in blocks))
    send = torch.zeros((world, per_k, L, cmax), dtype=torch.float64, device=local_t.device)
    for r, (a, b) in enumerate(blocks):
        if b > a and local_t.shape[0]:
            send[r, :local_t.shape[0], :, :b - a] = local_t[:, :, a:b]
    send = send.to(dev)
    recv = torch.empty_like(send)
    _exchange(send, recv, dist)
    a, b = blocks[rank]
    counts = [shard_range(K, world, src)[1] - shard_range(K, world, src)[0] for src in range(world)]
    if on_gpu and combine_fn is None:
        mine = torch.cat([recv[src, :counts[src]] for src in range(world)], dim=0)     # (K, L, cmax) in HBM
        buf = _device_combine(mine, method, gpu) if b > a else torch.zeros((L, cmax), dtype=torch.float64, device=dev)
        buf = buf.contiguous()
    else:
        mine = recv.cpu().numpy()
        grids = []
        for src in range(world):                       # global subset order
            grids += [mine[src, i, :, :b - a] for i in range(counts[src])]
        if combine_fn is None:
            from .post import combine_median
            from .session import combine
            if method == "mean":
                combine_fn = lambda g: combine(g, device=gpu)                 # noqa: E731
            elif method == "sum":
                combine_fn = lambda g: combine(g, device=gpu, mean=False)     # noqa: E731
            elif method == "median":
                combine_fn = lambda g: combine_median(g, device=gpu)[0]       # noqa: E731
            else:
                raise ValueError(f"error: unknown combine method '{method}'")
        buf = torch.zeros((L, cmax), dtype=torch.float64)
        if b > a:
            buf[:, :b - a] = torch.from_numpy(np.ascontiguousarray(combine_fn(grids)))
        buf = buf.to(dev)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return np.concatenate([outs[r].cpu().numpy()[:, :blocks[r][1] - blocks[r][0]] for r in range(world)], axis=1)


def combine_partial_sums(partial, K, dist, device=None, gpu=0, combine_fn=None):
    """result2 of MK.R:129-133 from per-rank partial sums (tiled kriging, cfg5's 1M sites, where
    per-subset grids never reach the host): rank r holds S_r = its subsets' grids summed in subset
    order (mk_outputs.w_predict_sum); result2 = (S_0 + S_1 + ...) / K, the S_r added in rank
    order on each column block's owner.  Deterministic for a given world size; equal to one
    GPU's sequential sum up to the re-association of the K terms into rank blocks."""
    world = dist.get_world_size()
    p = np.asarray(partial, dtype=np.float64)[None]
    total = combine_sharded(p, world, dist, method="sum", device=device, gpu=gpu, combine_fn=combine_fn)
    return total / K


def combine_tiles(tile_grids, n_test, tile, q, K, dist, method="mean", device=None, gpu=0, combine_fn=None):
    """result2 of MK.R:129-133 -- or its Weiszfeld median -- at configs[4] scale, one test-site tile
    at a time: tile_grids(t0) returns this rank's subsets' (n_local, 200, q*Tc) grids of sites
    [t0, t0 + Tc) (Session.tile_grids: that tile's kriging replay only), and each tile goes through
    the column-sharded exchange + combine (combine_sharded), so the combine is the sequential one
    -- bit-identical to one GPU -- or the per-column median, and a rank holds K x 200 x q*tile/world
    exchanged doubles, not K x 200 x q*n_test (400 GB at 1M sites).  Every rank calls it with the
    same tiling (an empty shard passes (0, 200, q*Tc) grids)."""
    out = np.zeros((200, q * n_test))
    for t0 in range(0, n_test, tile):
        tc = min(tile, n_test - t0)
        local = np.asarray(tile_grids(t0), dtype=np.float64).reshape(-1, 200, q * tc)
        out[:, t0 * q:(t0 + tc) * q] = combine_sharded(local, K, dist, method=method, device=device, gpu=gpu,
                                                       combine_fn=combine_fn)
    return out


def meta_fit_distributed(y, x, weight, coords, q, index_part, coords_test, cfg, dist, device=0, method="mean"):
    """Fit this rank's shard of subsets on its GPU, then the one exchange: the column-sharded
    combine (MK.R:119-133; method="median" for the Weiszfeld extension).

    Returns (obj_local, result, result2): the local `obj` entries (MK.R:108) and the
    combined grids (MK.R:127, MK.R:133), identical on every rank.  A rank whose shard is
    empty (K < world) fits nothing and still takes part in the exchange."""
    from .metakriging import meta_fit
    import torch
    K = len(index_part)
    lo, hi = shard_range(K, dist.get_world_size(), dist.get_rank())
    obj = []
    if hi > lo:
        obj = meta_fit(y, x, weight, coords, q, index_part[lo:hi], coords_test=coords_test, cfg=cfg, subset_base=lo,
                       device=device)
    dev = torch.device("cuda", device) if dist.get_backend() == "nccl" else None
    P = cfg.P
    par = np.stack([o["parameters"] for o in obj]) if obj else np.zeros((0, 200, P))
    result = combine_sharded(par, K, dist, method=method, device=dev, gpu=device)
    result2 = None
    if coords_test is not None:
        C = q * np.asarray(coords_test).shape[0]
        wp = np.stack([o["w.predict"] for o in obj]) if obj else np.zeros((0, 200, C))
        result2 = combine_sharded(wp, K, dist, method=method, device=dev, gpu=device)
    return obj, result, result2
