"""World-size-2 gloo test of the N>1 path on CPU: shard assignment covers every subset
once, the all-gather returns the grids in global subset order, and the sequential combine
of the gathered grids equals the single-process combine bit for bit."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grid(k):
    """Deterministic stand-in for subset k's 200 x C quantile grid."""
    rng = np.random.default_rng(1000 + k)
    return np.sort(rng.normal(size=(200, 5)), axis=0)


def _worker(rank, world, port, K, out_q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dmod = importlib.import_module(PKG + ".distributed")
    lo, hi = dmod.shard_range(K, world, rank)
    local = np.stack([_grid(k) for k in range(lo, hi)]) if hi > lo else np.zeros((0, 200, 5))
    full = dmod.allgather_grids(local, K, dist)
    out_q.put((rank, lo, hi, full))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("K,world", [(7, 2), (250, 2), (3, 2)])
def test_allgather_combine_matches_single_process(K, world):
    import torch.multiprocessing as mp
    from oracle.spmvglm import combine_mean
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = np.stack([_grid(k) for k in range(K)])
    covered = []
    for rank, lo, hi, full in res:
        covered += list(range(lo, hi))
        assert np.array_equal(full, ref)                       # global order on every rank
        assert np.array_equal(combine_mean(list(full)), combine_mean(list(ref)))
    assert sorted(covered) == list(range(K))


def test_shard_range_contiguous():
    dmod = importlib.import_module(PKG + ".distributed")
    for K in (1, 5, 250):
        for world in (1, 2, 3, 8):
            spans = [dmod.shard_range(K, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == K
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c


def _grid_wide(k, C):
    rng = np.random.default_rng(2000 + k)
    return np.sort(rng.normal(loc=0.3 * k, size=(200, C)), axis=0)


def _sharded_worker(rank, world, port, K, C, method, out_q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from oracle.post import weiszfeld_median
    from oracle.spmvglm import combine_mean
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dmod = importlib.import_module(PKG + ".distributed")
    lo, hi = dmod.shard_range(K, world, rank)
    local = np.stack([_grid_wide(k, C) for k in range(lo, hi)]) if hi > lo else np.zeros((0, 200, C))
    fn = combine_mean if method == "mean" else (lambda g: weiszfeld_median(np.stack(g))[0])
    full = dmod.combine_sharded(local, K, dist, method=method, combine_fn=fn)
    out_q.put((rank, full))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("K,C,world,method", [(7, 9, 2, "mean"), (5, 3, 3, "mean"), (6, 10, 2, "median"),
                                              (4, 2, 3, "median")])
def test_column_sharded_combine_matches_single_process(K, C, world, method):
    """One all-to-all + per-column combine + all-gather == the single-process combine, on every
    rank (mean: bit-identical, same summation order; median: per-column, so identical too)."""
    import torch.multiprocessing as mp
    from oracle.post import weiszfeld_median
    from oracle.spmvglm import combine_mean
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, K, C, method, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    grids = [_grid_wide(k, C) for k in range(K)]
    ref = combine_mean(grids) if method == "mean" else weiszfeld_median(np.stack(grids))[0]
    for rank, full in res:
        assert full.shape == (200, C)
        if method == "mean":
            assert np.array_equal(full, ref)
        else:
            np.testing.assert_allclose(full, ref, rtol=1e-14, atol=1e-14)


def test_col_blocks_cover_columns():
    dmod = importlib.import_module(PKG + ".distributed")
    for C in (1, 2, 7, 1000):
        for world in (1, 2, 3, 8):
            b = dmod.col_blocks(C, world)
            assert b[0][0] == 0 and b[-1][1] == C and all(x[1] == y[0] for x, y in zip(b, b[1:]))


def test_shard_range_balanced():
    """Balanced contiguous shards (ADVICE: ceil blocks left ranks empty, e.g. K=5 on 8 GPUs):
    sizes differ by at most one and no rank is empty while K >= world."""
    dmod = importlib.import_module(PKG + ".distributed")
    for K in (1, 5, 8, 20, 250):
        for world in (1, 2, 3, 8):
            sizes = [hi - lo for lo, hi in (dmod.shard_range(K, world, r) for r in range(world))]
            assert sum(sizes) == K and max(sizes) - min(sizes) <= 1
            if K >= world:
                assert min(sizes) >= 1
    assert [dmod.shard_range(250, 8, r) for r in (0, 7)] == [(0, 31), (218, 250)]


def _seq_sum(grids):
    acc = np.array(grids[0], copy=True)
    for g in grids[1:]:
        acc = acc + g
    return acc


def _partial_worker(rank, world, port, K, C, out_q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dmod = importlib.import_module(PKG + ".distributed")
    lo, hi = dmod.shard_range(K, world, rank)
    # this rank's term of the combine: its subsets' grids summed in subset order (w_predict_sum)
    part = _seq_sum([_grid_wide(k, C) for k in range(lo, hi)]) if hi > lo else np.zeros((200, C))
    full = dmod.combine_partial_sums(part, K, dist, combine_fn=_seq_sum)
    # an empty shard (K < world) still joins the column-sharded exchange
    k_small = world - 1
    lo2, hi2 = dmod.shard_range(k_small, world, rank)
    local = np.stack([_grid_wide(k, C) for k in range(lo2, hi2)]) if hi2 > lo2 else np.zeros((0, 200, C))
    from oracle.spmvglm import combine_mean
    small = dmod.combine_sharded(local, k_small, dist, combine_fn=combine_mean)
    out_q.put((rank, full, small))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("K,C,world", [(7, 9, 2), (10, 4, 3)])
def test_partial_sums_and_empty_shards(K, C, world):
    """cfg5 path (ADVICE high): per-rank partial sums of w.predict combined in rank order,
    result2 = (S_0 + S_1 + ...) / K on every rank; and a K < world exchange with an empty rank."""
    import torch.multiprocessing as mp
    from oracle.spmvglm import combine_mean
    dmod = importlib.import_module(PKG + ".distributed")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_partial_worker, args=(r, world, port, K, C, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    terms = []
    for r in range(world):
        lo, hi = dmod.shard_range(K, world, r)
        terms.append(_seq_sum([_grid_wide(k, C) for k in range(lo, hi)]))
    ref = _seq_sum(terms) / K
    one_gpu = combine_mean([_grid_wide(k, C) for k in range(K)])
    small_ref = combine_mean([_grid_wide(k, C) for k in range(world - 1)])
    for rank, full, small in res:
        assert np.array_equal(full, ref)
        np.testing.assert_allclose(full, one_gpu, rtol=1e-13, atol=1e-13)   # re-association only
        assert np.array_equal(small, small_ref)


def _tile_worker(rank, world, port, K, n_test, tile, method, out_q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from oracle.post import weiszfeld_median
    from oracle.spmvglm import combine_mean
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dmod = importlib.import_module(PKG + ".distributed")
    lo, hi = dmod.shard_range(K, world, rank)
    calls = []

    def tile_grids(t0):             # this rank's subsets' grids of sites [t0, t0 + Tc)
        calls.append(t0)
        tc = min(tile, n_test - t0)
        return np.stack([_grid_wide(k, n_test)[:, t0:t0 + tc] for k in range(lo, hi)]) if hi > lo \
            else np.zeros((0, 200, tc))

    fn = combine_mean if method == "mean" else (lambda g: weiszfeld_median(np.stack(g))[0])
    full = dmod.combine_tiles(tile_grids, n_test, tile, 1, K, dist, method=method, combine_fn=fn)
    out_q.put((rank, full, calls))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("K,n_test,tile,world,method", [(5, 11, 4, 2, "median"), (7, 9, 9, 2, "mean"),
                                                        (1, 6, 4, 2, "median")])
def test_tiled_combine_matches_whole_grid_combine(K, n_test, tile, world, method):
    """configs[4]'s combine tile by tile: per test-site tile a column-sharded
    exchange + combine of the subsets' grids of that tile; the assembled result equals the oracle's
    combine of the whole grids (mean: bit for bit; Weiszfeld median (oracle/post.py): per column)."""
    import torch.multiprocessing as mp
    from oracle.post import weiszfeld_median
    from oracle.spmvglm import combine_mean
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tile_worker, args=(r, world, port, K, n_test, tile, method, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    grids = [_grid_wide(k, n_test) for k in range(K)]
    ref = combine_mean(grids) if method == "mean" else weiszfeld_median(np.stack(grids))[0]
    for rank, full, calls in res:
        assert calls == list(range(0, n_test, tile))
        if method == "mean":
            assert np.array_equal(full, ref)
        else:
            np.testing.assert_allclose(full, ref, rtol=1e-14, atol=1e-14)
