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
