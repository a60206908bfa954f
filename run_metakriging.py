#!/usr/bin/env python3
"""MetaKriging_BinaryResponse.R end to end on the MI355X path, one process per GPU.

The reference script's flow with its drop-ins (MK.R line numbers):
  data (the driver the reference lacks)   -> synthetic.generate
  partition                      MK.R:15-41             -> metakriging.partition
  glm start values               MK.R:53-55             -> glm_binomial (device, once)
  foreach %dopar% worker         MK.R:100-114           -> Session: every subset of the shard at once
     spMvGLM + spPredict + quantiles  MK.R:80-89
  combine                        MK.R:119-133           -> combine / combine_median / column-sharded (N > 1)
  resample + p(y=1) + summaries  MK.R:136-165           -> posterior_summary (device)

Prints one JSON line with the wall-clock of every phase (rank 0).  Multi-GPU:
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 run_metakriging.py ...

  python run_metakriging.py --config 3          # configs[2]: n=500k, K=250, exponential, q=1
"""
import argparse
import os

# before HIP starts: libmk's lookahead schedule runs up to five HIP streams and HIP shares
# hardware queues beyond GPU_MAX_HW_QUEUES (4 by default)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import importlib
import json
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"

# BASELINE.json configs (1-based as in SURVEY.md): n, K, cov, q, n_test, n_batch x batch_length
CONFIGS = {
    1: dict(n=2000, K=5, cov="exponential", q=1, n_test=1000, n_batch=20, batch_length=50),
    2: dict(n=50000, K=50, cov="matern", q=1, n_test=1000, n_batch=100, batch_length=50),
    3: dict(n=500000, K=250, cov="exponential", q=1, n_test=1000, n_batch=100, batch_length=50),
    4: dict(n=100000, K=50, cov="exponential", q=3, n_test=1000, n_batch=100, batch_length=50),
    5: dict(n=500000, K=250, cov="exponential", q=1, n_test=1000000, n_batch=100, batch_length=50,
            predict_tile=65536),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1, choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int)
    ap.add_argument("--subsets", type=int)
    ap.add_argument("--n-test", type=int)
    ap.add_argument("--n-batch", type=int)
    ap.add_argument("--batch-length", type=int)
    ap.add_argument("--combine", default="mean", choices=["mean", "median"])
    ap.add_argument("--predict-tile", type=int)
    ap.add_argument("--seed", type=int, default=20250114)
    ap.add_argument("--partition", default="R", choices=["R", "permutation"],
                    help="R: the subsets R draws after set.seed(seed) (mk_partition_r)")
    ap.add_argument("--devices", default=None,
                    help="one process, libmk's multi-device driver (mk_meta_fit) over these HIP devices, e.g. "
                         "0,1,2,3,4,5,6,7 (a device may repeat: several shards on one GPU, device-copy exchange)")
    a = ap.parse_args()
    c = dict(CONFIGS[a.config])
    for k_arg, k_cfg in [("n", "n"), ("subsets", "K"), ("n_test", "n_test"), ("n_batch", "n_batch"),
                         ("batch_length", "batch_length"), ("predict_tile", "predict_tile")]:
        v = getattr(a, k_arg)
        if v is not None:
            c[k_cfg] = v
    if a.devices is not None:
        return node_main(a, c)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    mk = importlib.import_module(PKG)
    dmod = importlib.import_module(PKG + ".distributed")
    t = {}
    t0 = time.perf_counter()
    q, n, K = c["q"], c["n"], c["K"]
    d = mk.synthetic.generate(n, q=q, n_test=c["n_test"], cov_model=1 if c["cov"] == "matern" else 0, seed=a.seed)
    t["data_s"] = time.perf_counter() - t0

    t1 = time.perf_counter()
    n_part, index_part = mk.partition(n, K, seed=a.seed, method=a.partition)                     # MK.R:15-41
    beta0, bt = mk.start_values(d["y"], d["x"], 1.0, q, device=local)         # MK.R:53-55
    p = d["x"].shape[1]
    cfg = mk.SamplerConfig(q, p, beta0, bt, cov_model=c["cov"], n_batch=c["n_batch"], batch_length=c["batch_length"],
                           seed=a.seed, predict_tile=c.get("predict_tile", 0))
    lo, hi = dmod.shard_range(K, world, rank)
    subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], q, index_part[i]) for i in range(lo, hi)]
    t["setup_s"] = time.perf_counter() - t1

    t2 = time.perf_counter()
    big = cfg.predict_tile > 0 and cfg.predict_tile < c["n_test"]
    C = q * c["n_test"]
    P = cfg.P
    ses = None
    if subs:
        ses = mk.Session(subs, cfg, coords_test=d["coords_test"], subset_base=lo, device=local)   # MK.R:108
        for b in range(cfg.n_batch):          # progress every n.report = 10 batches (MK.R:84)
            ses.run(cfg.batch_length)
            if rank == 0 and (b + 1) % 10 == 0:
                print(f"batch {b + 1}/{cfg.n_batch}  {time.perf_counter() - t2:.1f}s", file=sys.stderr, flush=True)
        t3 = time.perf_counter()
        # 1M sites (tiled kriging): the parameter grids now; w.predict tile by tile in the combine
        # one process: the grids to the host for the combine; N > 1: they stay in HBM (shard_grids below)
        out = ses.outputs(quantiles=True, w_predict=not big) if world == 1 else {"parameters": [], "w_predict": []}
    else:                                         # K < world: this rank has no subsets, it joins the exchange
        t3 = time.perf_counter()
        out = {"parameters": [], "w_predict": []}
    t["fit_s"] = t3 - t2
    t["predict_quantiles_s"] = time.perf_counter() - t3

    t4 = time.perf_counter()
    par = np.stack(out["parameters"]) if out["parameters"] else np.zeros((0, 200, P))
    tile = ses.predict_tile if ses is not None else cfg.predict_tile   # the tile in use (HBM may shrink it)

    def tile_grids(t0):                           # this shard's grids of one test-site tile (kriging replay)
        tc = min(tile, c["n_test"] - t0)
        return ses.tile_grids(t0) if ses is not None else np.zeros((0, 200, q * tc))

    if world > 1:
        import torch
        dev = torch.device("cuda", local)

        def shard_grids(which, ncol):   # this shard's (S, 200, ncol) grids, written by libmk into HBM
            g = torch.empty((len(subs), ncol, 200), dtype=torch.float64, device=dev)
            if ses is not None:
                ses.grids_device(which, g.data_ptr())
            return g.transpose(1, 2)

        result = dmod.combine_sharded(shard_grids(0, P), K, dist, method=a.combine, device=dev, gpu=local)   # MK.R:123-127
        if big:   # the exchange runs tile by tile: every rank must replay the same tiles
            tl = torch.tensor([tile, -tile], dtype=torch.int64, device=dev)
            dist.all_reduce(tl, op=dist.ReduceOp.MIN)
            if int(tl[0]) != -int(tl[1]):
                raise SystemExit(f"ranks took different kriging tiles ({int(tl[0])} .. {-int(tl[1])} test sites: HBM "
                                 f"limits differ); pass --predict-tile {int(tl[0])} or less")
        if not big:
            result2 = dmod.combine_sharded(shard_grids(1, C), K, dist, method=a.combine, device=dev, gpu=local)
        else:
            # tiled kriging (cfg5): per test-site tile, the column-sharded exchange + combine of that
            # tile's grids (sequential mean, or the Weiszfeld median per column)
            result2 = dmod.combine_tiles(tile_grids, c["n_test"], tile, q, K, dist, method=a.combine, device=dev,
                                         gpu=local)
    elif not big:
        obj = [{"parameters": out["parameters"][i], "w.predict": out["w_predict"][i]} for i in range(len(subs))]
        result, result2 = mk.combine_results(obj, device=local, method=a.combine)             # MK.R:123-133
    else:   # tiled kriging (cfg5), one process: every tile's K grids combined as they are replayed
        result = mk.combine_results([{"parameters": g} for g in out["parameters"]], device=local,
                                    method=a.combine)[0]
        result2 = np.zeros((200, C))
        for t0 in range(0, c["n_test"], tile):
            g = tile_grids(t0)
            result2[:, t0 * q:t0 * q + g.shape[2]] = mk.combine_results([{"parameters": x} for x in g], device=local,
                                                                        method=a.combine)[0]
            del g
            print(f"tile {t0 // tile + 1}/{(c['n_test'] + tile - 1) // tile}  {time.perf_counter() - t4:.1f}s",
                  file=sys.stderr, flush=True)
    if ses is not None:
        ses.close()
    t["combine_s"] = time.perf_counter() - t4

    t5 = time.perf_counter()
    summ = None
    if result is not None:
        summ = mk.posterior_summary(result, result2, d["x_test"], samplesize=1000, seed=a.seed, device=local)
    t["post_s"] = time.perf_counter() - t5
    t["end_to_end_s"] = time.perf_counter() - t1
    if rank == 0:
        rec = dict(config=a.config, workload=c, n_gpus=world, combine=a.combine, phases=t,
                   subset_iters_per_s=K * cfg.n_samples / (t["fit_s"]) if world == 1 else None)
        if summ is not None:
            truth = np.concatenate([d["beta_true"], [1.0] if q == 1 else [], [6.0] if q == 1 else []])
            rec["param_median"] = summ["param_quant"][0].tolist()
            rec["param_95ci"] = [summ["param_quant"][1].tolist(), summ["param_quant"][2].tolist()]
            wq = summ["w_quant"]
            rec["w_test_coverage_95"] = float(np.mean((d["w_test_true"] >= wq[1]) & (d["w_test_true"] <= wq[2])))
            rec["truth_beta_phi"] = truth.tolist()
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def node_main(a, c):
    """The script in one process over a device list (mk_meta_fit): shards, combine (mean or median,
    per test-site tile at configs[4]) and post-processing without torch or a second process."""
    mk = importlib.import_module(PKG)
    devices = [int(x) for x in a.devices.split(",")]
    t0 = time.perf_counter()
    q, n, K = c["q"], c["n"], c["K"]
    d = mk.synthetic.generate(n, q=q, n_test=c["n_test"], cov_model=1 if c["cov"] == "matern" else 0, seed=a.seed)
    data_s = time.perf_counter() - t0

    def progress(it, n_samples):
        if it % (10 * c["batch_length"]) == 0:    # n.report = 10 batches (MK.R:84)
            print(f"iterations {it}/{n_samples}  {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        return False

    ph, result, result2, summ, cfg = mk.metakriging.reference_flow(
        d, K, q, cov_model=c["cov"], n_batch=c["n_batch"], batch_length=c["batch_length"], seed=a.seed,
        devices=devices, method=a.combine, predict_tile=c.get("predict_tile", 0), partition_method=a.partition,
        progress=progress)
    ph["data_s"] = data_s
    rec = dict(config=a.config, workload=c, devices=devices, combine=a.combine, phases=ph,
               subset_iters_per_s=K * cfg.n_samples / ph["chains_s"])
    truth = np.concatenate([d["beta_true"], [1.0] if q == 1 else [], [6.0] if q == 1 else []])
    rec["param_median"] = summ["param_quant"][0].tolist()
    rec["param_95ci"] = [summ["param_quant"][1].tolist(), summ["param_quant"][2].tolist()]
    wq = summ["w_quant"]
    rec["w_test_coverage_95"] = float(np.mean((d["w_test_true"] >= wq[1]) & (d["w_test_true"] <= wq[2])))
    rec["truth_beta_phi"] = truth.tolist()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
