#!/usr/bin/env python3
"""configs[4]'s per-GPU share measured end to end on one GPU: the kriging of
1,000,000 held-out sites (MK.R:87-89) from the busiest rank's block of an 8-GPU run of K = 250
(rank 7: subsets [218, 250), 32 subsets of n_s = 2,000; global indices, so its chains are the node
run's chains), with the reference's sampler as written -- 100 x 50 amcmc iterations, burn.in 3,750,
1,251 kept states (MK.R:57-59, 83, 85) -- through the tiled replay (predict_tile = 65,536): per test
tile, the replay of all 1,251 kept states (X = W P^T re-run where phi changed), the 200-level grids
of every subset and their sequential mean over the shard (the shard's share of the combine, MK.R:123-133).
Since round 6 the replay interpolates the kriging variance in phi (MK_KRIG_CHEB, mk_api.hip
predict_tile_cheb); MK_KRIG_CHEB=0 runs the exact replay.

Wall clock by phase.  One gpurun command may run at most 20 minutes, so the 16 test tiles can be
split over calls (--tiles a:b); the fit is deterministic (Philox streams keyed by the global subset
index), so every call replays the same chain, and the per-tile times add up.  Progress goes to stderr
once per tile.

    python tools/cfg5_share.py --tiles 0:8 > share_a.json     # then --tiles 8:16
"""
import argparse
import importlib
import json
import os
import sys
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000)
    ap.add_argument("--K", type=int, default=250)
    ap.add_argument("--gpus", type=int, default=8, help="node size whose per-GPU share this is")
    ap.add_argument("--rank", type=int, default=7, help="the share's rank (7: one of the 32-subset blocks)")
    ap.add_argument("--n-test", type=int, default=1_000_000)
    ap.add_argument("--tile", type=int, default=65536)
    ap.add_argument("--tiles", default="0:16", help="test tiles a:b to replay in this process")
    a = ap.parse_args()
    mk = importlib.import_module(PKG)
    dmod = importlib.import_module(PKG + ".distributed")
    t = {}
    t0 = time.perf_counter()
    d = mk.synthetic.generate(a.n, q=1, n_test=a.n_test, seed=20250114)
    t["generate_s"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    _, idx = mk.partition(a.n, a.K, seed=20250114, method="R")                   # MK.R:15-41
    beta0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)                         # MK.R:53-55
    lo, hi = dmod.shard_range(a.K, a.gpus, a.rank)
    subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], 1, idx[i]) for i in range(lo, hi)]
    cfg = mk.SamplerConfig(1, 2, beta0, bt, n_batch=100, batch_length=50, seed=20250114, predict_tile=a.tile)
    t["setup_s"] = time.perf_counter() - t1
    ta, tb = (int(x) for x in a.tiles.split(":"))
    per_tile = []
    with mk.Session(subs, cfg, coords_test=d["coords_test"], subset_base=lo) as ses:
        tile = ses.predict_tile                      # the tile in use (HBM may shrink the request)
        ntiles = (a.n_test + tile - 1) // tile
        tb = min(tb, ntiles)
        t2 = time.perf_counter()
        for b in range(cfg.n_batch):                                               # MK.R:80-84
            ses.run(cfg.batch_length)
            if (b + 1) % 20 == 0:
                print(f"cfg5 share: batch {b + 1}/{cfg.n_batch}, {time.perf_counter() - t2:.1f}s", file=sys.stderr,
                      flush=True)
        t["chains_s"] = time.perf_counter() - t2
        t3 = time.perf_counter()
        out = ses.outputs(quantiles=True, samples=True, w_predict=False)             # parameter grids, MK.R:88
        t["param_grids_s"] = time.perf_counter() - t3
        kept_phi = np.stack([smp[cfg.burn_in - 1:, 3] for smp in out["samples"]])
        refreshes = int(sum(1 + np.count_nonzero(np.diff(r)) for r in kept_phi))
        for ti in range(ta, tb):
            t4 = time.perf_counter()
            g = ses.tile_grids(ti * tile)            # (S, 200, Tc): the replay of 1,251 kept states, MK.R:87-89
            t5 = time.perf_counter()
            comb = mk.combine(g)                     # the shard's sequential mean of this tile (MK.R:127-133)
            t6 = time.perf_counter()
            per_tile.append({"tile": ti, "sites": int(g.shape[2]), "replay_grids_s": t5 - t4, "combine_s": t6 - t5,
                             "finite": bool(np.isfinite(comb).all())})
            print(f"cfg5 share: tile {ti} replay+grids {t5 - t4:.1f}s combine {t6 - t5:.2f}s", file=sys.stderr,
                  flush=True)
            del g, comb
        cheb = ses.kernel_stats(mk.session.KS_KRIG_CHEB)          # tiles kriged by phi interpolation
        fallback = ses.kernel_stats(mk.session.KS_KRIG_FALLBACK)  # tiles whose check sent them to the exact replay
    t["tiles_replay_grids_s"] = sum(p["replay_grids_s"] for p in per_tile)
    t["tiles_combine_s"] = sum(p["combine_s"] for p in per_tile)
    t["process_s"] = time.perf_counter() - t0
    sites = sum(p["sites"] for p in per_tile)
    draws = len(subs) * sites * cfg.kept
    rec = {"workload": f"configs[4] per-GPU share: rank {a.rank} of {a.gpus} (subsets {lo}..{hi - 1}, {hi - lo} of "
                       f"K={a.K}, n_s={len(subs[0]['coords'])}), n={a.n}, {a.n_test} test sites in tiles of {tile}, "
                       f"100 x 50 amcmc iterations, burn.in {cfg.burn_in}, {cfg.kept} kept states",
           "tiles": [ta, tb], "n_tiles": ntiles, "phases_s": t, "per_tile": per_tile,
           "x_refreshes_per_kept_sample": refreshes / kept_phi.size,
           "draws": draws, "draws_per_s_replay": draws / max(t["tiles_replay_grids_s"], 1e-9),
           "krig_mode": os.environ.get("MK_KRIG_CHEB", "1"),
           "interpolated_tiles": cheb["launches"], "exact_evaluations": cheb["flops"],
           "max_check_difference": cheb["ms"], "fallback_tiles": fallback["launches"]}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
