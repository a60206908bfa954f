"""Helper run as a subprocess by tests/test_gpu_post.py (not a test module).

Multi-GPU runs (bench.py / run_metakriging.py under torch.distributed.run) initialise torch's
HIP runtime and the RCCL group BEFORE libmk loads, so libmk then runs on the runtime torch
brought.  This script reproduces that order on one GPU (an RCCL group of world 1): a short chain
replayed against the oracle, the shard's grids written by libmk into torch's HBM
(mk_session_grids) and combined there, then the device-resident column-sharded combine (mean,
sum, median) against the CPU restatements.  Prints one JSON line; exit status 0 iff all checks pass.
"""
import importlib
import json
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


def main():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    mk = importlib.import_module(PKG)                     # libmk after torch: torch's HIP runtime
    dmod = importlib.import_module(PKG + ".distributed")
    from oracle import post
    from oracle import spmvglm as om
    res = {}
    # ---- a short chain vs the oracle
    d = mk.synthetic.generate(120, q=1, n_test=8, seed=5)
    kw = dict(n_batch=2, batch_length=3, burn_in=4, seed=3)
    cfg = mk.SamplerConfig(1, 2, [0, 0], [0.05, 0.05], **kw)
    sub = dict(coords=d["coords"], y=d["y"], weights=np.ones(120), x=d["x"])
    dev = torch.device("cuda", 0)
    with mk.Session([sub, sub], cfg, coords_test=d["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        out = ses.outputs(samples=True)
        # the shard's grids written by libmk straight into torch's HBM (mk_session_grids), then the
        # column-sharded combine packs and exchanges them on the device
        gp = torch.empty((2, cfg.P, 200), dtype=torch.float64, device=dev)
        gw = torch.empty((2, 8, 200), dtype=torch.float64, device=dev)
        ses.grids_device(0, gp.data_ptr())
        ses.grids_device(1, gw.data_ptr())
    res["grids_device_exact"] = bool(np.array_equal(gp.transpose(1, 2).cpu().numpy(), np.stack(out["parameters"])) and
                                     np.array_equal(gw.transpose(1, 2).cpu().numpy(), np.stack(out["w_predict"])))
    r1 = dmod.combine_sharded(gp.transpose(1, 2), 2, dist, method="mean", device=dev, gpu=0)
    r2 = dmod.combine_sharded(gw.transpose(1, 2), 2, dist, method="mean", device=dev, gpu=0)
    res["device_combine_exact"] = bool(np.array_equal(r1, om.combine_mean(out["parameters"])) and
                                       np.array_equal(r2, om.combine_mean(out["w_predict"])))
    ref = om.fit_subset(d["coords"], d["y"], np.ones(120), d["x"], om.Config(1, 2, [0, 0], [0.05, 0.05], **kw),
                        subset=0, coords_test=d["coords_test"])
    res["chain_max_dev"] = float(np.max(np.abs(out["samples"][0] - ref["samples"])))
    res["kriging_q_max_dev"] = float(np.max(np.abs(out["w_predict"][0] - ref["w_q"])))
    # ---- device-resident combine over the RCCL group
    rng = np.random.default_rng(5)
    g = np.stack([np.sort(rng.normal(loc=rng.normal(), size=(200, 37)), axis=0) for _ in range(13)])
    mean = dmod.combine_sharded(g, 13, dist, method="mean", device=dev, gpu=0)
    tot = dmod.combine_sharded(g, 13, dist, method="sum", device=dev, gpu=0)
    med = dmod.combine_sharded(g, 13, dist, method="median", device=dev, gpu=0)
    part = dmod.combine_partial_sums(np.cumsum(g, axis=0)[-1], 13, dist, device=dev, gpu=0)
    dist.destroy_process_group()
    res["mean_exact"] = bool(np.array_equal(mean, om.combine_mean(list(g))))
    res["sum_exact"] = bool(np.array_equal(tot, np.cumsum(g, axis=0)[-1]))
    mref, _ = post.weiszfeld_median(g)
    res["median_max_dev"] = float(np.max(np.abs(med - mref)))
    res["partial_exact"] = bool(np.array_equal(part, np.cumsum(g, axis=0)[-1] / 13))
    ok = (res["chain_max_dev"] < 1e-8 and res["kriging_q_max_dev"] < 1e-8 and res["mean_exact"] and res["sum_exact"]
          and res["grids_device_exact"] and res["device_combine_exact"]
          and res["median_max_dev"] < 1e-9 * (1 + np.abs(mref).max()) and res["partial_exact"])
    res["ok"] = bool(ok)
    print(json.dumps(res), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
