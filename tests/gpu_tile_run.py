"""Helper run as a subprocess by tests/test_gpu_linalg.py (not a test module): a short chain
under the code paths the environment forces (MK_TILE, MK_SWEEP, MK_CHOL_SPLIT, MK_CHOL_DEPTH, MK_PRED_GEN; read once per process), outputs
saved to the .npz named on the command line; the latent sweeps k_sweep_mg refused admission (its
k_sweep fallback ran) are counted into <path>.fallback."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


def main(path):
    mk = importlib.import_module(PKG)
    out = {}
    fallback = 0
    for q, sizes, cov in ((1, [700, 640, 333], 0), (2, [300, 257], 0), (1, [500, 260], 1)):
        d = mk.synthetic.generate(sum(sizes), q=q, n_test=300, seed=71 + q + cov, cov_model=cov)
        p = 2 * q
        cfg = mk.SamplerConfig(q, p, np.zeros(p), np.full(p, 0.05), cov_model="matern" if cov else "exponential",
                               n_batch=2, batch_length=3, burn_in=4, seed=5)
        subs, off = [], 0
        for m in sizes:
            rows = slice(off * q, (off + m) * q)
            subs.append(dict(coords=d["coords"][off:off + m], y=d["y"][rows], weights=np.ones(m * q), x=d["x"][rows]))
            off += m
        with mk.Session(subs, cfg, coords_test=d["coords_test"], record_w=True) as ses:
            ses.run(cfg.n_samples)
            fallback += ses.kernel_stats(mk.session.KS_SWEEP_FALLBACK)["launches"]
            o = ses.outputs(samples=True, w_samples=True, w_pred_samples=True)
        for s in range(len(sizes)):
            out[f"q{q}c{cov}_samples_{s}"] = o["samples"][s]
            out[f"q{q}c{cov}_w_{s}"] = o["w_samples"][s]
            out[f"q{q}c{cov}_pred_{s}"] = o["w_pred_samples"][s]
    # tiled kriging replay (predict_tile): its own candidate factorisations of the kept states
    d = mk.synthetic.generate(557, q=1, n_test=300, seed=77)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=2, batch_length=3, burn_in=4, seed=5,
                           predict_tile=128)
    subs = [dict(coords=d["coords"][:300], y=d["y"][:300], weights=np.ones(300), x=d["x"][:300]),
            dict(coords=d["coords"][300:], y=d["y"][300:], weights=np.ones(257), x=d["x"][300:])]
    with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        o = ses.outputs(w_pred_samples=True)
    for s in range(2):
        out[f"tiled_pred_{s}"] = o["w_pred_samples"][s]
        out[f"tiled_wq_{s}"] = o["w_predict"][s]
    L, ld = mk.cholesky_batched(np.stack([np.eye(300) + 0.5 * np.exp(-np.abs(np.subtract.outer(np.arange(300.0),
                                                                                               np.arange(300.0))) / 7)
                                          for _ in range(2)]), inverse=False)
    out["chol_L"], out["chol_ld"] = L, ld
    np.savez(path, **out)
    with open(path + ".fallback", "w") as f:
        f.write(str(fallback))


if __name__ == "__main__":
    main(sys.argv[1])
