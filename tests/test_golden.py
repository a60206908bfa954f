"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the oracle).

CPU: the oracle still reproduces its fixtures (regression guard of the spec).
GPU: libmk reproduces them through the C ABI -- chains, kriging draws, per-subset quantile
grids and the combined grids (tolerance 1e-8 absolute; fp64 throughout)."""
import glob
import os

import numpy as np
import pytest

from oracle import spmvglm as om

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
TOL = 1e-8


def _load(path):
    z = np.load(path)          # allow_pickle=False (default): data only
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_oracle_reproduces_golden(path):
    g = _load(path)
    q, p, cov = int(g["q"]), int(g["p"]), int(g["cov"])
    cfg = om.Config(q, p, beta_starting=np.zeros(p), beta_tuning=np.full(p, 0.05), cov_model=cov,
                    n_batch=int(g["n_batch"]), batch_length=int(g["batch_length"]), burn_in=int(g["burn_in"]),
                    seed=int(g["seed"]))
    s = 1
    r = om.fit_subset(g[f"coords_{s}"], g[f"y_{s}"], np.ones(g[f"y_{s}"].size), g[f"x_{s}"], cfg, subset=s,
                      coords_test=g["coords_test"])
    np.testing.assert_allclose(r["samples"], g[f"samples_{s}"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(r["w_q"], g[f"w_q_{s}"], rtol=0, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_device_reproduces_golden(mk, path):
    g = _load(path)
    q, p, cov, S = int(g["q"]), int(g["p"]), int(g["cov"]), int(g["S"])
    cfg = mk.SamplerConfig(q, p, beta_starting=np.zeros(p), beta_tuning=np.full(p, 0.05),
                           cov_model="matern" if cov else "exponential", n_batch=int(g["n_batch"]),
                           batch_length=int(g["batch_length"]), burn_in=int(g["burn_in"]), seed=int(g["seed"]))
    subs = [dict(coords=g[f"coords_{s}"], y=g[f"y_{s}"], weights=np.ones(g[f"y_{s}"].size), x=g[f"x_{s}"])
            for s in range(S)]
    with mk.Session(subs, cfg, coords_test=g["coords_test"], record_w=True) as ses:
        ses.run(cfg.n_samples)
        out = ses.outputs(samples=True, w_samples=True, w_pred_samples=True)
    for s in range(S):
        np.testing.assert_allclose(out["samples"][s], g[f"samples_{s}"], rtol=0, atol=TOL)
        np.testing.assert_allclose(out["w_samples"][s].T, g[f"w_samples_{s}"], rtol=0, atol=TOL)
        np.testing.assert_allclose(out["w_pred_samples"][s].T, g[f"w_pred_{s}"], rtol=0, atol=TOL)
        np.testing.assert_allclose(out["parameters"][s], g[f"param_q_{s}"], rtol=0, atol=TOL)
        np.testing.assert_allclose(out["w_predict"][s], g[f"w_q_{s}"], rtol=0, atol=TOL)
    res = mk.combine(out["parameters"])
    res2 = mk.combine(out["w_predict"])
    np.testing.assert_allclose(res, g["combined_param_q"], rtol=0, atol=TOL)
    np.testing.assert_allclose(res2, g["combined_w_q"], rtol=0, atol=TOL)
