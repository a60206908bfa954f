"""configs[4] geometry pinned against the oracle (MK.R:87-89 at 1M held-out sites).

The configs[4] path krigs over tiles of 65,536 test sites after the fit (predict_tile), replaying
the recorded chain states of every kept iteration through the n_s = 2,000 kriging GEMM.  Here two
exponential subsets of n_s = 2,000 (configs[2]'s subset size) krig 70,000 sites: one full tile
and a ragged one.  A fixed sample of sites spread over both tiles (both tile edges and the last
site included) is checked against the CPU oracle, which krigs only those sites but draws the same
Philox streams (keyed by the global site index, ``site_index``): per-site draws of every kept
iteration, the 200-level quantile grids and the two subsets' sum of grids, all to 1e-8.
"""
import numpy as np
import pytest

from oracle import spmvglm as om

pytestmark = pytest.mark.gpu
TOL = 1e-8


def test_cfg5_tiled_kriging_matches_oracle_on_sampled_sites(mk):
    n, n_test, tile, S, base = 2000, 70_000, 65536, 2, 3
    d = mk.synthetic.generate(S * n, q=1, n_test=n_test, seed=505, cov_model=0)
    ct = d["coords_test"]
    kw = dict(n_batch=2, batch_length=3, burn_in=3, seed=21)     # 6 iterations, 4 kept
    cfg = mk.SamplerConfig(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05), predict_tile=tile, **kw)
    ocfg = om.Config(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05), cov_model=0, **kw)
    subs = [dict(coords=d["coords"][s * n:(s + 1) * n], y=d["y"][s * n:(s + 1) * n], weights=np.ones(n),
                 x=d["x"][s * n:(s + 1) * n]) for s in range(S)]
    with mk.Session(subs, cfg, coords_test=ct, subset_base=base) as ses:
        ses.run(cfg.n_samples)
        dev = ses.outputs(samples=True, w_pred_samples=True, w_predict_sum=True)
    assert dev["w_predict"][0].shape == (200, n_test)
    rng = np.random.default_rng(7)
    edges = {0, tile - 1, tile, n_test - 1}
    sites = np.array(sorted(edges | set(rng.choice(n_test, 60, replace=False).tolist())), dtype=np.int64)
    assert (sites < tile).any() and (sites >= tile).any()
    grid_sum = None
    for s, sb in enumerate(subs):
        ref = om.fit_subset(sb["coords"], sb["y"], sb["weights"], sb["x"], ocfg, subset=base + s,
                            coords_test=ct[sites], site_index=sites)
        np.testing.assert_allclose(dev["samples"][s], ref["samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_pred_samples"][s][sites].T, ref["w_pred"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_predict"][s][:, sites], ref["w_q"], rtol=0, atol=TOL)
        grid_sum = ref["w_q"] if grid_sum is None else grid_sum + ref["w_q"]
    np.testing.assert_allclose(dev["w_predict_sum"][:, sites], grid_sum, rtol=0, atol=TOL)
    # the sum over the two subsets is the sequential one (MK.R:129-132), over every site
    assert np.array_equal(dev["w_predict_sum"], dev["w_predict"][0] + dev["w_predict"][1])


def test_kriging_tile_shrinks_to_fit_and_draws_do_not_change(mk, monkeypatch):
    """A tiled session whose requested tile's kriging buffers do not fit (here a budget,
    MK_KRIG_MEM_GB; in production HBM itself: configs[4]'s 250 subsets at 65,536 sites would need
    ~700 GB on one GPU) takes the largest tile that fits, halving in 256-site steps, and reports it
    (mk_session_predict_tile).  The draws are keyed by the global site index, so they equal a session
    given that tile outright and the fused path, bit for bit; the grids likewise."""
    n, n_test, S = 200, 20_000, 3
    d = mk.synthetic.generate(S * n, q=1, n_test=n_test, seed=77, cov_model=0)
    kw = dict(n_batch=2, batch_length=3, burn_in=4, seed=5)      # 6 iterations, 3 kept
    subs = [dict(coords=d["coords"][s * n:(s + 1) * n], y=d["y"][s * n:(s + 1) * n], weights=np.ones(n),
                 x=d["x"][s * n:(s + 1) * n]) for s in range(S)]

    def run(tile, budget=None):
        if budget is not None:
            monkeypatch.setenv("MK_KRIG_MEM_GB", str(budget))
        else:
            monkeypatch.delenv("MK_KRIG_MEM_GB", raising=False)
        cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), predict_tile=tile, **kw)
        with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
            t = ses.predict_tile
            ses.run(cfg.n_samples)
            out = ses.outputs(w_pred_samples=True)
        monkeypatch.delenv("MK_KRIG_MEM_GB", raising=False)
        return t, out

    # 16,384 sites need 3 x 16,384 x (1 + 2 + 2 x 256) doubles + the draws = 0.2 GB; 0.06 GB allows 4,096
    t_small, small = run(16384, budget=0.06)
    assert t_small < 16384 and t_small % 256 == 0
    t_ref, ref = run(t_small)
    assert t_ref == t_small
    _, fused = run(0)
    for k in ("w_pred_samples", "w_predict"):
        assert np.array_equal(small[k], ref[k]), k
        assert np.array_equal(small[k], fused[k]), k
