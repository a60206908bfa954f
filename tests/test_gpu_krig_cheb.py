"""The kriging variance by phi interpolation (MK.R:87-89): the tiled replay
(spPredict after the fit, mk_api.hip predict_tile_cheb) and the fused path's phi tables (krig_tables).

The kriging variance s(t; phi) = rho_t(phi)' R(phi)^-1 rho_t(phi) is computed exactly at Chebyshev
nodes of each subset's kept phi range and interpolated at every kept state's phi; the mean is
rho_t(phi_k)' g_k with g_k = W_k' z_k.  Every tile checks the interpolant against exact values at the
range's ends and middle and sends the tile to the exact replay when they differ by more than
MK_KRIG_CHEB_TOL (1e-10).  The draws then agree with the exact replay (and through it with the CPU
oracle) to rounding: 1e-8 absolute here, the tolerance the configs[4] oracle test uses.
MK_KRIG_CHEB: 0 exact replay, 1 (default) where it saves exact evaluations, -1 always, n > 1 always
with n nodes (the library reads it at every tile).
"""
import numpy as np
import pytest

from oracle import spmvglm as om

pytestmark = pytest.mark.gpu
TOL = 1e-8


def _problem(mk, sizes, n_test, seed):
    d = mk.synthetic.generate(sum(sizes), q=1, n_test=n_test, seed=seed, cov_model=0)
    subs, off = [], 0
    for m in sizes:
        subs.append(dict(coords=d["coords"][off:off + m], y=d["y"][off:off + m], weights=np.ones(m),
                         x=d["x"][off:off + m]))
        off += m
    return subs, d["coords_test"]


def _run(mk, monkeypatch, subs, ct, cfg, mode, base=0):
    monkeypatch.setenv("MK_KRIG_CHEB", mode)
    with mk.Session(subs, cfg, coords_test=ct, subset_base=base) as ses:
        ses.run(cfg.n_samples)
        out = ses.outputs(samples=True, w_pred_samples=True, w_predict_sum=True)
        out["cheb"] = ses.kernel_stats(mk.session.KS_KRIG_CHEB)
        out["fallback"] = ses.kernel_stats(mk.session.KS_KRIG_FALLBACK)
    monkeypatch.delenv("MK_KRIG_CHEB", raising=False)
    return out


def test_interpolated_kriging_matches_the_exact_replay(mk, monkeypatch):
    """Ragged subsets, three tiles (the last short), 31 kept states over which phi moves: the
    interpolated tiles' draws, quantile grids and grid sum equal the exact replay's to 1e-8, every
    tile passed its check (none replayed), and the largest check difference is at rounding level."""
    subs, ct = _problem(mk, [400, 350, 301], 2500, seed=61)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=4, batch_length=10, burn_in=10, seed=8,
                           predict_tile=1024)
    exact = _run(mk, monkeypatch, subs, ct, cfg, "0")
    cheb = _run(mk, monkeypatch, subs, ct, cfg, "-1")
    assert exact["cheb"]["launches"] == 0
    assert cheb["cheb"]["launches"] == 3 and cheb["fallback"]["launches"] == 0, (cheb["cheb"], cheb["fallback"])
    assert cheb["cheb"]["ms"] < 1e-11, cheb["cheb"]            # the largest check difference
    n_phi = [len(set(np.round(exact["samples"][s][cfg.burn_in - 1:, -1], 15))) for s in range(3)]
    assert min(n_phi) >= 5, n_phi                                # phi moved over the kept window
    for s in range(3):
        assert np.array_equal(cheb["samples"][s], exact["samples"][s])
        np.testing.assert_allclose(cheb["w_pred_samples"][s], exact["w_pred_samples"][s], rtol=0, atol=TOL)
        np.testing.assert_allclose(cheb["w_predict"][s], exact["w_predict"][s], rtol=0, atol=TOL)
    np.testing.assert_allclose(cheb["w_predict_sum"], exact["w_predict_sum"], rtol=0, atol=3 * TOL)


def test_failed_check_replays_the_tile_exactly(mk, monkeypatch):
    """Two nodes cannot follow s over a moving phi range: every tile's check fails and the tile is
    replayed exactly -- the same bits as the exact replay, and the fallback counted."""
    subs, ct = _problem(mk, [300, 260], 1500, seed=62)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=3, batch_length=8, burn_in=6, seed=4,
                           predict_tile=1024)
    exact = _run(mk, monkeypatch, subs, ct, cfg, "0")
    forced = _run(mk, monkeypatch, subs, ct, cfg, "2")
    assert forced["cheb"]["launches"] == 0 and forced["fallback"]["launches"] == 2, forced["fallback"]
    assert forced["fallback"]["ms"] > 1e-10
    for s in range(2):
        assert np.array_equal(forced["w_pred_samples"][s], exact["w_pred_samples"][s])
        assert np.array_equal(forced["w_predict"][s], exact["w_predict"][s])


def test_auto_mode_keeps_the_exact_replay_for_short_windows(mk, monkeypatch):
    """With few kept states the exact replay refreshes less often than a range needs nodes: the
    default mode keeps it (the bit-identity tests of the tiled path rely on this)."""
    subs, ct = _problem(mk, [200, 180], 600, seed=63)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=2, batch_length=4, burn_in=5, seed=2,
                           predict_tile=256)
    auto = _run(mk, monkeypatch, subs, ct, cfg, "1")
    exact = _run(mk, monkeypatch, subs, ct, cfg, "0")
    assert auto["cheb"]["launches"] == 0 and auto["fallback"]["launches"] == 0
    for s in range(2):
        assert np.array_equal(auto["w_pred_samples"][s], exact["w_pred_samples"][s])


def test_interpolated_kriging_matches_the_oracle(mk, monkeypatch):
    """Against the CPU oracle (which krigs every kept state exactly, MK.R:87) at sampled sites of two
    tiles, subset_base offset: draws, grids and their sum to 1e-8 (configs[4]'s oracle bar)."""
    n, n_test, tile, S, base = 600, 3000, 2048, 2, 5
    subs, ct = _problem(mk, [n] * S, n_test, seed=64)
    kw = dict(n_batch=3, batch_length=8, burn_in=5, seed=13)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), predict_tile=tile, **kw)
    dev = _run(mk, monkeypatch, subs, ct, cfg, "-1", base=base)
    assert dev["cheb"]["launches"] == 2 and dev["fallback"]["launches"] == 0
    ocfg = om.Config(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05), cov_model=0, **kw)
    rng = np.random.default_rng(3)
    sites = np.array(sorted({0, tile - 1, tile, n_test - 1} | set(rng.choice(n_test, 40, replace=False).tolist())))
    grid_sum = None
    for s, sb in enumerate(subs):
        ref = om.fit_subset(sb["coords"], sb["y"], sb["weights"], sb["x"], ocfg, subset=base + s,
                            coords_test=ct[sites], site_index=sites)
        np.testing.assert_allclose(dev["samples"][s], ref["samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_pred_samples"][s][sites].T, ref["w_pred"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_predict"][s][:, sites], ref["w_q"], rtol=0, atol=TOL)
        grid_sum = ref["w_q"] if grid_sum is None else grid_sum + ref["w_q"]
    np.testing.assert_allclose(dev["w_predict_sum"][:, sites], grid_sum, rtol=0, atol=2 * TOL)


# ---- the fused path's phi tables (mk_api.hip krig_tables): s(t; phi) tabulated over the prior's phi
# range at session creation; kept iterations draw with g = W' z and the interpolated s

def _fused(mk, monkeypatch, subs, ct, cfg, mode, base=0, lookahead=-1):
    monkeypatch.setenv("MK_KRIG_CHEB", mode)
    with mk.Session(subs, cfg, coords_test=ct, subset_base=base) as ses:
        ses.set_lookahead(lookahead)
        assert lookahead == -1 or ses.lookahead == bool(lookahead)
        ses.run(cfg.n_samples)
        out = ses.outputs(samples=True, w_pred_samples=True, w_predict_sum=True)
        out["cheb"] = ses.kernel_stats(mk.session.KS_KRIG_CHEB)
        out["fallback"] = ses.kernel_stats(mk.session.KS_KRIG_FALLBACK)
    monkeypatch.delenv("MK_KRIG_CHEB", raising=False)
    return out


@pytest.mark.parametrize("lookahead", [True, False])
def test_fused_phi_tables_match_the_exact_refresh(mk, monkeypatch, lookahead):
    """Fused kriging (draws inside the kept iterations, MK.R:87 fused into the fit) from the phi tables
    against the exact X = W P^T refresh: the chain is untouched (samples bit for bit), the draws, grids
    and their sum agree to 1e-8, every kept iteration drew from the tables, and the set-up check
    (5 points of the prior's range) is at rounding level.  Both launch schedules."""
    subs, ct = _problem(mk, [300, 257, 280], 700, seed=65)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=4, batch_length=10, burn_in=10, seed=6)
    exact = _fused(mk, monkeypatch, subs, ct, cfg, "0", lookahead=int(lookahead))
    tab = _fused(mk, monkeypatch, subs, ct, cfg, "-1", lookahead=int(lookahead))
    assert exact["cheb"]["launches"] == 0
    assert tab["cheb"]["launches"] == cfg.kept and tab["fallback"]["launches"] == 0, (tab["cheb"], tab["fallback"])
    assert 0 < tab["cheb"]["ms"] < 1e-11, tab["cheb"]
    for s in range(3):
        assert np.array_equal(tab["samples"][s], exact["samples"][s])
        np.testing.assert_allclose(tab["w_pred_samples"][s], exact["w_pred_samples"][s], rtol=0, atol=TOL)
        np.testing.assert_allclose(tab["w_predict"][s], exact["w_predict"][s], rtol=0, atol=TOL)
    np.testing.assert_allclose(tab["w_predict_sum"], exact["w_predict_sum"], rtol=0, atol=3 * TOL)


def test_fused_phi_tables_failed_check_keeps_the_exact_refresh(mk, monkeypatch):
    """Two nodes over the prior's range fail the set-up check: the session keeps the exact refresh
    (the same bits) and counts the failure."""
    subs, ct = _problem(mk, [200, 220], 300, seed=66)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=2, batch_length=6, burn_in=4, seed=3)
    exact = _fused(mk, monkeypatch, subs, ct, cfg, "0")
    forced = _fused(mk, monkeypatch, subs, ct, cfg, "2")
    assert forced["cheb"]["launches"] == 0 and forced["fallback"]["launches"] == 1
    assert forced["fallback"]["ms"] > 1e-10
    for s in range(2):
        assert np.array_equal(forced["w_pred_samples"][s], exact["w_pred_samples"][s])


def test_fused_phi_tables_match_the_oracle(mk, monkeypatch):
    """The fused path from the tables against the CPU oracle's exact spPredict (per kept iteration),
    subset_base offset: samples, draws and grids to 1e-8."""
    n, n_test, S, base = 500, 400, 2, 9
    subs, ct = _problem(mk, [n] * S, n_test, seed=67)
    kw = dict(n_batch=3, batch_length=6, burn_in=5, seed=17)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), **kw)
    dev = _fused(mk, monkeypatch, subs, ct, cfg, "-1", base=base)
    assert dev["cheb"]["launches"] == cfg.kept
    ocfg = om.Config(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05), cov_model=0, **kw)
    for s, sb in enumerate(subs):
        ref = om.fit_subset(sb["coords"], sb["y"], sb["weights"], sb["x"], ocfg, subset=base + s, coords_test=ct)
        np.testing.assert_allclose(dev["samples"][s], ref["samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_pred_samples"][s].T, ref["w_pred"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_predict"][s], ref["w_q"], rtol=0, atol=TOL)


@pytest.mark.parametrize("tile", [0, 700])
def test_interpolated_kriging_is_shard_invariant(mk, monkeypatch, tile):
    """mk_meta_fit over virtual blocks (each its own session of some of the subsets) gives what one
    session gives, bit for bit, with the interpolation forced on both sides: a subset's nodes depend
    only on its own phi range and distances, its node GEMMs and draws only on its own data (fused tables,
    tile = 0; tiled replay exchanged tile by tile, tile = 700)."""
    subs, ct = _problem(mk, [260, 300, 241], 1500, seed=68)
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=3, batch_length=8, burn_in=6, seed=7,
                           predict_tile=tile)
    monkeypatch.setenv("MK_KRIG_CHEB", "-1")
    with mk.Session(subs, cfg, coords_test=ct, subset_base=4) as ses:
        ses.run(cfg.n_samples)
        ref = ses.outputs(w_pred_samples=True, w_predict_sum=True)
        assert ses.kernel_stats(mk.session.KS_KRIG_CHEB)["launches"] > 0
    got = mk.meta_fit_node(subs, cfg, coords_test=ct, devices=[0, 0], subset_base=4, w_pred_samples=True,
                           w_predict_sum=True)
    for s in range(3):
        assert np.array_equal(got["w_pred_samples"][s], ref["w_pred_samples"][s]), s
        assert np.array_equal(got["w_predict"][s], ref["w_predict"][s]), s
    assert np.array_equal(got["w_predict_sum"], ref["w_predict_sum"])
