"""Short-horizon replay: the device chain vs the CPU oracle on identical inputs and
identical Philox draws.  Every accept/reject decision must agree (samples equal to
fp rounding, tolerance 1e-8 absolute on O(1) parameters); kriging draws and the
200-level quantile grids likewise.  Quantiles of identical inputs are bit-exact."""
import numpy as np
import pytest

from oracle import spmvglm as om
from oracle.rstats import PROBS200, r_quantile7

pytestmark = pytest.mark.gpu
TOL = 1e-8


def _run_both(mk, n, q, cov, n_test=12, n_batch=3, batch_length=4, burn_in=7, seed=9, subset_base=0, S=2,
              sizes=None, link="logit", lookahead=None, chunks=None):
    sizes = list(sizes) if sizes is not None else [n] * S
    off = np.concatenate([[0], np.cumsum(sizes)])
    d = mk.synthetic.generate(int(off[-1]), q=q, n_test=n_test, seed=seed + q, cov_model=cov, link=link)
    ct = d["coords_test"] if n_test else None
    p = 2 * q
    kw = dict(n_batch=n_batch, batch_length=batch_length, burn_in=burn_in, seed=seed)
    cfg = mk.SamplerConfig(q, p, beta_starting=np.zeros(p), beta_tuning=np.full(p, 0.05),
                           cov_model="matern" if cov else "exponential", link=link, **kw)
    ocfg = om.Config(q, p, beta_starting=np.zeros(p), beta_tuning=np.full(p, 0.05), cov_model=cov,
                     link=om.LINK_PROBIT if link == "probit" else om.LINK_LOGIT, **kw)
    subs = []
    for s, m in enumerate(sizes):
        sl = slice(off[s], off[s] + m)
        rows = slice(off[s] * q, (off[s] + m) * q)
        subs.append(dict(coords=d["coords"][sl], y=d["y"][rows], weights=np.ones(m * q), x=d["x"][rows]))
    with mk.Session(subs, cfg, coords_test=ct, subset_base=subset_base, record_w=True, lookahead=lookahead) as ses:
        if lookahead is not None:
            assert ses.lookahead == bool(lookahead)
        for c in (chunks or [cfg.n_samples]):
            ses.run(c)
        dev = ses.outputs(samples=True, w_samples=True, w_pred_samples=True, acceptance=True)
    refs = [om.fit_subset(sb["coords"], sb["y"], sb["weights"], sb["x"], ocfg, subset=subset_base + s,
                          coords_test=ct, record_w=True) for s, sb in enumerate(subs)]
    return dev, refs


def _check(dev, refs):
    for s, ref in enumerate(refs):
        np.testing.assert_allclose(dev["samples"][s], ref["samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_samples"][s].T, ref["w_samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["parameters"][s], ref["param_q"], rtol=0, atol=TOL)
        if "w_q" in ref:
            np.testing.assert_allclose(dev["w_pred_samples"][s].T, ref["w_pred"], rtol=0, atol=TOL)
            np.testing.assert_allclose(dev["w_predict"][s], ref["w_q"], rtol=0, atol=TOL)
        else:
            assert "w_predict" not in dev and "w_pred_samples" not in dev
        # accept rates of beta / A / phi per batch
        o_w = dev["acceptance"][s].shape[1] - 1
        np.testing.assert_allclose(dev["acceptance"][s][:, :o_w], ref["accept"][:, :o_w], atol=1e-12)


@pytest.mark.parametrize("n,q,cov", [(150, 1, 0), (300, 1, 0), (64, 2, 0), (100, 1, 1), (40, 3, 0), (48, 2, 1), (30, 4, 0)])
def test_replay_matches_oracle(mk, n, q, cov):
    dev, refs = _run_both(mk, n, q, cov)
    _check(dev, refs)


@pytest.mark.parametrize("sizes,q", [([150, 163, 127], 1), ([128, 129], 1), ([64, 71], 2)])
def test_replay_ragged_subsets(mk, sizes, q):
    """Subsets of different sizes in one session (the reference's last subset takes the
    remainder, MK.R:18); sizes straddle the 128-tile boundary with the bordered row."""
    dev, refs = _run_both(mk, None, q, 0, sizes=sizes)
    _check(dev, refs)


@pytest.mark.parametrize("sizes,q,cov", [([1, 2, 3], 1, 0), ([1, 2], 2, 0), ([1, 3], 1, 1)])
def test_replay_tiny_subsets(mk, sizes, q, cov):
    """Subsets of one to three sites (the remainder subset of MK.R:18 can be that small): the
    bordered row sits in the first tile next to the identity padding."""
    dev, refs = _run_both(mk, None, q, cov, sizes=sizes, n_test=5)
    _check(dev, refs)


@pytest.mark.parametrize("q", [1, 2])
def test_replay_without_test_sites(mk, q):
    """No kriging sites (coords.test empty): the fit alone replays the oracle and no
    w.predict output is produced."""
    dev, refs = _run_both(mk, None, q, 0, sizes=[70, 45], n_test=0)
    _check(dev, refs)


def test_replay_cfg3_subset_size(mk):
    """A configs[2] subset (n_s = 2000, 16 tiles of 128 with the bordered row in the last):
    a short chain replayed against the oracle."""
    dev, refs = _run_both(mk, 2000, 1, 0, n_test=40, n_batch=2, batch_length=2, burn_in=3, S=1)
    _check(dev, refs)


def test_replay_cfg2_matern_geometry(mk):
    """configs[1] geometry: Matern, q = 1, n_s = 1000 (50,000 sites / 50 subsets; 8 tiles of 128
    with the bordered row in the last).  Every phi and nu candidate goes through the binned
    Bessel candidate kernel; 6 iterations with accepted and rejected phi / nu steps
    (MK.R:80-84 with cov.model = "matern")."""
    dev, refs = _run_both(mk, 1000, 1, 1, n_test=40, n_batch=2, batch_length=3, burn_in=4, S=1)
    acc = refs[0]["accept"]
    assert 0 < acc[:, 4].sum() < 2 and 0 < acc[:, 3].sum() < 2     # nu, phi: some accepted, some not
    _check(dev, refs)


def test_replay_cfg4_lmc_geometry(mk):
    """configs[3] geometry: q = 3 LMC, n_s = 2000 (100,000 sites / 50 subsets), N = 6000: multi-tile
    factors for each outcome (16 tiles), k_trmv_Z staging four 512-column chunks, 64-site sweep
    blocks with three outcomes per site, kriging of 3 x 40 test outcomes (MK.R:80 formula list)."""
    dev, refs = _run_both(mk, 2000, 3, 0, n_test=40, n_batch=2, batch_length=3, burn_in=4, S=1)
    _check(dev, refs)


def test_replay_lmc_ragged_multi_tile(mk):
    """q = 2 and q = 3 LMC with several multi-tile subsets of different sizes in one session
    (ragged across the 128 and 512 boundaries)."""
    for q, sizes in ((2, [700, 513]), (3, [600, 129])):
        dev, refs = _run_both(mk, None, q, 0, sizes=sizes, n_test=24, n_batch=2, batch_length=2, burn_in=3)
        _check(dev, refs)


@pytest.mark.parametrize("n,q,cov", [(150, 1, 0), (48, 2, 0), (100, 1, 1), (40, 3, 0)])
def test_replay_probit_matches_oracle(mk, n, q, cov):
    """Probit link (north-star "logit/probit"; the reference is logit, so the oracle's probit
    likelihood is the spec): y log Phi(eta) + (wt - y) log Phi(-eta) in the beta and w steps."""
    dev, refs = _run_both(mk, n, q, cov, link="probit")
    _check(dev, refs)


def test_replay_subset_beyond_2048_sites(mk):
    """n_s = 2200 (18 tiles): the sweep's row-pair pass wraps (more rows than 2 x its 1024
    threads) and the diagonal-tile kernel runs past 16 pivots; replayed against the oracle."""
    dev, refs = _run_both(mk, 2200, 1, 0, n_test=16, n_batch=2, batch_length=2, burn_in=3, S=1)
    _check(dev, refs)


@pytest.mark.parametrize("n,q,sizes,cov", [(150, 1, None, 0), (None, 1, [700, 333], 0), (64, 2, None, 0),
                                           (None, 3, [300, 129], 0), (None, 1, [1, 2, 3], 0), (100, 1, None, 1),
                                           (None, 2, [130, 90], 1)])
def test_replay_sequential_schedule(mk, n, q, sizes, cov):
    """The sequential launch schedule (bordered candidates: z' is the factor's row n_s) replays the
    oracle too (exponential and Matern); the default for shards of up to 224 (subset, outcome)
    pairs is the lookahead schedule."""
    dev, refs = _run_both(mk, n, q, cov, sizes=sizes, lookahead=0)
    _check(dev, refs)


@pytest.mark.parametrize("n,q,sizes,cov", [(150, 1, None, 0), (None, 1, [1300, 700, 129], 0), (None, 2, [400, 257], 0),
                                           (None, 3, [300, 2, 129], 0), (None, 1, [1000, 300], 1),
                                           (48, 2, None, 1), (None, 1, [1, 3], 1)])
def test_lookahead_schedule_replays_oracle(mk, n, q, sizes, cov):
    """Lookahead schedule: iteration t+1's phi candidates are factored without a
    bordered row while iteration t's inverse and sweep run, and z' = L'^-1 u comes from the
    trailing border solve (k_border_step / k_border_combine); Matern: the nu candidate follows the
    phi decision with its bordered row, and its row replaces z' where nu is accepted (k_nu_border).
    Replayed against the oracle across batch ends (adapted proposal scales) and across
    mk_session_run calls that stop mid-batch (the candidate queued by one call is used by the
    next); [1000, 300] is the configs[1] subset size."""
    dev, refs = _run_both(mk, n, q, cov, sizes=sizes, lookahead=1, chunks=[1, 4, 2, 5])
    _check(dev, refs)


@pytest.mark.parametrize("cov,sizes", [(0, [900, 650]), (1, [700, 400])])
def test_lookahead_equals_sequential_schedule(mk, cov, sizes):
    """Both schedules run the same chain: every decision agrees and the states differ by rounding
    only (z' from a forward solve instead of the bordered factor row)."""
    a, _ = _run_both(mk, None, 1, cov, sizes=sizes, n_batch=4, batch_length=3, burn_in=9, lookahead=1)
    b, _ = _run_both(mk, None, 1, cov, sizes=sizes, n_batch=4, batch_length=3, burn_in=9, lookahead=0)
    for s in range(2):
        np.testing.assert_allclose(a["samples"][s], b["samples"][s], rtol=0, atol=1e-10)
        np.testing.assert_allclose(a["w_samples"][s], b["w_samples"][s], rtol=0, atol=1e-10)
        np.testing.assert_allclose(a["w_pred_samples"][s], b["w_pred_samples"][s], rtol=0, atol=1e-10)
        assert np.array_equal(a["acceptance"][s], b["acceptance"][s])


def test_lookahead_is_rejected_where_ineligible(mk):
    """Sessions that run their subsets as several stream groups (n_streams > 1) keep the
    sequential schedule; asking for lookahead there is an argument error, as is changing the
    schedule after the chain has started.  Both covariance models are eligible otherwise."""
    d = mk.synthetic.generate(60, q=1, n_test=3, seed=3, cov_model=1)
    sub = [dict(coords=d["coords"][:30], y=d["y"][:30], weights=np.ones(30), x=d["x"][:30]),
           dict(coords=d["coords"][30:], y=d["y"][30:], weights=np.ones(30), x=d["x"][30:])]
    cfg = mk.SamplerConfig(1, 2, [0, 0], [0.05, 0.05], cov_model="matern", n_batch=1, batch_length=3, burn_in=2,
                           n_streams=2)
    with mk.Session(sub, cfg) as ses:
        assert not ses.lookahead
        with pytest.raises(mk.MkError):
            ses.set_lookahead(1)
    for cov in ("exponential", "matern"):
        cfg = mk.SamplerConfig(1, 2, [0, 0], [0.05, 0.05], cov_model=cov, n_batch=1, batch_length=3, burn_in=2)
        with mk.Session(sub, cfg) as ses:
            assert ses.lookahead
            ses.run(1)
            with pytest.raises(mk.MkError):
                ses.set_lookahead(0)


@pytest.mark.parametrize("shift", [(2.5, -1.0), (0.0, 0.0)])
def test_matern_kriging_test_sites_outside_the_subsets(mk, shift):
    """Matern kriging tables (k_matern_table_list / k_pred_PT_matern) span phi x the largest
    subset-to-test-site distance (host bounding boxes): test sites moved outside the subsets'
    extent still replay the oracle's kriging draws (sites beyond the table take the exact path)."""
    sizes = [300, 170]
    d = mk.synthetic.generate(sum(sizes), q=1, n_test=40, seed=31, cov_model=1)
    ct = d["coords_test"] + np.asarray(shift)[None, :]
    kw = dict(n_batch=2, batch_length=3, burn_in=4, seed=13)
    cfg = mk.SamplerConfig(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05), cov_model="matern", **kw)
    ocfg = om.Config(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05), cov_model=1, **kw)
    subs, off = [], 0
    for m in sizes:
        subs.append(dict(coords=d["coords"][off:off + m], y=d["y"][off:off + m], weights=np.ones(m),
                         x=d["x"][off:off + m]))
        off += m
    with mk.Session(subs, cfg, coords_test=ct) as ses:
        ses.run(cfg.n_samples)
        dev = ses.outputs(samples=True, w_pred_samples=True)
    for s, sb in enumerate(subs):
        ref = om.fit_subset(sb["coords"], sb["y"], sb["weights"], sb["x"], ocfg, subset=s, coords_test=ct)
        np.testing.assert_allclose(dev["samples"][s], ref["samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_pred_samples"][s].T, ref["w_pred"], rtol=0, atol=TOL)


def test_quantiles_bit_exact_on_device_samples(mk):
    dev, _ = _run_both(mk, 130, 1, 0, n_batch=4, batch_length=5, burn_in=3)
    for s in range(len(dev["samples"])):
        kept = dev["samples"][s][2:]
        assert np.array_equal(dev["parameters"][s], r_quantile7(kept, PROBS200, axis=0))
        assert np.array_equal(dev["w_predict"][s], r_quantile7(dev["w_pred_samples"][s].T, PROBS200, axis=0))


def test_subset_streams_independent_of_sharding(mk):
    """Subset k's chain depends only on (seed, global subset index): sharding-invariant."""
    d = mk.synthetic.generate(240, q=1, n_test=4, seed=2)
    cfg = mk.SamplerConfig(1, 2, beta_starting=[0, 0], beta_tuning=[0.05, 0.05], n_batch=2, batch_length=3, burn_in=4)
    subs = [dict(coords=d["coords"][i * 80:(i + 1) * 80], y=d["y"][i * 80:(i + 1) * 80], weights=np.ones(80),
                 x=d["x"][i * 80:(i + 1) * 80]) for i in range(3)]
    with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        allq = ses.outputs()
    with mk.Session(subs[2:], cfg, coords_test=d["coords_test"], subset_base=2) as ses:
        ses.run(cfg.n_samples)
        oneq = ses.outputs()
    assert np.array_equal(allq["parameters"][2], oneq["parameters"][0])
    assert np.array_equal(allq["w_predict"][2], oneq["w_predict"][0])


@pytest.mark.parametrize("n,q,cov,tile", [(150, 1, 0, 5), (64, 2, 0, 7), (100, 1, 1, 4), (120, 1, 0, 1)])
def test_tiled_kriging_is_bit_identical_to_fused(mk, n, q, cov, tile):
    """spPredict replayed after the fit over test-site tiles (the cfg5 path: 1M sites) gives the
    fused path's draws, quantile grids and their subset sum exactly."""
    S, n_test = 3, 12
    d = mk.synthetic.generate(n * S, q=q, n_test=n_test, seed=31 + q, cov_model=cov)
    p = 2 * q
    subs = [dict(coords=d["coords"][s * n:(s + 1) * n], y=d["y"][s * n * q:(s + 1) * n * q], weights=np.ones(n * q),
                 x=d["x"][s * n * q:(s + 1) * n * q]) for s in range(S)]
    outs = []
    for pt in (0, tile):
        cfg = mk.SamplerConfig(q, p, beta_starting=np.zeros(p), beta_tuning=np.full(p, 0.05),
                               cov_model="matern" if cov else "exponential", n_batch=3, batch_length=4, burn_in=5,
                               seed=12, predict_tile=pt)
        with mk.Session(subs, cfg, coords_test=d["coords_test"], subset_base=4) as ses:
            ses.run(cfg.n_samples)
            outs.append(ses.outputs(samples=True, w_pred_samples=True, w_predict_sum=True))
    fused, tiled = outs
    for s in range(S):
        assert np.array_equal(tiled["samples"][s], fused["samples"][s])
        assert np.array_equal(tiled["w_pred_samples"][s], fused["w_pred_samples"][s])
        assert np.array_equal(tiled["w_predict"][s], fused["w_predict"][s])
    assert np.array_equal(tiled["w_predict_sum"], fused["w_predict_sum"])
    seq = fused["w_predict"][0].copy()
    for s in range(1, S):
        seq = seq + fused["w_predict"][s]
    assert np.array_equal(fused["w_predict_sum"], seq)


@pytest.mark.parametrize("cov", [0, 1])
def test_tiled_kriging_at_the_cfg5_tile_size(mk, cov):
    """configs[4]'s tile geometry: 70,000 test sites over tiles of 65,536 (run_metakriging.py's
    predict_tile; a full tile and a short ragged one) give the fused path's draws and quantile
    grids exactly (draws keyed by the global site index; Matern: the kriging tables per tile)."""
    n, n_test = 300, 70_000
    d = mk.synthetic.generate(2 * n, q=1, n_test=n_test, seed=77 + cov, cov_model=cov)
    subs = [dict(coords=d["coords"][s * n:(s + 1) * n], y=d["y"][s * n:(s + 1) * n], weights=np.ones(n),
                 x=d["x"][s * n:(s + 1) * n]) for s in range(2)]
    outs = []
    for pt in (0, 65536):
        cfg = mk.SamplerConfig(1, 2, beta_starting=np.zeros(2), beta_tuning=np.full(2, 0.05),
                               cov_model="matern" if cov else "exponential", n_batch=2, batch_length=3, burn_in=5,
                               seed=3, predict_tile=pt)
        with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
            ses.run(cfg.n_samples)
            outs.append(ses.outputs(w_pred_samples=True, w_predict_sum=True))
    fused, tiled = outs
    for s in range(2):
        assert np.array_equal(tiled["w_pred_samples"][s], fused["w_pred_samples"][s])
        assert np.array_equal(tiled["w_predict"][s], fused["w_predict"][s])
    assert np.array_equal(tiled["w_predict_sum"], fused["w_predict_sum"])


@pytest.mark.parametrize("q,cov", [(1, 0), (2, 0), (1, 1)])
def test_sppredict_reuses_the_fit_without_refitting(mk, q, cov):
    """spMvGLM keeps every chain state on the device; spPredict(start, end, thin) only krigs
    (mk_session_set_test_sites + mk_session_set_kept_window).  Its draws equal those of a session
    that fused the kriging into iterations start..n.samples (burn_in = start), and spMvGLM's
    samples equal that session's chain (MK.R:80-87: spMvGLM then spPredict(start = burn.in))."""
    n, n_test, start = 90, 11, 7
    d = mk.synthetic.generate(n, q=q, n_test=n_test, seed=41 + q + cov, cov_model=cov)
    p = 2 * q
    formula = [(d["y"][a::q], d["x"][a::q, 2 * a:2 * a + 2]) for a in range(q)]
    starting = {"beta": np.zeros(p), "phi": 3 / 0.5, "A": np.eye(q)[np.tril_indices(q)], "w": 0.0}
    tuning = {"beta": np.full(p, 0.05), "phi": 1.0, "A": 0.1, "w": 0.5}
    priors = {"phi.Unif": (3 / 0.75, 3 / 0.25), "K.IW": (q, 0.1 * np.eye(q))}
    if cov:
        starting["nu"], tuning["nu"], priors["nu.Unif"] = 0.5, 0.1, (0.1, 2.0)
    amcmc = {"n.batch": 3, "batch.length": 4, "accept.rate": 0.43}
    model = "matern" if cov else "exponential"
    fit = mk.spMvGLM(formula, d["coords"], np.ones((n, q)), starting, tuning, priors, amcmc, cov_model=model, seed=9)
    pred = mk.spPredict(fit, d["coords_test"], start=start)["p.w.predictive.samples"]
    part = mk.spPredict(fit, d["coords_test"][:5], start=start + 2, end=10, thin=2)["p.w.predictive.samples"]
    # reference: one session with the kriging fused into iterations start..12
    from importlib import import_module
    sb = import_module(mk.__name__ + ".spbayes")
    cfg = sb._config(q, p, starting, tuning, priors, amcmc, model, burn_in=start, seed=9)
    q_, p_, n_, y, X, wt = sb._stack(formula, np.ones((n, q)))
    with mk.Session([dict(coords=d["coords"], y=y, weights=wt, x=X)], cfg, coords_test=d["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        ref = ses.outputs(quantiles=False, samples=True, w_pred_samples=True)
    assert np.array_equal(fit["p.beta.theta.samples"], ref["samples"][0])
    assert np.array_equal(pred, ref["w_pred_samples"][0])
    # start + 2 .. 10, every 2nd, first 5 sites: rows (site, outcome) location-major
    sub = ref["w_pred_samples"][0][:5 * q, 2:10 - start + 1:2]
    assert np.array_equal(part, sub)


@pytest.mark.parametrize("krig", ["0", "1"])
def test_sppredict_at_the_reference_amcmc_length(mk, monkeypatch, krig):
    """MK.R:83-87 as written: amcmc n.batch = 100 x batch.length = 50 (5,000 samples, every one of
    them recorded by spMvGLM for spPredict), then spPredict(start = burn.in = 3,750, end = 5,000):
    1,251 kept draws per site, equal to a session that fused the kriging into those iterations --
    bit for bit through the exact replay (MK_KRIG_CHEB=0), to 1e-8 through the default
    phi-interpolated replay, which a window this long takes (tests/test_gpu_krig_cheb.py).
    The fit's quantile grid of the 5,000 recorded samples is not needed, so no 2,048-sample cap
    applies to the recording (the quantile sort takes up to 16,384)."""
    monkeypatch.setenv("MK_KRIG_CHEB", krig)
    n, n_test = 40, 6
    d = mk.synthetic.generate(n, q=1, n_test=n_test, seed=88)
    formula = [(d["y"], d["x"])]
    starting = {"beta": np.zeros(2), "phi": 3 / 0.5, "A": np.ones(1), "w": 0.0}
    tuning = {"beta": np.full(2, 0.05), "phi": 1.0, "A": 0.1, "w": 0.5}
    priors = {"phi.Unif": (3 / 0.75, 3 / 0.25), "K.IW": (1, 0.1 * np.eye(1))}
    amcmc = {"n.batch": 100, "batch.length": 50, "accept.rate": 0.43}
    start = int(0.75 * 5000)                 # MK.R:85-87: burn.in = 0.75 n.samples, start = burn.in
    with mk.spMvGLM(formula, d["coords"], np.ones((n, 1)), starting, tuning, priors, amcmc, seed=4) as fit:
        assert fit["p.beta.theta.samples"].shape == (5000, 4)
        pred = mk.spPredict(fit, d["coords_test"], start=start)["p.w.predictive.samples"]
    assert pred.shape == (n_test, 5000 - start + 1)
    with pytest.raises(ValueError):
        mk.spPredict(fit, d["coords_test"], start=start)     # closed: the chain states are gone
    from importlib import import_module
    sb = import_module(mk.__name__ + ".spbayes")
    cfg = sb._config(1, 2, starting, tuning, priors, amcmc, "exponential", burn_in=start, seed=4)
    _, _, _, y, X, wt = sb._stack(formula, np.ones((n, 1)))
    with mk.Session([dict(coords=d["coords"], y=y, weights=wt, x=X)], cfg, coords_test=d["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        ref = ses.outputs(samples=True, w_pred_samples=True)
    assert np.array_equal(fit["p.beta.theta.samples"], ref["samples"][0])
    if krig == "0":
        assert np.array_equal(pred, ref["w_pred_samples"][0])
    else:
        np.testing.assert_allclose(pred, ref["w_pred_samples"][0], rtol=0, atol=1e-8)
    # the 1,250-sample quantile grid of the reference workflow (MK.R:88-89)
    assert np.array_equal(ref["w_predict"][0], r_quantile7(ref["w_pred_samples"][0].T, PROBS200, axis=0))
