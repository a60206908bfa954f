"""Monte Carlo-error parity at configs[1], configs[2] and configs[3] geometry against the oracle's
fixtures (tests/golden/stat/cfg2_matern.npz, cfg3_exp.npz, cfg4_lmc.npz, made by
tests/golden/stat/make_meta_fixture.py).

  cfg2_matern  Matern with nu free (U(0.1, 2)), q = 1, K = 3 subsets of n_s = 1,000 (configs[1]'s subset
               size), 1,000 amcmc iterations (20 x 50), 251 kept, 200 kriging sites
  cfg3_exp     exponential, q = 1, K = 3 subsets of n_s = 2,000 (configs[2]'s subset size), 1,000 amcmc
               iterations, 251 kept, 200 kriging sites
  cfg4_lmc     q = 3 LMC (3n x 3n cross-covariance blocks), exponential, K = 2 subsets of n_s = 500,
               1,000 iterations, 251 kept, 200 kriging sites (600 w.predict columns)

Both: R's partition after set.seed (MK.R:15-41), glm start values on the full data (MK.R:53-55),
per-subset spMvGLM + spPredict + 200 quantiles (MK.R:46-96), combine MK.R:123-133.

GPU: one session of 16 replicate meta-fits per case (replicate r = global subsets rK .. rK + K - 1, so
replicate 0 runs the oracle fixture's Philox streams and replicates 1..15 are independent chains):
  * replicate 0 replays the oracle over all 1,000 iterations (adaptation across 20 batch ends, the
    K and nu chains' drift included): samples, per-subset grids and the combined grids within 1e-6;
  * Monte Carlo-error parity against INDEPENDENT oracle chains: tests/golden/stat/<case>_indep.npz
    (tests/golden/stat/make_indep_replicates.py) holds R_O more oracle meta-fits of the same data on
    global subsets 1,000 + rK .. -- streams no device replicate runs; R_O = 12 for cfg3_exp and
    cfg4_lmc, 4 for cfg2_matern -- and their combined grids are compared with the device's replicates
    1..15 by a two-sample t statistic per (column, level),
    t = (mean_oracle - mean_device) / (s_pooled sqrt(1/R_O + 1/15)), R_O + 13 df: every parameter
    |t| <= 5; over the w.predict (site, level) pairs at most 3 % with |t| > 3.5 and mean t^2 in
    [0.5, 2].  Detectable shift: |t| > 5 needs a mean shift of 5 sqrt(1/12 + 1/15) = 1.94 replicate
    standard deviations at R_O = 12 (2.9 at R_O = 4); a negative control (phi.Unif's upper bound
    12 -> 10 on the device only) must fail the same criteria.
    (Round 4 compared the oracle's own fixture with replicates 1..15 -- but that fixture IS replicate
    0's chain, so the test measured the device's spread against itself.)
CPU: the fixtures' own consistency (inputs regenerate, the combine is the sequential mean, the
independent replicates are distinct chains of the same fit).
The fixtures pin the device to the build's oracle, not to spBayes (absent); the oracle
itself is pinned to the model by tests/test_geweke.py.
"""
import importlib
import os

import numpy as np
import pytest

from oracle import spmvglm as om

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"
CASES = ("cfg2_matern", "cfg3_exp", "cfg4_lmc")
LEVELS3 = (4, 99, 194)
R_REP = 16
# the negative controls' perturbed targets (_perturbed): phi.Unif's upper bound 12 -> 8 (cfg4_lmc) or
# -> 6.5 (cfg3_exp; the starting value 6 must stay inside).  tools/mc_power.py (profiles/r06/mc_power_*.jsonl) measured the criteria's power:
# phi -> 10 and K.IW's scale x 2 pass at both geometries; cfg4_lmc also fails phi -> 8 (max |t| 8.9)
# and K.IW x 10 (w.predict mean t^2 3.1); cfg3_exp passes phi -> 8 and K.IW x 10 -- its 1,000-
# iteration chains of a weakly identified phi spread too widely between replicates
NEG_CONTROL = {"cfg3_exp": ("phi_b", 6.5), "cfg4_lmc": ("phi_b", 8.0)}


def _load(case):
    z = np.load(os.path.join(HERE, "golden", "stat", case + ".npz"))   # allow_pickle=False (default): data only
    return {k: z[k] for k in z.files}


def _subsets(g):
    q = int(g["q"])
    offs = np.concatenate([[0], np.cumsum(g["n_part"])])
    out = []
    for s in range(int(g["K"])):
        idx = g["index"][offs[s]:offs[s + 1]].astype(np.int64) - 1
        rows = (idx[:, None] * q + np.arange(q)[None, :]).reshape(-1)
        out.append(dict(coords=g["coords"][idx], y=g["y"][rows], weights=np.ones(rows.size), x=g["x"][rows]))
    return out


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("case", CASES)
def test_fixture_inputs_regenerate(case):
    """The stored inputs are the SURVEY.md 8d generator's draw, R's partition and the glm.fit start
    values (guards against generator or oracle drift)."""
    from oracle import rrng, rstats
    syn = importlib.import_module(PKG + ".synthetic")
    g = _load(case)
    n, q = int(g["n"]), int(g["q"])
    d = syn.generate(n, q=q, n_test=int(g["n_test"]), cov_model=int(g["cov_model"]), seed=int(g["seed"]))
    for k in ("coords", "y", "x", "coords_test", "x_test"):
        assert np.array_equal(d[k], g[k]), k
    # the exact GP draw goes through a BLAS Cholesky: its last bits follow the BLAS thread count
    np.testing.assert_allclose(d["w_test_true"], g["w_test_true"], rtol=1e-9, atol=1e-12)
    n_part, idx = rrng.partition(n, int(g["K"]), int(g["seed"]))
    assert np.array_equal(n_part, g["n_part"])
    assert np.array_equal(np.concatenate(idx), g["index"])
    coef, _ = rstats.glm_binomial(g["y"], g["x"], np.ones(g["y"].size))
    np.testing.assert_allclose(coef, g["beta_starting"], rtol=1e-12)


@pytest.mark.parametrize("case", CASES)
def test_fixture_combine_is_the_sequential_mean(case):
    g = _load(case)
    assert np.array_equal(om.combine_mean(list(g["param_q"])), g["result"])
    assert g["result2"].shape == (200, int(g["q"]) * int(g["n_test"]))
    # the slope of every outcome is covered by its combined 99 % interval (truth recovery; at 1,000
    # iterations the Matern fixture's 95 % interval ends at -0.986 for a true -1)
    q = int(g["q"])
    for a in range(q):
        j = 2 * a + 1
        assert g["result"][0, j] <= g["beta_true"][j] <= g["result"][198, j], (a, g["result"][[0, 198], j])


# ------------------------------------------------------------------ GPU
_cache = {}


def _perturbed(q, which):
    """SamplerConfig overrides of a perturbed target (negative controls): phi.Unif's upper bound
    (MK.R:63's 3/0.25 = 12) -> b, or K.IW's scale matrix (MK.R:64's 0.1 I) -> s I."""
    kind, v = which
    if kind == "phi_b":
        return {"phi_unif": (np.full(q, 3.0 / 0.75), np.full(q, float(v)))}
    if kind == "iw_s":
        return {"K_IW_S": float(v) * np.eye(q)}
    raise ValueError(kind)


def _device_replicates(mk, case, perturb=None):
    """R_REP device meta-fits of the case in one session; perturb = (kind, value) samples another
    target (negative controls only, _perturbed)."""
    key = (case, perturb)
    if key in _cache:
        return _cache[key]
    g = _load(case)
    subs = _subsets(g)
    K, q = int(g["K"]), int(g["q"])
    kw = {} if perturb is None else _perturbed(q, perturb)
    cfg = mk.SamplerConfig(q, 2 * q, g["beta_starting"], g["beta_tuning"],
                           cov_model="matern" if int(g["cov_model"]) == 1 else "exponential",
                           n_batch=int(g["n_batch"]), batch_length=int(g["batch_length"]), seed=int(g["seed"]), **kw)
    with mk.Session(subs * R_REP, cfg, coords_test=g["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        out = ses.outputs(samples=True)
    res = np.stack([mk.combine(out["parameters"][r * K:(r + 1) * K]) for r in range(R_REP)])
    res2 = np.stack([mk.combine(out["w_predict"][r * K:(r + 1) * K]) for r in range(R_REP)])
    _cache[key] = (g, out, res, res2)
    return _cache[key]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_replica0_replays_oracle(mk, case):
    g, out, res, res2 = _device_replicates(mk, case)
    for s in range(int(g["K"])):
        np.testing.assert_allclose(out["samples"][s], g["samples"][s], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out["parameters"][s], g["param_q"][s], rtol=0, atol=1e-6)
        np.testing.assert_allclose(out["w_predict"][s][list(LEVELS3)], g["w_q3"][s], rtol=0, atol=1e-6)
    np.testing.assert_allclose(res[0], g["result"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(res2[0], g["result2"], rtol=0, atol=1e-6)


def _load_indep(case):
    z = np.load(os.path.join(HERE, "golden", "stat", case + "_indep.npz"))   # allow_pickle=False (default)
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("case", CASES)
def test_independent_oracle_replicates_are_distinct_chains(case):
    """The independent oracle replicates run other Philox streams than the fixture (replicate 0's):
    same data and start values, different chains, similar answers."""
    g, ind = _load(case), _load_indep(case)
    assert int(ind["base"]) >= R_REP * int(g["K"])            # no device replicate's streams
    assert ind["result"].shape == (int(ind["R_O"]), 200, g["result"].shape[1])
    assert ind["result2_3"].shape == (int(ind["R_O"]), len(LEVELS3), g["result2"].shape[1])
    for r in range(int(ind["R_O"])):
        assert not np.array_equal(ind["result"][r], g["result"])
    # the regression coefficients' medians within a loose band of the fixture's (a gross drift check, not
    # the MC test; phi is weakly identified at 1,000 iterations and its chains' medians spread widely)
    p = 2 * int(g["q"])
    assert np.all(np.abs(ind["result"][:, 99, :p] - g["result"][99, :p]) < 0.5)


def _t2(a, b):
    """Two-sample t (pooled variance) of the replicate means, per element: a [n_a, ...], b [n_b, ...]."""
    na, nb = a.shape[0], b.shape[0]
    sp2 = ((na - 1) * a.var(axis=0, ddof=1) + (nb - 1) * b.var(axis=0, ddof=1)) / (na + nb - 2)
    se = np.sqrt(sp2 * (1.0 / na + 1.0 / nb))
    return (a.mean(axis=0) - b.mean(axis=0)) / np.where(se > 0, se, np.inf)


def _mc_criteria(ind, res, res2):
    """The MC-error criteria on the device's replicates 1..15 against the independent oracle
    replicates: (every parameter |t| <= 5, share of w.predict |t| > 3.5 <= 3 %, mean t^2 in [0.5, 2]),
    each as a bool, plus the statistics."""
    L = list(LEVELS3)
    tp = _t2(ind["result"][:, L], res[1:, L])            # 3 levels x P parameters
    tw = _t2(ind["result2_3"], res2[1:, L])              # 3 levels x q n_test columns
    frac, mt2 = float(np.mean(np.abs(tw) > 3.5)), float(np.mean(tw ** 2))
    return (bool(np.all(np.abs(tp) <= 5.0)), frac <= 0.03, 0.5 <= mt2 <= 2.0), (tp, frac, mt2)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_independent_oracle_chains_within_mc_error_of_device(mk, case):
    g, _, res, res2 = _device_replicates(mk, case)
    ok, (tp, frac, mt2) = _mc_criteria(_load_indep(case), res, res2)
    assert ok[0], tp
    assert ok[1], frac
    assert ok[2], mt2


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["cfg3_exp", "cfg4_lmc"])
def test_mc_parity_detects_a_perturbed_phi_prior(mk, case):
    """Negative control: the same criteria must FAIL when the device samples
    another target -- phi.Unif's upper bound 12 -> NEG_CONTROL[case] (MK.R:63) -- against the
    unperturbed oracle replicates (12 of them for these cases)."""
    _, _, res, res2 = _device_replicates(mk, case, perturb=NEG_CONTROL[case])
    ok, (tp, frac, mt2) = _mc_criteria(_load_indep(case), res, res2)
    assert not all(ok), (np.round(tp, 2), frac, mt2)
