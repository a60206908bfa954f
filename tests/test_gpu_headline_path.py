"""The headline's default code path against the oracle.

At more than 224 (subset, outcome) pairs a session takes the sequential launch schedule, the
fused 128-row column update + panel solve (k_chol_update_trsm) with the diagonal correction folded
into k_chol_diag, and the lean site sweep at n_s = 2,000 -- the path bench.py times at configs[2]
(250 subsets of 2,000, exponential, q = 1).  The short replays in test_gpu_sampler.py run 1-48
subsets, i.e. the lookahead schedule and mostly 64-row parts.  Here 225 subsets of n_s = 2,000 run 8
amcmc iterations (the last two kept, with kriging) and three of them -- the first, the middle and the
last global index -- are replayed by the oracle on the same Philox streams (MK.R:80-89): samples,
w and the kriging draws within 1e-8.
"""
import numpy as np
import pytest

from oracle import spmvglm as om

pytestmark = pytest.mark.gpu
TOL = 1e-8
S, N_S, N_TEST = 225, 2000, 40


def _data(seed=20260601):
    """S subsets of N_S sites: uniform coordinates on the unit square, an intercept and one N(0,1)
    covariate, Bernoulli(0.5) responses (the sampler's work does not depend on the field)."""
    rng = np.random.default_rng(seed)
    subs = []
    for _ in range(S):
        x = np.column_stack([np.ones(N_S), rng.standard_normal(N_S)])
        subs.append(dict(coords=rng.uniform(0.0, 1.0, (N_S, 2)), y=rng.integers(0, 2, N_S).astype(np.float64),
                         weights=np.ones(N_S), x=np.asfortranarray(x)))
    return subs, rng.uniform(0.0, 1.0, (N_TEST, 2))


def test_sequential_schedule_fused_update_matches_oracle(mk):
    subs, ct = _data()
    kw = dict(n_batch=1, batch_length=8, burn_in=7, seed=77)
    beta0, bt = np.array([0.1, -0.2]), np.array([0.05, 0.05])
    cfg = mk.SamplerConfig(1, 2, beta_starting=beta0, beta_tuning=bt, **kw)
    ocfg = om.Config(1, 2, beta_starting=beta0, beta_tuning=bt, **kw)
    with mk.Session(subs, cfg, coords_test=ct, record_w=True) as ses:
        # the schedule the library picks for > 224 pairs: sequential, so this test cannot drift onto
        # the lookahead path
        assert not ses.lookahead
        ses.profile(True)
        ses.run(cfg.n_samples)
        upd = ses.kernel_stats(mk.session.KS_CHOL_UPDATE)
        trsm = ses.kernel_stats(mk.session.KS_CHOL_TRSM)
        diag = ses.kernel_stats(mk.session.KS_CHOL_DIAG)
        dev = ses.outputs(samples=True, w_samples=True, w_pred_samples=True)
    nt = (N_S + 1 + 127) // 128
    # fused schedule: per factorisation 1 diagonal launch per column, one panel-0 trsm and nt - 2
    # fused update + solve launches (128-row form, except where the grid would be short of workgroups)
    n_fact = diag["launches"] // nt
    assert n_fact >= cfg.n_samples and diag["launches"] == n_fact * nt
    assert trsm["launches"] == n_fact
    assert upd["launches"] >= n_fact * (nt - 3) and upd["flops"] > 0
    for s in (0, S // 2, S - 1):
        sb = subs[s]
        ref = om.fit_subset(sb["coords"], sb["y"], sb["weights"], sb["x"], ocfg, subset=s, coords_test=ct,
                            record_w=True)
        np.testing.assert_allclose(dev["samples"][s], ref["samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_samples"][s].T, ref["w_samples"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_pred_samples"][s].T, ref["w_pred"], rtol=0, atol=TOL)
        np.testing.assert_allclose(dev["w_predict"][s], ref["w_q"], rtol=0, atol=TOL)
