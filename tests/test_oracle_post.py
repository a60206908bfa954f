"""Pin oracle/post.py (CPU): the MK.R:136-165 restatement against independent numpy code,
and the Weiszfeld combine spec against its defining properties (it has no reference: the
reference averages, MK.R:123-133 -- parity for the median is against this spec only)."""
import numpy as np
import pytest
from scipy.optimize import minimize

from oracle import post, rstats
from oracle.spmvglm import combine_mean


def _grids(K, L=200, C=5, seed=0):
    rng = np.random.default_rng(seed)
    return np.stack([np.sort(rng.normal(loc=rng.normal(), size=(L, C)), axis=0) for _ in range(K)])


def test_resample_index_uniform_over_996_levels():
    idx = post.resample_index(200000, seed=3)
    assert idx.min() == 0 and idx.max() == 995
    counts = np.bincount(idx, minlength=996)
    assert abs(counts.mean() - 200000 / 996) < 1e-9 and counts.std() < 4 * np.sqrt(200000 / 996)
    assert np.array_equal(post.resample_index(50, 3), idx[:50])     # a counter stream: prefix-stable


def test_posterior_summary_matches_independent_numpy():
    g = _grids(1, C=9, seed=1)[0]
    res, res2 = g[:, :4], g[:, 4:]
    x_test = np.column_stack([np.ones(5), np.linspace(-1, 1, 5), np.zeros(5)])
    out = post.posterior_summary(res, res2, x_test, samplesize=1000, seed=7)
    idx = out["index"]
    interp = lambda y: np.stack([np.interp(rstats.XOUT996, rstats.PROBS200, y[:, c])   # noqa: E731
                                 for c in range(y.shape[1])], axis=1)
    np.testing.assert_allclose(out["SamplePar"], interp(res)[idx], rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(out["Samplew"], interp(res2)[idx], rtol=1e-14, atol=1e-14)
    eta = out["SamplePar"][:, :3] @ x_test.T + out["Samplew"]
    np.testing.assert_allclose(out["p_sample"], 1.0 / (1.0 + np.exp(-eta)), rtol=1e-13)
    probs = [0.5, 0.025, 0.975]
    np.testing.assert_allclose(out["w_quant"], np.quantile(out["Samplew"], probs, axis=0), rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(out["param_quant"], np.quantile(out["SamplePar"], probs, axis=0), rtol=1e-14,
                               atol=1e-15)
    assert out["w_quant"].shape == (3, 5) and out["param_quant"].shape == (3, 4)


def test_weiszfeld_identical_grids_is_fixed_point():
    g = np.repeat(_grids(1, seed=2), 6, axis=0)
    med, it = post.weiszfeld_median(g)
    np.testing.assert_allclose(med, g[0], rtol=1e-15, atol=1e-15)
    assert it.max() <= 2


def test_weiszfeld_scalar_case_is_the_median():
    vals = np.array([0.3, -1.2, 5.0, 0.9, 0.1, 40.0, -0.4])    # odd K: the geometric median is the middle value
    med, _ = post.weiszfeld_median(vals.reshape(-1, 1, 1), max_iter=2000, tol=1e-15)
    assert abs(med[0, 0] - np.median(vals)) < 1e-8


def test_weiszfeld_minimises_sum_of_w2_distances():
    g = _grids(7, L=20, C=1, seed=4)[:, :, 0]
    med, _ = post.weiszfeld_median(g[:, :, None], max_iter=500, tol=1e-14)
    f = lambda y: np.sum(np.sqrt(np.mean((g - y[None]) ** 2, axis=1)))    # noqa: E731
    ref = minimize(f, g.mean(0), method="BFGS", options=dict(gtol=1e-12, maxiter=10000)).x
    assert f(med[:, 0]) <= f(ref) + 1e-10
    np.testing.assert_allclose(med[:, 0], ref, atol=1e-5)


def test_weiszfeld_is_robust_and_monotone():
    g = _grids(9, seed=5)
    bad = g.copy()
    bad[0] = bad[0] + 50.0                         # one corrupted subset posterior
    med, _ = post.weiszfeld_median(bad)
    clean, _ = post.weiszfeld_median(g)
    mean_shift = np.abs(combine_mean(list(bad)) - combine_mean(list(g))).max()
    assert np.abs(med - clean).max() < 0.2 * mean_shift
    assert np.all(np.diff(med, axis=0) >= -1e-12)  # still a quantile function


@pytest.mark.parametrize("K", [1, 2, 5])
def test_weiszfeld_small_K(K):
    g = _grids(K, C=3, seed=6)
    med, it = post.weiszfeld_median(g)
    assert med.shape == (200, 3) and np.all(np.isfinite(med)) and it.min() >= 1
    if K <= 2:                                     # any point of the segment is a median; we stay at the mean
        np.testing.assert_allclose(med, combine_mean(list(g)), rtol=1e-12, atol=1e-12)


def test_posterior_summary_r_index_and_probit():
    """A caller-given (R-stream) 1-based sampleparIndex is used as is; link="probit" gives
    p(y=1) = Phi(eta) (extension; MK.R:160 is logistic)."""
    from scipy.special import ndtr
    from oracle.rrng import RRng
    g = _grids(1, C=7, seed=4)[0]
    res, res2 = g[:, :4], g[:, 4:]
    x_test = np.column_stack([np.ones(3), np.linspace(-1, 1, 3)])
    idx1 = RRng(20250114).sample_int_replace(996, 800)
    out = post.posterior_summary(res, res2, x_test, samplesize=800, index=idx1, link="probit")
    assert np.array_equal(out["index"], np.asarray(idx1) - 1)
    interp = lambda y: np.stack([np.interp(rstats.XOUT996, rstats.PROBS200, y[:, c])   # noqa: E731
                                 for c in range(y.shape[1])], axis=1)
    np.testing.assert_allclose(out["SamplePar"], interp(res)[np.asarray(idx1) - 1], rtol=1e-14, atol=1e-14)
    eta = out["SamplePar"][:, :2] @ x_test.T + out["Samplew"]
    np.testing.assert_allclose(out["p_sample"], ndtr(eta), rtol=1e-14)
