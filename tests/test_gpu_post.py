"""Device post-processing, median combine, glm start values and stream grouping, through
the C ABI, against the CPU oracle.

* posterior_summary (MK.R:136-165): resample index and interpolated draws bit-exact;
  p(y=1) within 1e-14 relative (device vs libm exp); summaries of identical draws bit-exact.
* combine_median (Weiszfeld, extension): within 1e-9 of oracle/post.py (reduction order differs).
* glm start values (MK.R:53-55): coefficients 1e-10, vcov 1e-8 relative to the QR-based oracle.
* n_streams: the chains are independent of how subsets are grouped onto streams (bit-exact)."""
import numpy as np
import pytest

from oracle import post, rstats

pytestmark = pytest.mark.gpu


def _grids(K, L=200, C=5, seed=0):
    rng = np.random.default_rng(seed)
    return np.stack([np.sort(rng.normal(loc=rng.normal(), size=(L, C)), axis=0) for _ in range(K)])


@pytest.mark.parametrize("C,p,S", [(7, 2, 1000), (1, 4, 17), (300, 6, 2048)])
def test_posterior_summary_matches_oracle(mk, C, p, S):
    P = max(4, p + 2)
    g = _grids(1, C=P + C, seed=C)[0]
    res, res2 = g[:, :P], g[:, P:P + C]
    x_test = np.random.default_rng(1).normal(size=(C, p))
    dev = mk.posterior_summary(res, res2, x_test, samplesize=S, seed=11)
    ref = post.posterior_summary(res, res2, x_test, samplesize=S, seed=11)
    assert np.array_equal(dev["index"], ref["index"])
    assert np.array_equal(dev["SamplePar"], ref["SamplePar"])
    assert np.array_equal(dev["Samplew"], ref["Samplew"])
    np.testing.assert_allclose(dev["p_sample"], ref["p_sample"], rtol=1e-14, atol=0)
    assert np.array_equal(dev["w_quant"], ref["w_quant"])
    assert np.array_equal(dev["param_quant"], ref["param_quant"])
    np.testing.assert_allclose(dev["p_quant"], ref["p_quant"], rtol=1e-14, atol=0)


@pytest.mark.parametrize("link", ["logit", "probit"])
def test_posterior_summary_r_stream_index(mk, link):
    """MK.R:141 on R's stream: rng="R" draws sampleparIndex as sample(seq(1, 996, 1), S, replace=TRUE)
    right after set.seed(seed) (mk_r_sample_replace); the summaries then match the oracle given
    R's index.  link="probit": p(y=1) = Phi(eta)."""
    from oracle.rrng import RRng
    C, p, S, seed = 40, 2, 1000, 20250114
    g = _grids(1, C=4 + C, seed=3)[0]
    res, res2 = g[:, :4], g[:, 4:]
    x_test = np.random.default_rng(2).normal(size=(C, p))
    dev = mk.posterior_summary(res, res2, x_test, samplesize=S, seed=seed, rng="R", link=link)
    r_idx = RRng(seed).sample_int_replace(996, S)
    ref = post.posterior_summary(res, res2, x_test, samplesize=S, index=r_idx, link=link)
    assert np.array_equal(dev["index"], np.asarray(r_idx) - 1)
    assert np.array_equal(dev["SamplePar"], ref["SamplePar"])
    assert np.array_equal(dev["Samplew"], ref["Samplew"])
    np.testing.assert_allclose(dev["p_sample"], ref["p_sample"], rtol=1e-14, atol=1e-300)
    assert np.array_equal(dev["w_quant"], ref["w_quant"])
    dev2 = mk.posterior_summary(res, res2, x_test, samplesize=S, index=r_idx, link=link)
    assert np.array_equal(dev2["SamplePar"], dev["SamplePar"])


def test_posterior_summary_parameters_only(mk):
    res = _grids(1, C=3, seed=9)[0]
    dev = mk.posterior_summary(res, None, None, samplesize=500, seed=2)
    ref = post.posterior_summary(res, np.zeros((200, 1)), np.zeros((1, 0)), samplesize=500, seed=2)
    assert np.array_equal(dev["SamplePar"], ref["SamplePar"])
    assert np.array_equal(dev["param_quant"], ref["param_quant"])


@pytest.mark.parametrize("K,L,C", [(9, 200, 11), (1, 200, 3), (2, 200, 4), (250, 200, 33), (5, 256, 2), (3, 17, 5)])
def test_combine_median_matches_oracle(mk, K, L, C):
    g = _grids(K, L=L, C=C, seed=K + C)
    if K > 3:
        g[0] += 20.0                               # an outlying subset
    med, it = mk.combine_median(list(g))
    ref, rit = post.weiszfeld_median(g)
    np.testing.assert_allclose(med, ref, rtol=0, atol=1e-9 * (1 + np.abs(ref).max()))
    assert np.all(np.abs(it - rit) <= 1)


def test_combine_median_rejects_bad_levels(mk):
    with pytest.raises(mk.MkError):
        mk.combine_median(list(_grids(3, L=300, C=2)))


@pytest.mark.parametrize("q,n", [(1, 20000), (2, 6000)])
def test_glm_start_values_match_oracle(mk, q, n):
    d = mk.synthetic.generate(n, q=q, n_test=0, seed=8)
    coef, vcov, bt = mk.glm_binomial(d["y"], d["x"], np.ones(n * q))
    rc, rv = rstats.glm_binomial(d["y"], d["x"], np.ones(n * q))
    np.testing.assert_allclose(coef, rc, rtol=1e-10)
    np.testing.assert_allclose(vcov, rv, rtol=1e-8)
    np.testing.assert_allclose(bt @ bt.T, vcov, rtol=1e-12)        # t(chol(vcov)) is lower


@pytest.mark.parametrize("q,n", [(1, 20000), (2, 6000)])
def test_glm_probit_start_values_match_oracle(mk, q, n):
    """binomial(link = "probit") IRLS (extension's start values) vs the QR oracle."""
    d = mk.synthetic.generate(n, q=q, n_test=0, seed=9, link="probit")
    coef, vcov, bt = mk.glm_binomial(d["y"], d["x"], np.ones(n * q), link="probit")
    rc, rv = rstats.glm_binomial(d["y"], d["x"], np.ones(n * q), link="probit")
    np.testing.assert_allclose(coef, rc, rtol=1e-10)
    np.testing.assert_allclose(vcov, rv, rtol=1e-8)


def test_glm_binomial_trials(mk):
    """weights > 1: glm((y/weight) ~ x - 1, weights = weight) on counts."""
    rng = np.random.default_rng(3)
    n = 4000
    x = np.column_stack([np.ones(n), rng.normal(size=n)])
    wt = rng.integers(1, 6, size=n).astype(float)
    y = rng.binomial(wt.astype(int), 1 / (1 + np.exp(-(0.3 - 0.8 * x[:, 1])))).astype(float)
    coef, vcov, _ = mk.glm_binomial(y, x, wt)
    rc, rv = rstats.glm_binomial(y / wt, x, wt)
    np.testing.assert_allclose(coef, rc, rtol=1e-10)
    np.testing.assert_allclose(vcov, rv, rtol=1e-8)


def test_stream_grouping_does_not_change_the_chains(mk):
    """Subset groups on several HIP streams give the one-stream chains bit for bit (sequential
    schedule: the lookahead schedule needs one group; its own equivalence is tested in
    test_gpu_sampler.py)."""
    d = mk.synthetic.generate(5 * 90, q=1, n_test=6, seed=21)
    subs = [dict(coords=d["coords"][i * 90:(i + 1) * 90], y=d["y"][i * 90:(i + 1) * 90], weights=np.ones(90),
                 x=d["x"][i * 90:(i + 1) * 90]) for i in range(5)]
    outs = []
    for ns in (1, 2, 3, 5):
        cfg = mk.SamplerConfig(1, 2, [0, 0], [0.05, 0.05], n_batch=2, batch_length=5, burn_in=6, seed=4, n_streams=ns)
        with mk.Session(subs, cfg, coords_test=d["coords_test"], lookahead=0 if ns == 1 else None) as ses:
            assert not ses.lookahead
            ses.run(cfg.n_samples)
            outs.append(ses.outputs(samples=True, w_pred_samples=True))
    for o in outs[1:]:
        for s in range(5):
            assert np.array_equal(o["samples"][s], outs[0]["samples"][s])
            assert np.array_equal(o["w_pred_samples"][s], outs[0]["w_pred_samples"][s])
            assert np.array_equal(o["w_predict"][s], outs[0]["w_predict"][s])


def test_torch_first_process_rccl_combine(mk):
    """Multi-GPU launch order (torch's HIP runtime + an RCCL group initialised before libmk loads,
    as bench.py / run_metakriging.py do under torch.distributed.run), in a fresh process: a chain
    replays the oracle and the device-resident column-sharded combine -- mean, sum, Weiszfeld
    median, rank-ordered partial sums -- matches the CPU restatements (MK.R:123-133)."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "gpu_torch_first.py")], capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert json.loads(lines[-1])["ok"]
