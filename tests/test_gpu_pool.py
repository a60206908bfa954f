"""libmk's stream pool (mk_api.hip pool_stream): sessions take their HIP streams -- the plain ones,
the lookahead schedule's high-priority candidate stream and its CU-masked main stream, the split
Cholesky's CU-masked bulk stream -- from a per-process pool and hand them back drained.  Many short
sessions in a row (a test suite's pattern) must each replay the same chain on reused streams."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_sessions_in_a_row_reuse_pooled_streams(mk):
    d = mk.synthetic.generate(150, q=1, n_test=6, seed=31)
    sub = dict(coords=d["coords"], y=d["y"], weights=np.ones(150), x=d["x"])
    cfg = mk.SamplerConfig(1, 2, beta_starting=[0.2, -0.2], beta_tuning=[0.05, 0.05], n_batch=2, batch_length=4,
                           burn_in=5, seed=9)
    ref = None
    for i in range(40):
        with mk.Session([sub], cfg, coords_test=d["coords_test"]) as ses:
            ses.run(cfg.n_samples)
            out = ses.outputs(samples=True)
        if ref is None:
            ref = out
            continue
        assert np.array_equal(out["samples"][0], ref["samples"][0]), i
        assert np.array_equal(out["w_predict"][0], ref["w_predict"][0]), i
    assert mk.load().mk_session_count() == 0


def test_alternating_configurations_evict_idle_streams(mk):
    """Sessions of two shard sizes in turn: the split Cholesky's CU-masked bulk streams differ (reserve 8
    vs 16 CUs), so each new configuration finds no exact match and the pool drops its idle streams
    before creating queues (MK_POOL_CAP, default 1: idle queues of another configuration serialised
    the next session's streams).  Every session replays its configuration's chain."""
    d = mk.synthetic.generate(9 * 400, q=1, n_test=6, seed=33)
    subs = [dict(coords=d["coords"][400 * i:400 * (i + 1)], y=d["y"][400 * i:400 * (i + 1)], weights=np.ones(400),
                 x=d["x"][400 * i:400 * (i + 1)]) for i in range(9)]
    cfg = mk.SamplerConfig(1, 2, beta_starting=[0.2, -0.2], beta_tuning=[0.05, 0.05], n_batch=2, batch_length=3,
                           burn_in=4, seed=11)
    refs = {}
    for i in range(6):
        S = 1 if i % 2 == 0 else 9
        with mk.Session(subs[:S], cfg, coords_test=d["coords_test"]) as ses:
            ses.run(cfg.n_samples)
            out = ses.outputs(samples=True)
        if S not in refs:
            refs[S] = out
            continue
        for s in range(S):
            assert np.array_equal(out["samples"][s], refs[S]["samples"][s]), (i, s)
    # subset 0 runs the same chain (its own Philox streams) in both configurations, up to rounding
    np.testing.assert_allclose(refs[1]["samples"][0], refs[9]["samples"][0], rtol=0, atol=1e-9)
    assert mk.load().mk_session_count() == 0
