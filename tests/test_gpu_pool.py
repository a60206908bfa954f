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
