"""Error paths of the C ABI on a GPU: a failing mk_session_create frees the session and every
device buffer it had allocated (no leaked handle, device memory back to its level), and the
library keeps working afterwards."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_bytes(mk):
    import ctypes
    f, t = ctypes.c_int64(), ctypes.c_int64()
    mk._lib.check(mk.load().mk_device_memory(0, ctypes.byref(f), ctypes.byref(t)))
    return f.value


def test_failed_create_leaves_nothing_behind(mk):
    lib = mk.load()
    base = lib.mk_session_count()
    n = 200_000        # one subset: its two factor slots alone need 2 x 200064^2 x 8 B = 640 GB > HBM
    d = mk.synthetic.generate(n, q=1, n_test=0, seed=1, exact_max=0)
    cfg = mk.SamplerConfig(1, 2, [0, 0], [0.1, 0.1], n_batch=1, batch_length=2)
    sub = dict(coords=d["coords"], y=d["y"], weights=np.ones(n), x=d["x"])
    small = dict(coords=d["coords"][:50], y=d["y"][:50], weights=np.ones(50), x=d["x"][:50])
    with mk.Session([small], cfg) as ses:      # warm the context so the baseline is steady
        ses.run(1)
    free0 = _free_bytes(mk)
    for _ in range(3):
        with pytest.raises(mk.MkError) as e:
            mk.Session([sub], cfg)
        assert e.value.code == mk._lib.MK_E_NOMEM
        assert lib.mk_session_count() == base
    assert abs(_free_bytes(mk) - free0) < 64 << 20           # the partial allocations were freed
    with mk.Session([small], cfg) as ses:
        assert lib.mk_session_count() == base + 1
        ses.run(2)
    assert lib.mk_session_count() == base


def test_bad_config_after_device_checks_frees_session(mk):
    lib = mk.load()
    base = lib.mk_session_count()
    d = mk.synthetic.generate(60, q=1, n_test=0, seed=2)
    sub = dict(coords=d["coords"], y=d["y"], weights=np.ones(60), x=d["x"])
    cfg = mk.SamplerConfig(1, 2, [0, 0], [0.1, 0.1], n_batch=1, batch_length=2)
    cfg.beta_tuning = np.array([0.1, -1.0])           # rejected after the allocations
    with pytest.raises(mk.MkError):
        mk.Session([sub], cfg)
    assert lib.mk_session_count() == base


def test_profile_every_samples_iterations_and_keeps_the_chain(mk):
    """mk_session_profile_every (bench.py's sampled roofline events): bracketing the launches of every
    k-th iteration only times a subset of the launches -- in proportion -- and, like any profiling, leaves
    the chain unchanged; the inverse's flops follow the device-side count of accepted factors."""
    d = mk.synthetic.generate(900, q=1, n_test=0, seed=4)
    cfg = mk.SamplerConfig(1, 2, [0.0, 0.0], [0.05, 0.05], n_batch=1, batch_length=12, seed=8)
    subs = [dict(coords=d["coords"][i * 300:(i + 1) * 300], y=d["y"][i * 300:(i + 1) * 300], weights=np.ones(300),
                 x=d["x"][i * 300:(i + 1) * 300]) for i in range(3)]
    res = {}
    for every in (0, 1, 4):
        with mk.Session(subs, cfg, lookahead=False) as ses:
            if every:
                ses.profile(True, every=every)
            ses.run(cfg.n_samples)
            res[every] = (ses.kernel_stats(mk.session.KS_CHOL_DIAG)["launches"], ses.kernel_stats(mk.session.KS_INV),
                          ses.outputs(quantiles=False, samples=True)["samples"])
    assert np.array_equal(res[1][2], res[0][2]) and np.array_equal(res[4][2], res[0][2])
    assert res[0][0] == 0
    # iterations 0, 4, 8 of 12: a quarter of the diagonal launches
    assert res[4][0] * 4 == res[1][0]
    inv = res[1][1]
    assert inv["launches"] > 0 and inv["flops"] > 0 and inv["ms"] > 0
