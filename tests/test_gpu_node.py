"""mk_meta_fit: the whole node behind the C ABI (MK.R:100-133 without a cluster).

One device through RCCL (a communicator of one: pack, grouped send/recv, combine on the
receive buffer) and several "virtual" blocks on one device (the device-copy exchange, SURVEY.md
4 item 5) must give bit for bit what one session + the sequential combine gives: the same
chains (global subset indices), the same 200-level grids, MK.R:123-133's mean in its summation
order, and the Weiszfeld median per column.  Tiled kriging (configs[4]'s path) exchanges one
test-site tile at a time.  The progress callback between batches can stop the fit cleanly."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _library_default_exchange(monkeypatch):
    """The node tests run the library's default exchange in the pytest process: RCCL for a list of
    distinct devices (here a communicator of one), device copies where a device is listed more than
    once.  A communicator that cannot be created fails the call (MK_E_HIP) -- there is no silent
    fallback to copies any more (round 3 forced MK_EXCHANGE=copy here and hid exactly that)."""
    monkeypatch.delenv("MK_EXCHANGE", raising=False)


def _problem(mk, sizes, q=1, n_test=9, seed=3, cov=0):
    d = mk.synthetic.generate(sum(sizes), q=q, n_test=n_test, seed=seed, cov_model=cov)
    subs, off = [], 0
    for m in sizes:
        rows = slice(off * q, (off + m) * q)
        subs.append(dict(coords=d["coords"][off:off + m], y=d["y"][rows], weights=np.ones(m * q), x=d["x"][rows]))
        off += m
    return subs, d["coords_test"]


def _cfg(mk, q=1, cov=0, predict_tile=0, n_batch=3, batch_length=3, burn_in=5):
    p = 2 * q
    return mk.SamplerConfig(q, p, np.zeros(p), np.full(p, 0.05), cov_model="matern" if cov else "exponential",
                            n_batch=n_batch, batch_length=batch_length, burn_in=burn_in, seed=17,
                            predict_tile=predict_tile)


def _session_reference(mk, subs, cfg, ct, base=0):
    with mk.Session(subs, cfg, coords_test=ct, subset_base=base, record_w=True) as ses:
        ses.run(cfg.n_samples)
        return ses.outputs(samples=True, w_samples=True, w_pred_samples=True, acceptance=True, w_predict_sum=True)


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_node_equals_one_session_and_sequential_combine(mk, devices):
    subs, ct = _problem(mk, [150, 163, 127, 140, 90])
    cfg = _cfg(mk)
    ref = _session_reference(mk, subs, cfg, ct, base=2)
    got = mk.meta_fit_node(subs, cfg, coords_test=ct, devices=devices, subset_base=2, samples=True, w_samples=True,
                           w_pred_samples=True, acceptance=True, w_predict_sum=True)
    assert got["exchange"] == ("copy" if len(devices) > 1 else "rccl")
    for k in ("parameters", "w_predict", "samples", "w_samples", "w_pred_samples", "acceptance"):
        for s in range(len(subs)):
            assert np.array_equal(got[k][s], ref[k][s]), (k, s)
    assert np.array_equal(got["w_predict_sum"], ref["w_predict_sum"])
    assert np.array_equal(got["result"], mk.combine(ref["parameters"]))
    assert np.array_equal(got["result2"], mk.combine(ref["w_predict"]))


def test_node_blocks_more_than_subsets_and_multi_outcome(mk):
    """K = 2 subsets over 3 blocks (one block holds none and still owns columns of the combine);
    q = 2 LMC grids."""
    subs, ct = _problem(mk, [70, 64], q=2, n_test=5, seed=8)
    cfg = _cfg(mk, q=2)
    ref = _session_reference(mk, subs, cfg, ct)
    got = mk.meta_fit_node(subs, cfg, coords_test=ct, devices=[0, 0, 0])
    assert np.array_equal(got["result"], mk.combine(ref["parameters"]))
    assert np.array_equal(got["result2"], mk.combine(ref["w_predict"]))


def test_node_tiled_kriging_and_median_combine(mk):
    """Tiled kriging (a full tile of 7 sites and a ragged one) exchanged tile by tile over two
    blocks, combined by the Weiszfeld W2 median (north-star extension) and by the mean."""
    subs, ct = _problem(mk, [120, 100, 111], n_test=12, seed=5)
    cfg = _cfg(mk, predict_tile=7)
    ref = _session_reference(mk, subs, cfg, ct)
    med = mk.meta_fit_node(subs, cfg, coords_test=ct, devices=[0, 0], method="median", w_predict_sum=True)
    assert np.array_equal(med["w_predict_sum"], ref["w_predict_sum"])
    for s in range(len(subs)):
        assert np.array_equal(med["w_predict"][s], ref["w_predict"][s])
    exp2, _ = mk.combine_median(ref["w_predict"])
    exp1, _ = mk.combine_median(ref["parameters"])
    np.testing.assert_allclose(med["result2"], exp2, rtol=0, atol=1e-12)
    np.testing.assert_allclose(med["result"], exp1, rtol=0, atol=1e-12)
    mean = mk.meta_fit_node(subs, cfg, coords_test=ct, devices=[0, 0], per_subset=False)
    assert np.array_equal(mean["result2"], mk.combine(ref["w_predict"]))


def test_node_progress_and_interrupt(mk):
    """The callback sees every batch boundary; returning True stops the fit with
    MK_E_INTERRUPT and frees every session (R: the user interrupt between batches)."""
    subs, ct = _problem(mk, [60, 50])
    cfg = _cfg(mk, n_batch=4, batch_length=2, burn_in=5)
    seen = []
    mk.meta_fit_node(subs, cfg, coords_test=ct, devices=[0, 0], progress=lambda it, n: seen.append((it, n)) and False)
    assert seen == [(2, 8), (4, 8), (6, 8), (8, 8)]
    with pytest.raises(mk.MkError) as e:
        mk.meta_fit_node(subs, cfg, coords_test=ct, devices=[0], progress=lambda it, n: it >= 4)
    assert e.value.code == -5
    assert mk.load().mk_session_count() == 0


def test_session_tile_grids_equal_the_whole_grids(mk):
    """mk_session_tile_grids: one tile's kriging replay gives exactly the columns of the tiled
    session's whole w.predict grids (the per-tile combine of configs[4] reads these)."""
    subs, ct = _problem(mk, [90, 80], n_test=10, seed=12)
    cfg = _cfg(mk, predict_tile=4)
    with mk.Session(subs, cfg, coords_test=ct) as ses:
        ses.run(cfg.n_samples)
        whole = ses.outputs()["w_predict"]
        for t0 in (0, 4, 8):
            g = ses.tile_grids(t0)
            tc = min(4, 10 - t0)
            assert g.shape == (2, 200, tc)
            for s in range(2):
                assert np.array_equal(g[s], whole[s][:, t0:t0 + tc])


def test_node_exchanges_over_rccl_in_a_fresh_process():
    """A process that starts with the node driver (the R host's situation, and bench.py's
    end-to-end leg) builds an RCCL communicator and combines over it, bit-identically."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = {k: v for k, v in os.environ.items() if k != "MK_EXCHANGE"}
    env["NCCL_DEBUG"] = "WARN"
    r = subprocess.run([sys.executable, os.path.join(here, "gpu_node_rccl.py")], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["exchange"] == "rccl" and res["exact"], res
