"""Device covariance / Cholesky / inverse vs independent scipy references (SURVEY.md 8c:
covariance and Cholesky within 1e-10 relative error)."""
import numpy as np
import pytest
import scipy.linalg as sla

from oracle import spmvglm as om

pytestmark = pytest.mark.gpu

REL = 1e-10


def _coords(S, n, seed):
    return np.random.default_rng(seed).uniform(size=(S, n, 2))


@pytest.mark.parametrize("model,nu", [("exponential", None), ("matern", [0.5, 1.3, 0.21])])
def test_correlation_matches_oracle(mk, model, nu):
    S, n = 3, 200
    c = _coords(S, n, 1)
    phi = np.array([4.5, 7.0, 11.0])
    R = mk.correlation_batched(c, phi, nu=nu, cov_model=model)
    for s in range(S):
        D = om.distance_matrix(c[s], c[s])
        ref = om.correlation(D, phi[s], 0.0 if nu is None else nu[s], 1 if model == "matern" else 0)
        np.fill_diagonal(ref, 1.0)
        assert np.max(np.abs(R[s] - ref)) <= REL * np.max(np.abs(ref))


@pytest.mark.parametrize("nu", [0.05, 0.7, 3.4])
def test_candidate_matern_table_ranges_vs_scipy(mk, nu):
    """The Matern candidate kernel's Chebyshev tables (mk_corr.hpp cheb_*) at their edges: a tight
    cluster (x = phi d < 0.5: exact series), a duplicated site (d = 0 off the diagonal: rho = 1),
    sites spread over [0, 8]^2 so x runs past the last table interval (48.9: exact continued
    fraction) and every interval in between; element by element vs scipy.special.kv, 1e-10
    relative."""
    import scipy.special as ssp
    rng = np.random.default_rng(5)
    n = 600
    phi = np.array([6.5, 10.0])
    c = np.empty((len(phi), n, 2))
    for s in range(len(phi)):
        c[s] = np.concatenate([rng.uniform(0, 0.02, size=(200, 2)), rng.uniform(0, 8.0, size=(n - 200, 2))])
        c[s, 1] = c[s, 0]                                 # duplicated site
    R = mk.correlation_batched(c, phi, nu=np.full(len(phi), nu), cov_model="matern")
    for s in range(len(phi)):
        x = phi[s] * om.distance_matrix(c[s], c[s])
        assert x.max() > 60.0 and (x[x > 0] < 0.5).sum() > 1000
        ref = np.ones_like(x)
        m = x > 0
        ref[m] = np.power(x[m], nu) / (2.0 ** (nu - 1.0) * ssp.gamma(nu)) * ssp.kv(nu, x[m])
        np.fill_diagonal(ref, 1.0)
        ok = ref > 1e-280
        err = np.abs(R[s] - ref)[ok] / ref[ok]
        assert np.max(err) <= REL, (s, np.max(err))
        assert R[s][1, 0] == 1.0


@pytest.mark.parametrize("nu", [0.21, 0.5, 1.3, 1.9])
def test_candidate_matern_cfg2_geometry_vs_scipy(mk, nu):
    """configs[1] geometry (n_s = 1000, 8 tiles of 128): the sampler's binned Matern candidate
    kernel (k_cov_candidate<MK_COV_MATERN>, series / CF2 branches and x-range bins) against
    scipy.special.kv element by element, 1e-10 relative.  phi spans the
    prior support (4, 12) so x = phi d covers both Bessel branches and every bin."""
    import scipy.special as ssp
    n = 1000
    phi = np.array([4.0 + 1e-9, 7.3, 12.0 - 1e-9])
    c = _coords(len(phi), n, 17)
    R = mk.correlation_batched(c, phi, nu=np.full(len(phi), nu), cov_model="matern")
    for s in range(len(phi)):
        x = phi[s] * om.distance_matrix(c[s], c[s])
        ref = np.ones_like(x)
        m = x > 0
        ref[m] = np.power(x[m], nu) / (2.0 ** (nu - 1.0) * ssp.gamma(nu)) * ssp.kv(nu, x[m])
        np.fill_diagonal(ref, 1.0)
        err = np.abs(R[s] - ref)
        assert np.max(err / np.maximum(np.abs(ref), 1e-300)) <= REL, (s, np.max(err))
        assert np.array_equal(R[s], R[s].T)


@pytest.mark.parametrize("n", [1, 5, 127, 128, 200, 255, 256, 400, 700, 2000, 2047, 2048, 2049])
def test_cholesky_logdet_inverse(mk, n):
    S = 3
    c = _coords(S, n, n)
    A = np.stack([om.correlation(om.distance_matrix(c[s], c[s]), 4.0 + 3 * s, 0.0, 0) for s in range(S)])
    L, ld, inv = mk.cholesky_batched(A, inverse=True)
    for s in range(S):
        Lr = sla.cholesky(A[s], lower=True)
        assert np.linalg.norm(L[s] - Lr) <= REL * np.linalg.norm(Lr)
        ldr = 2.0 * np.sum(np.log(np.diag(Lr)))
        assert abs(ld[s] - ldr) <= REL * max(1.0, abs(ldr))
        Ir = om.cho_inverse(Lr)
        assert np.linalg.norm(inv[s] - Ir) <= 1e-9 * np.linalg.norm(Ir)


_FUSED_RUN = """
import importlib, sys, numpy as np
sys.path.insert(0, {root!r})
mk = importlib.import_module({pkg!r})
rng = np.random.default_rng(11)
S, n = 136, 700                     # >= 128 factors of 6 tiles: every launch takes 128-tiles
c = rng.uniform(size=(S, n, 2))
d = np.sqrt(((c[:, :, None, :] - c[:, None, :, :]) ** 2).sum(-1))
A = np.exp(-(3.0 + rng.uniform(size=(S, 1, 1)) * 6.0) * d)
L, ld = mk.cholesky_batched(A, inverse=False)
np.savez({path!r}, A=A[:4], L=L, ld=ld)
"""


def test_fused_update_trsm_is_bit_identical(tmp_path):
    """The fused column update + panel solve (k_chol_update_trsm, the default where every launch of a
    factorisation takes 128-tiles: >= 128 factors) gives the bits of the separate update, diagonal
    and trsm launches (MK_CHOL_FUSED=0), and a factor LAPACK agrees with."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"
    res = {}
    for fused in ("1", "0"):
        path = str(tmp_path / f"fused{fused}.npz")
        r = subprocess.run([sys.executable, "-c", _FUSED_RUN.format(root=root, pkg=pkg, path=path)],
                           capture_output=True, text=True, timeout=240, env=dict(os.environ, MK_CHOL_FUSED=fused))
        assert r.returncode == 0, r.stderr[-4000:]
        z = np.load(path)
        res[fused] = {k: z[k] for k in z.files}
    assert np.array_equal(res["1"]["L"], res["0"]["L"]) and np.array_equal(res["1"]["ld"], res["0"]["ld"])
    for s in range(4):
        Lr = sla.cholesky(res["1"]["A"][s], lower=True)
        assert np.linalg.norm(res["1"]["L"][s] - Lr) <= REL * np.linalg.norm(Lr)


def test_cholesky_rejects_non_pd(mk):
    A = np.eye(4)[None].copy()
    A[0, 3, 3] = -1.0
    with pytest.raises(mk.MkError):
        mk.cholesky_batched(A)


def test_combine_is_sequential_mean(mk):
    rng = np.random.default_rng(3)
    grids = [rng.normal(size=(200, 7)) for _ in range(13)]
    out = mk.combine(grids)
    ref = om.combine_mean(grids)
    assert np.array_equal(out, ref)          # same summation order -> bit identical


def test_sub_tile_gemm_split_cholesky_and_multi_wg_sweep_are_bit_identical(tmp_path):
    """Small-shard code paths give exactly the large-shard results: the 64- and 32-sub-tile GEMMs
    (Cholesky update / trsm, inverse levels; mk_gemm.hpp: same MFMA sequence per element), the
    split two-stream Cholesky schedule (bulk update by panels < k-d on a CU-masked stream, the
    rank-128d correction on the critical stream; the accumulator passes through fp64 memory) at
    depths 1-3, the 64-site-block sweeps -- one workgroup per subset (MK_SWEEP=1, k_sweep), the
    fused column update + panel solve (k_chol_update_trsm, 128- and 64-row forms, the unsplit
    factorisation; MK_CHOL_FUSED=0 the separate U, D, T launches), the sequential schedule's next
    candidates assembled beside the sweep (MK_EARLY_COV=0: in-line), the tiled replay's draws per
    phi run (MK_DRAW_RUNS=0: per kept state), the split launches (3: k_sweep_step, one launch per block) and the
    multi-workgroup kernel (2:
    k_sweep_mg behind its admission consensus, on both schedules; MK_ADM_SPINS=0 refuses the subsets
    whose workgroups do not arrive together, -1 every subset, and the k_sweep fallback queued behind
    it sweeps them) -- and the kriging GEMM with P^T generated in LDS (MK_PRED_GEN=1,
    exponential model) against the stored-P^T path.  Chains, latent w, kriging draws and a plain
    factorisation, each configuration forced in its own process (the MK_* switches are read once
    per process); the two launch schedules agree to rounding, not bit for bit, so each configuration
    is compared with the reference of its schedule."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = {}
    # (MK_TILE, MK_SWEEP, MK_CHOL_SPLIT, MK_PRED_GEN, MK_CHOL_DEPTH, lookahead)
    configs = (("128", "1", "0", "0", "2", "1"),
               ("128", "2", "0", "0", "2", "1"),
               ("128", "2", "0", "0", "2", "0"),
               ("64", "3", "1", "0", "1", "0"),
               ("64", "1", "0", "0", "2", "1"),
               ("32", "1", "1", "0", "2", "1"),
               ("128", "3", "1", "0", "3", "0"),
               ("128", "1", "0", "1", "2", "1"),
               ("64", "1", "1", "0", "2", "1"),
               ("128", "3", "0", "0", "2", "1"),
               ("64", "2", "1", "0", "3", "0"),
               ("64", "3", "1", "0", "2", "0"),
               ("128", "1", "0", "0", "2", "0"))
    runs = [(cfg, {}) for cfg in configs] + [(("128", "2", "0", "0", "2", "1"), {"MK_ADM_SPINS": "0"}),
                                              (("64", "2", "1", "0", "3", "0"), {"MK_ADM_SPINS": "-1"}),
                                              (("128", "2", "0", "0", "2", "1"), {"MK_ADM_SPINS": "-1"}),
                                              (("128", "1", "0", "0", "2", "0"), {"MK_CHOL_FUSED": "0"}),
                                              (("128", "1", "0", "0", "2", "1"), {"MK_CHOL_FUSED": "0"}),
                                              (("64", "1", "0", "0", "2", "1"), {"MK_CHOL_FUSED": "0"}),
                                              (("128", "1", "0", "0", "2", "0"), {"MK_EARLY_COV": "0"}),
                                              (("128", "3", "1", "0", "3", "0"), {"MK_EARLY_COV": "0"}),
                                              (("128", "1", "0", "0", "2", "1"), {"MK_DRAW_RUNS": "0"})]
    for cfg, extra in runs:
        tile, sweep, split, gen, depth, la = cfg
        key = cfg + tuple(k_[3:] + v for k_, v in extra.items())
        path = str(tmp_path / ("run_" + "_".join(key) + ".npz"))
        r = subprocess.run([sys.executable, os.path.join(here, "gpu_tile_run.py"), path], capture_output=True,
                           text=True, timeout=240,
                           env=dict(os.environ, MK_TILE=tile, MK_SWEEP=sweep, MK_CHOL_SPLIT=split, MK_PRED_GEN=gen,
                                    MK_CHOL_DEPTH=depth, **extra,
                                    **({} if la == "1" else {"MK_LOOKAHEAD": "0"})))
        assert r.returncode == 0, r.stderr[-4000:]
        z = np.load(path)
        res[key] = {k: z[k] for k in z.files}
        if extra.get("MK_ADM_SPINS") == "-1":   # the fallback did run (with 0 it depends on arrival timing)
            assert int(open(path + ".fallback").read()) > 0, key
    refs = {"1": res[configs[0]], "0": res[configs[-1]]}
    for cfg, got in res.items():
        ref = refs[cfg[5]]
        assert got.keys() == ref.keys()
        for k in ref:
            assert np.array_equal(got[k], ref[k]), (cfg, k)


def test_site_sweep_runs_the_block_sweeps_chain(tmp_path):
    """The one-pass site sweep (k_sweep_site, the default: W read once, no Q_BB tiles; q = 1 its lean
    pair form, with the border-row factor where a subset's n_s is odd) and the 64-site-block sweep
    (MK_SWEEP=1, k_sweep) run the same chain: the dot products are summed in a different order, so
    the chains agree to rounding -- identical accept decisions, samples, latent w and kriging draws
    within 1e-9 -- under both launch schedules (q = 1 ragged subsets and the Matern model; q = 2 with
    two subsets is a multi-outcome small shard and runs the block sweeps either way).  q = 3 and
    n_s > 2047 (two row pairs per thread) are covered by the oracle replays of
    tests/test_gpu_sampler.py, which run the default sweep."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for la in ("1", "0"):
        res = {}
        for sweep in ("1", "0"):
            path = str(tmp_path / f"site_{sweep}_{la}.npz")
            env = dict(os.environ, MK_SWEEP=sweep, **({} if la == "1" else {"MK_LOOKAHEAD": "0"}))
            r = subprocess.run([sys.executable, os.path.join(here, "gpu_tile_run.py"), path], capture_output=True,
                               text=True, timeout=240, env=env)
            assert r.returncode == 0, r.stderr[-4000:]
            z = np.load(path)
            res[sweep] = {k: z[k] for k in z.files}
        for k in res["1"]:
            np.testing.assert_allclose(res["0"][k], res["1"][k], rtol=0, atol=1e-9, err_msg=f"{k} la={la}")
