"""Meta-kriging fixtures at configs[1] / configs[3] geometry from the CPU oracle (TEST INFRASTRUCTURE
ONLY).  The configs[0] fixture has its own script (make_cfg1_meta.py); this one makes the two
geometries whose long-chain behaviour that fixture does not cover:

  cfg2_matern  BASELINE.json configs[1] geometry: Matern (nu free, U(0.1, 2)), q = 1, subsets of
               n_s = 1,000 (configs[1]'s subset size), K = 3, exact Matern GP field (nu = 0.5)
  cfg3_exp     BASELINE.json configs[2] geometry: exponential, q = 1, subsets of n_s = 2,000 (the
               headline's subset size), K = 3
  cfg4_lmc     BASELINE.json configs[3] geometry: q = 3 LMC (3n x 3n blocks), exponential,
               subsets of n_s = 500, K = 2, exact LMC field (beta)

Both: 1,000 amcmc iterations (20 x 50), burn-in 750 -> 251 kept, 200 kriging sites, seed
20250114, partition = R's stream after set.seed (MK.R:15-41), glm start values on the full data
(MK.R:53-55), per-subset spMvGLM + spPredict + 200 quantiles (MK.R:46-96, oracle/spmvglm.py),
combine MK.R:123-133.  Stored: the inputs and the oracle's per-subset samples, grids and the
combined result / result2.  The reference holds no fixtures and spBayes is absent:
this pins the device to the build's own oracle, not to spBayes.

    python tests/golden/stat/make_meta_fixture.py cfg2_matern   (~25 min on 3 cores: scipy kv)
    python tests/golden/stat/make_meta_fixture.py cfg3_exp      (~3 min on 3 cores)
    python tests/golden/stat/make_meta_fixture.py cfg4_lmc      (~3 min on 2 cores)
"""
import os
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")   # one BLAS thread per worker (set before numpy loads)
import importlib  # noqa: E402
import multiprocessing as mp  # noqa: E402
import sys  # noqa: E402

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"

CASES = {
    "cfg2_matern": dict(n=3000, K=3, q=1, cov_model=1, n_test=200),
    "cfg3_exp": dict(n=6000, K=3, q=1, cov_model=0, n_test=200),
    "cfg4_lmc": dict(n=1000, K=2, q=3, cov_model=0, n_test=200),
}
N_BATCH, BATCH_LENGTH, SEED = 20, 50, 20250114
LEVELS3 = (4, 99, 194)      # rows of the 200-level grid at probs 0.025, 0.5, 0.975


def _rows(idx, q):
    return (np.asarray(idx)[:, None] * q + np.arange(q)[None, :]).reshape(-1)


def _fit(args):
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    from oracle import spmvglm as om
    coords, y, x, coords_test, beta0, bt, s, q, cov_model = args
    cfg = om.Config(q, x.shape[1], beta_starting=beta0, beta_tuning=bt, cov_model=cov_model, n_batch=N_BATCH,
                    batch_length=BATCH_LENGTH, seed=SEED)
    r = om.fit_subset(coords, y, np.ones(y.size), x, cfg, subset=s, coords_test=coords_test)
    return r["param_q"], r["w_q"], r["samples"], r["accept"]


def make(case):
    from oracle import rrng, rstats
    from oracle import spmvglm as om
    c = CASES[case]
    n, K, q = c["n"], c["K"], c["q"]
    syn = importlib.import_module(PKG + ".synthetic")
    d = syn.generate(n, q=q, n_test=c["n_test"], cov_model=c["cov_model"], seed=SEED)
    n_part, index_part = rrng.partition(n, K, SEED)                 # 1-based, R's draw order
    coef, vcov = rstats.glm_binomial(d["y"], d["x"], np.ones(n * q))
    bt = np.diag(np.linalg.cholesky(vcov).T).copy()                 # diag(t(chol(vcov(fit)))), MK.R:55
    jobs = []
    for s in range(K):
        idx = np.asarray(index_part[s]) - 1
        r = _rows(idx, q)
        jobs.append((d["coords"][idx], d["y"][r], d["x"][r], d["coords_test"], coef, bt, s, q, c["cov_model"]))
    with mp.get_context("spawn").Pool(K) as pool:
        res = pool.map(_fit, jobs)
    n_rep = q * 2 + q * (q + 1) // 2 + q * (2 if c["cov_model"] == 1 else 1)
    out = dict(n=n, K=K, q=q, cov_model=c["cov_model"], n_test=c["n_test"], n_batch=N_BATCH,
               batch_length=BATCH_LENGTH, seed=SEED,
               coords=d["coords"], y=d["y"], x=d["x"], coords_test=d["coords_test"], x_test=d["x_test"],
               w_test_true=d["w_test_true"], beta_true=d["beta_true"], phi_true=d["phi_true"],
               n_part=np.asarray(n_part, dtype=np.int32),
               index=np.concatenate([np.asarray(i, dtype=np.int32) for i in index_part]),
               beta_starting=coef, beta_tuning=bt,
               param_q=np.stack([r[0] for r in res]),
               w_q3=np.stack([r[1][list(LEVELS3)] for r in res]),
               samples=np.stack([r[2] for r in res]),
               accept=np.stack([r[3][:, :n_rep] for r in res]))
    out["result"] = om.combine_mean([r[0] for r in res])           # MK.R:123-127
    out["result2"] = om.combine_mean([r[1] for r in res])          # MK.R:129-133
    np.savez_compressed(os.path.join(HERE, case + ".npz"), **out)
    print(case, "result median", out["result"][99], "95% CI", out["result"][4], out["result"][194])


if __name__ == "__main__":
    for name in sys.argv[1:] or sorted(CASES):
        make(name)
