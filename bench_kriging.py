#!/usr/bin/env python3
"""Kriging throughput at BASELINE.json configs[4] scale: spPredict of 1,000,000 held-out sites
(the line's value: the phi-interpolated replay over a real 1,251-state window; beside
it, `exact_sample`, the exact replay on a 6-state sample with the kriging GEMM's roofline)
(n = 500k, K = 250 subsets of 2,000, exponential, q = 1), run through the tiled path
(predict_tile): the kept chain states are recorded during the fit and the kriging replays them
over test-site tiles, so 1M x kept draws per subset never coexist in HBM.

A full cfg5 run (250 subsets x 1M sites x 1,251 kept samples) is ~10^17 flops; this script times a
bounded sample -- `--subsets` subsets, `--kept` kept samples, all 1M sites -- and reports the
measured rates plus the extrapolation to the full configuration.  Unit of work: one kriging draw
(subset, test site, kept sample).  Algorithmic flops: per (subset, distinct (phi, nu) run) the
triangular X = W P^T costs n_s^2 * n_test (W lower-triangular n_s x n_s); the per-run Cholesky +
inverse (2 n_s^3 / 3) and the draws (2 n_s per draw) are counted too.

  python bench_kriging.py [--subsets 32] [--n-test 1000000] [--kept 6] [--tile 65536]
"""
import argparse
import os

# before HIP starts: libmk's lookahead schedule runs up to five HIP streams and HIP shares
# hardware queues beyond GPU_MAX_HW_QUEUES (4 by default)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import importlib
import json
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"
FP64_PEAK_TFLOPS = 78.6


def kriging_leg(mk, subs, coords_test, beta0, bt, kept=6, burn=14, tile=65536, kernel_events=True, subset_base=0,
                fit_chunk=0):
    """Tiled spPredict of `coords_test` from the subsets `subs` (n_s each): burn + kept iterations with
    the kept states recorded, then the replay over test-site tiles, timed.  Returns the result dict
    (draws/s, k_pred_var roofline, the configs[4] extrapolation).  bench.py runs it on the per-GPU
    share of configs[2]'s own subsets with 1M sites (the driver-measured configs[4] rate)."""
    S = len(subs)
    ns = int(max(len(s_["coords"]) for s_ in subs))
    n_test = int(np.asarray(coords_test).shape[0])
    n_samples = burn + kept
    cfg = mk.SamplerConfig(1, 2, beta0, bt, n_batch=1, batch_length=n_samples, burn_in=burn + 1, seed=20250114,
                           predict_tile=tile)
    with mk.Session(subs, cfg, coords_test=coords_test, subset_base=subset_base) as ses:
        t0 = time.perf_counter()
        if fit_chunk > 0:   # the fit in pieces of fit_chunk iterations (each mk_session_run ends with the device idle)
            for i in range(0, n_samples, fit_chunk):
                ses.run(min(fit_chunk, n_samples - i))
        else:
            ses.run(n_samples)
        t1 = time.perf_counter()
        if kernel_events:   # HIP events around every k_pred_var launch (the kriging GEMM)
            ses.profile(True, kinds=[mk.session.KS_PRED_VAR])
        out = ses.outputs(quantiles=False, samples=True, w_predict_sum=True)
        t2 = time.perf_counter()
        pv = ses.kernel_stats(mk.session.KS_PRED_VAR)
    kept_phi = np.stack([smp[burn:, 3] for smp in out["samples"]])          # phi column of p.beta.theta.samples
    runs = int(sum(1 + np.count_nonzero(np.diff(r)) for r in kept_phi))
    pred_s = t2 - t1
    flops = runs * (ns * ns * n_test + 2.0 * ns ** 3 / 3.0 * ((n_test + tile - 1) // tile)) \
        + 2.0 * ns * S * n_test * kept
    draws = S * n_test * kept
    # extrapolation: cfg5 = 250 subsets x 1M sites x 1251 kept; runs scale with the kept acceptance of phi
    run_frac = runs / (S * kept)
    cfg5_flops = 250 * 1251 * run_frac * ns * ns * 1_000_000
    rate_tf = flops / pred_s / 1e12
    res = {
        "metric": "kriging draws/s (tiled spPredict, configs[4] scale)",
        "value": draws / pred_s, "unit": "draws/s", "n_gpus": 1, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"configs[4] sample: {S} subsets of {ns}, {n_test} test sites, {kept} kept samples, "
                               f"tile {tile}", "subsets": S, "n_test": n_test, "kept": kept, "tile": tile},
        "fit_seconds": t1 - t0, "predict_seconds": pred_s, "phi_runs": runs,
        "roofline": {"bound": "mfma", "achieved": rate_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": rate_tf / FP64_PEAK_TFLOPS},
        "cfg5_extrapolation": {"flops": cfg5_flops, "seconds_1gpu": cfg5_flops / (rate_tf * 1e12),
                               "seconds_8gpu": cfg5_flops / (rate_tf * 1e12) / 8,
                               "assumes": f"phi runs per kept sample {run_frac:.3f} as measured here"},
        "w_predict_sum_finite": bool(np.isfinite(out["w_predict_sum"]).all()),
    }
    if kernel_events and pv["ms"] > 0:
        gemm_flops = runs * ns * ns * n_test   # X = W P^T, W lower-triangular, per (subset, phi run)
        tf = gemm_flops / (pv["ms"] * 1e-3) / 1e12
        gen = os.environ.get("MK_PRED_GEN", "0") not in ("", "0")
        res["k_pred_var"] = {"launches": pv["launches"], "ms": pv["ms"], "avg_launch_ms": pv["ms"] / pv["launches"],
                             "algorithmic_flops": gemm_flops, "achieved": tf, "unit": "TFLOP/s",
                             "frac": tf / FP64_PEAK_TFLOPS, "p_t": "generated in LDS" if gen else "stored",
                             "algorithmic_bytes": runs * (ns * ns / 2 + (1 if gen else 2) * ns * n_test) * 8.0,
                             "bytes_note": "per (subset, phi run): W (lower) read once, X written once"
                                           + ("" if gen else ", P^T read once")}
    return res


def interpolated_share(mk, subs, coords_test, beta0, bt, tile=65536, subset_base=0):
    """configs[4] through the phi-interpolated replay (mk_api.hip predict_tile_cheb), measured on a real
    kept window: the fit of MK.R:83 as written (100 x 50 amcmc iterations, burn.in 3,750 -> 1,251 kept)
    on `subs` with the test sites, then the first two test tiles' replay + 200-level grids (the first
    also makes every kept state's g = W' z, once per window).  Returns the measured phases, the
    per-tile rate (draws/s), the exact-path refresh count of the same window, and the per-GPU share
    of the full job priced from them (fit + g pass + tiles x the second tile's time)."""
    S = len(subs)
    n_test = int(np.asarray(coords_test).shape[0])
    cfg = mk.SamplerConfig(1, 2, beta0, bt, n_batch=100, batch_length=50, seed=20250114, predict_tile=tile)
    with mk.Session(subs, cfg, coords_test=coords_test, subset_base=subset_base) as ses:
        tile = ses.predict_tile
        t0 = time.perf_counter()
        ses.run(cfg.n_samples)
        t1 = time.perf_counter()
        out = ses.outputs(quantiles=False, samples=True, w_predict=False)
        times, sites = [], []
        for ti in range(min(2, (n_test + tile - 1) // tile)):
            ta = time.perf_counter()
            g = ses.tile_grids(ti * tile)
            times.append(time.perf_counter() - ta)
            sites.append(int(g.shape[2]))
            finite = bool(np.isfinite(g).all())
            del g
        cheb = ses.kernel_stats(mk.session.KS_KRIG_CHEB)
        fb = ses.kernel_stats(mk.session.KS_KRIG_FALLBACK)
    kept = np.stack([smp[cfg.burn_in - 1:, 3] for smp in out["samples"]])
    runs = int(sum(1 + np.count_nonzero(np.diff(r)) for r in kept))
    n_tiles = (1_000_000 + tile - 1) // tile
    per_tile = times[-1]
    g_pass = times[0] - times[-1] if len(times) > 1 else 0.0
    return {"workload": f"{S} subsets, {n_test} test sites, 100 x 50 amcmc iterations, burn.in {cfg.burn_in} "
                        f"({cfg.kept} kept), tiles of {tile}: the first {len(times)} replayed",
            "fit_seconds": t1 - t0, "tile_seconds": times, "tile_sites": sites, "g_pass_seconds": g_pass,
            "draws_per_s": S * sites[-1] * cfg.kept / per_tile, "interpolated_tiles": cheb["launches"],
            "fallback_tiles": fb["launches"], "exact_evaluations_per_subset_tile": cheb["flops"] / max(1, S * cheb["launches"]),
            "max_check_difference": cheb["ms"], "grids_finite": finite,
            "exact_refreshes_per_subset": runs / S, "refreshes_per_kept_sample": runs / kept.size,
            "cfg5_share_seconds_estimate": (t1 - t0) + g_pass + n_tiles * per_tile,
            "estimate_note": f"fit + g pass + {n_tiles} tiles x the second tile's replay + grids (the host combine of "
                             f"the grids not included); tools/cfg5_share.py measures the whole share"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--subsets", type=int, default=32)   # the per-GPU share of K = 250 on 8 GPUs
    ap.add_argument("--n-sub", type=int, default=2000)
    ap.add_argument("--n-test", type=int, default=1_000_000)
    ap.add_argument("--kept", type=int, default=6)
    ap.add_argument("--burn", type=int, default=14)
    ap.add_argument("--tile", type=int, default=65536)
    ap.add_argument("--kernel-events", type=int, default=1, help="HIP events around k_pred_var (0: off)")
    ap.add_argument("--fit-chunk", type=int, default=0,
                    help="run the fit in pieces of this many iterations, each ending with the device idle (0: one "
                         "call). Under rocprofv3 --pmc (kernels serialised) one 16-iteration call queues more "
                         "launches than the profiler's packet intercept survives (DESIGN.md 6)")
    ap.add_argument("--phi-window", type=int, default=1,
                    help="price the configs[4] extrapolation from a full 5,000-iteration fit's kept window (0: off)")
    a = ap.parse_args()
    if os.environ.get("MK_SEGV_DIAG"):
        # diagnostic (tools/segv_diag.c): a host SIGSEGV appends its PC, frames and the process maps here
        import ctypes
        ctypes.CDLL(os.path.join(ROOT, "tools", "segv_diag.so")).segv_diag_install(os.environ["MK_SEGV_DIAG"].encode())
    mk = importlib.import_module(PKG)
    S, ns = a.subsets, a.n_sub
    d = mk.synthetic.generate(S * ns, q=1, n_test=a.n_test, seed=20250114)
    beta0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)
    subs = [dict(coords=d["coords"][i * ns:(i + 1) * ns], y=d["y"][i * ns:(i + 1) * ns], weights=np.ones(ns),
                 x=d["x"][i * ns:(i + 1) * ns]) for i in range(S)]
    res = kriging_leg(mk, subs, d["coords_test"], beta0, bt, kept=a.kept, burn=a.burn, tile=a.tile,
                      kernel_events=bool(a.kernel_events), fit_chunk=a.fit_chunk)
    if a.phi_window:
        # price the full job from the phi sequence of a full 1,251-sample kept window (the sample above
        # holds only a few kept states, the first always a refresh); the same window through the
        # phi-interpolated replay, two tiles measured
        inter = interpolated_share(mk, subs, d["coords_test"], beta0, bt, tile=a.tile)
        res["interpolated"] = inter
        frac, fit_s, n_kept = inter["refreshes_per_kept_sample"], inter["fit_seconds"], 1251
        ex = res["cfg5_extrapolation"]
        rate_tf = res["roofline"]["achieved"]
        cfg5_flops = 250 * 1251 * frac * ns * ns * 1_000_000
        res["cfg5_extrapolation_sample"] = ex
        res["cfg5_extrapolation"] = {
            "flops": cfg5_flops, "seconds_1gpu": cfg5_flops / (rate_tf * 1e12),
            "seconds_8gpu": cfg5_flops / (rate_tf * 1e12) / 8,
            "path": "exact replay (MK_KRIG_CHEB=0; the 6-state sample above runs it: its window is too short "
                    "for the interpolation to pay)",
            "refreshes_per_kept_sample": frac,
            "assumes": f"X = W P^T refreshes per kept sample {frac:.3f}, measured on these {S} subsets' full kept "
                       f"window ({n_kept} kept of 100 x 50 amcmc iterations, burn.in 3,750; fit {fit_s:.1f} s) at "
                       f"the rate measured above"}
        # the headline of this leg is the path the job takes: the interpolated replay over the real window
        # (the exact replay's 6-state sample stays beside it, with the kriging GEMM's roofline)
        res["exact_sample"] = {"value": res["value"], "unit": "draws/s", "path": "exact replay, the 6-state sample",
                               "config": res["config"]}
        res["value"] = inter["draws_per_s"]
        res["config"] = {"workload": f"configs[4] per-GPU share: {S} subsets of {ns}, {a.n_test} test sites in tiles "
                                     f"of {a.tile}, 100 x 50 amcmc iterations (1,251 kept states), phi-interpolated "
                                     f"replay; rate over the second tile (the first also makes the window's g)",
                         "subsets": S, "n_test": a.n_test, "kept": 1251, "tile": a.tile}
        res["cfg5_share_seconds_estimate"] = inter["cfg5_share_seconds_estimate"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
