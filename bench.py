#!/usr/bin/env python3
"""Benchmark: MCMC subset-iterations/s (all subsets, whole node) on BASELINE.json's
headline configuration -- n=500,000 binary sites split into K=250 subsets of 2,000,
exponential covariance, q=1, 1,000 kriging sites (configs[2]).

A step = one spMvGLM amcmc iteration of EVERY subset (beta, A, phi MH with a fresh
2000x2000 Cholesky per subset, inverse where phi moved, single-site w sweep) plus,
on kept iterations, the fused spPredict kriging draw.  The timed window follows the
reference schedule (MK.R:57-59, 85): 3 burn-in iterations per kept one.

Multi-GPU (torch.distributed.run, one rank per GPU): by default the ONE configs[2] job is
split over the ranks (strong scaling, balanced contiguous subset blocks: 250 over 8 GPUs is
31-32 subsets each) -- the job BASELINE's metric is quoted on.  --scaling weak is opt-in:
every rank then fits its own configs[2]-sized shard (a node job of n = N x 500k, K = N x 250)
and the metric / config strings say so.  No data-path collective either way (the subsets are
independent until the combine, which run_metakriging.py measures).

roofline.traffic is the PMC-measured HBM traffic of the same kernel from profiles/
(rocprofv3 --pmc passes of this command, gfx950 FETCH_SIZE x2 correction).

  python bench.py --gpus N --steps K --warmup W
"""
import argparse
import os

# before HIP starts: libmk's lookahead schedule runs up to five HIP streams and HIP shares
# hardware queues beyond GPU_MAX_HW_QUEUES (4 by default)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
# the fused kriging of the windows' kept iterations draws from phi tables made at session set-up (DESIGN.md
# 4.7), as the whole job does: libmk's default selects them for the job's 1,251-state kept window, but a
# bench window session keeps only a few dozen states, so the choice is stated here (the set-up is outside
# the timed window; the end-to-end leg runs the job as written and pays it)
KRIG_SET_HERE = "MK_KRIG_CHEB" not in os.environ
if KRIG_SET_HERE:
    os.environ["MK_KRIG_CHEB"] = "-1"
import importlib
import json
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"

FP64_PEAK_TFLOPS = 78.6     # MI355X dense fp64 (vector = MFMA), AMD datasheet
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=500_000)
    ap.add_argument("--subsets", type=int, default=250)
    ap.add_argument("--n-test", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the extra legs (N=1): the 32-subset shard window and the configs[4] kriging sample")
    ap.add_argument("--shard-subsets", type=int, default=32,
                    help="subsets of the shard leg (the per-GPU share of configs[2] on 8 GPUs)")
    ap.add_argument("--krig-subsets", type=int, default=32, help="subsets of the configs[4] kriging leg")
    ap.add_argument("--krig-sites", type=int, default=1_000_000, help="test sites of the configs[4] kriging leg")
    ap.add_argument("--leg", choices=("configs1", "configs3", "configs3_share7"), default=None,
                    help="run only this window leg (configs[1] Matern K=50, configs[3] q=3 K=50 or its 7-subset "
                         "8-GPU share) and print its JSON")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostic: no per-kernel HIP events in the timed region (roofline fields then null)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="bracket the roofline kernel's launches of every k-th iteration of the timed window (a "
                         "sample; events on every launch cost 0.5 %% of the rate at 250 subsets, ~4 %% at 32: "
                         "profiles/r06/events)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): the one K-subset job split over the ranks; weak: K subsets per rank "
                         "(node job N*K)")
    ap.add_argument("--streams", type=int, default=0, help="HIP streams per GPU for subset groups (0: library default)")
    ap.add_argument("--adapt-batches", type=int, default=6,
                    help="untimed amcmc batches of 50 before the warmup (adapted proposal scales in the window)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the measured end-to-end leg (N=1: the whole configs[2] script, ~2 minutes)")
    ap.add_argument("--e2e-devices", default="0",
                    help="GPUs of the end-to-end leg, one process through libmk's multi-device driver "
                         "(mk_meta_fit), e.g. 0,1,2,3,4,5,6,7 on a node")
    ap.add_argument("--e2e-only", action="store_true",
                    help="internal: run only the end-to-end leg on --e2e-devices and print its JSON (rank 0 of a "
                         "multi-GPU bench starts this as a child process)")
    return ap.parse_args()


# ------------------------------------------------------------------ CPU baseline (oracle, rank 0, N=1)
def _cpu_worker(args):
    sub, coords_test, cfg_kw, subset, state, end = args
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    sys.path.insert(0, ROOT)
    from oracle import spmvglm as om
    cfg = om.Config(1, 2, **cfg_kw)
    r = om.fit_subset(sub["coords"], sub["y"], sub["weights"], sub["x"], cfg, subset=subset, coords_test=coords_test,
                      max_iter=end, quantiles=False, sweep="c", start=state)
    # the MCMC iterations only (set-up and the resume's re-factorisation excluded, as on the GPU side)
    return r["loop_seconds"], r["phase_seconds"], r["samples"][state["iteration"]:end]


def cpu_baseline(subs, coords_test, cfg_kw, states, end, workers):
    """The oracle over the device's own timed window: subset i (i < workers, global index i, the same
    Philox streams) resumes from the device's chain state at the window's first iteration
    (mk_session_chain_state: adapted proposal scales, the current batch's accept counts) and runs the
    same iterations -- the same burn-in : kept split, kriging on the kept ones -- one process and one
    BLAS thread per core.  Returns the rate, the per-phase seconds per subset-iteration and the
    window's samples (to compare with the device's)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    saved = {k: os.environ.get(k) for k in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS")}
    os.environ["OPENBLAS_NUM_THREADS"] = os.environ["OMP_NUM_THREADS"] = "1"   # inherited by the spawned workers
    jobs = [(subs[i], coords_test, cfg_kw, i, states[i], end) for i in range(workers)]
    t0 = time.perf_counter()
    try:
        with ctx.Pool(workers) as pool:
            res = pool.map(_cpu_worker, jobs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    wall = time.perf_counter() - t0
    steps = end - states[0]["iteration"]
    loops = [r[0] for r in res]
    rate = workers * steps / max(loops)      # over the slowest worker's iteration loop
    phases = {k: sum(r[1][k] for r in res) / (workers * steps) for k in res[0][1]}
    return dict(value=rate, unit="subset-iters/s", cores=workers, kind="port",
                phase_s_per_subset_iter=phases,
                sample=f"{workers} of the device's subsets (global indices 0..{workers - 1}, n_s="
                       f"{len(subs[0]['coords'])}, {np.asarray(coords_test).shape[0]} kriging sites) over the device's "
                       f"own timed window, iterations {states[0]['iteration'] + 1}-{end}, resumed from the device's "
                       f"chain state there (adapted scales); oracle/spmvglm.py: LAPACK dpotrf/dpotri (OpenBLAS), "
                       f"NumPy vector work and the latent sweep in C (oracle/csrc/sweep.c), one process and one BLAS "
                       f"thread per core; wall {wall:.1f}s incl. start-up"), [r[2] for r in res]


def physical_cores():
    """Physical cores of the host: distinct SMT sibling sets in sysfs (None if unreadable)."""
    import glob
    sets = set()
    for p_ in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/topology/thread_siblings_list"):
        try:
            with open(p_) as f:
                sets.add(f.read().strip())
        except OSError:
            pass
    return len(sets) or None


def window_leg(mk, d, idx, S, q, cov, beta0, bt, adapt_batches, warmup, steps, event_every=1):
    """S subsets (global indices 0..S-1 of the partition idx of data d) over the headline's kind of
    window: adapt, warm up, then `steps` iterations timed with the 3:1 burn-in : kept split (kriging
    on the kept ones).  Returns rate, ms per step, schedule and the k_chol_update union rate."""
    A = max(0, adapt_batches) * 50
    W = max(1, warmup) + A
    n_burn = int(round(0.75 * steps))
    post = 8       # the roofline's evented pass after the window (kept iterations)
    cfg = mk.SamplerConfig(q, 2 * q, beta0, bt, cov_model=cov, n_batch=(W + steps + post + 49) // 50,
                           batch_length=50, burn_in=W + n_burn + 1, seed=20250114)
    subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], q, idx[i]) for i in range(S)]
    with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
        ses.run(W)
        # the window runs without per-launch events (at 32 subsets they cost ~4 % of the rate,
        # profiles/r06/events); the column-update launches are timed in a pass of `post` iterations after it
        t0 = time.perf_counter()
        ses.run(steps)
        el = time.perf_counter() - t0
        fb = ses.kernel_stats(mk.session.KS_SWEEP_FALLBACK)["launches"]
        ses.profile(True, kinds=[mk.session.KS_CHOL_UPDATE, mk.session.KS_CHOL_UPDATE_SUB], every=event_every)
        ses.run(post)
        st = ses.kernel_stats(mk.session.KS_UPDATE_BUSY)
        la = ses.lookahead
    tf = st["flops"] / (st["ms"] * 1e-3) / 1e12 if st["ms"] > 0 else 0.0
    return {"value": S * steps / el, "unit": "subset-iters/s", "ms_per_step": el / steps * 1e3,
            "sweep_fallbacks": fb,   # (subset, iteration) sweeps k_sweep_mg refused admission (k_sweep ran them)
            "window": f"{n_burn} burn-in + {steps - n_burn} kept iterations at {W + 1}-{W + steps} (after {A} "
                      f"adaptation + {W - A} warmup iterations)",
            "schedule": "lookahead" if la else "sequential",
            "roofline": {"kernel": "column-update launches: k_chol_update_trsm / k_chol_update (union of their launch "
                                   "intervals; algorithmic flops as the headline roofline's)", "achieved": tf,
                         "source": f"{post} kept iterations after the window, every launch evented",
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                         "note": "lookahead schedule: update launches share the chip with the main stream, so "
                                 "the fraction understates the kernel's own rate" if la else
                                 "sequential schedule: update launches run alone"}}


def shard_leg(mk, d, idx, S, beta0, bt, adapt_batches, warmup, steps):
    """The per-GPU share of configs[2] on 8 GPUs (S = 32 of its 250 subsets): the rate an 8-GPU
    strong-scaling run's ranks each see."""
    r = window_leg(mk, d, idx, S, 1, "exponential", beta0, bt, adapt_batches, warmup, steps)
    r["workload"] = (f"{S} of configs[2]'s subsets (the per-GPU share of K=250 on 8 GPUs), n_s=2000, exponential, "
                     f"q=1, n_test=1000, window " + r.pop("window"))
    # an 8-GPU strong-scaling run: every rank holds <= S (31-32) of the 250 subsets at this chain rate
    r["projected_8gpu_value"] = 250 * 1e3 / r["ms_per_step"]
    return r


def config_leg(mk, which, adapt_batches, warmup, steps, subsets=None):
    """configs[1] (Matern, n = 50,000, K = 50 subsets of 1,000) or configs[3] (q = 3 LMC, n = 100,000,
    K = 50 subsets of 2,000) on one GPU -- all K subsets, or the first `subsets` (configs[3]'s per-GPU
    share on 8 GPUs is 6-7) -- over the headline's kind of window; data from the SURVEY.md 8d
    generator, R's partition, glm start values on the full data."""
    n, K, q, cov = {1: (50_000, 50, 1, "matern"), 3: (100_000, 50, 3, "exponential")}[which]
    d = mk.synthetic.generate(n, q=q, n_test=1000, cov_model=1 if cov == "matern" else 0, seed=20250114)
    _, idx = mk.partition(n, K, seed=20250114, method="R")
    beta0, bt = mk.start_values(d["y"], d["x"], 1.0, q)
    S = K if subsets is None else min(subsets, K)
    r = window_leg(mk, d, idx, S, q, cov, beta0, bt, adapt_batches, warmup, steps)
    r["workload"] = (f"configs[{which}]: n={n}, K={K} subsets of {n // K}, {cov}, q={q}, n_test=1000; "
                     + (f"all {K} subsets" if S == K else f"the first {S} (the per-GPU share on 8 GPUs)")
                     + ", window " + r.pop("window"))
    return r


def host_cores():
    """Cores this process may use: the affinity mask, capped by the job's CPU share when the
    launcher states one (OMP_NUM_THREADS: 16 per GPU on the MI355X pool, whose nproc shows the
    whole machine).  Returns the count used plus nproc, the affinity size and the CPU model."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    usable, note = aff, "all cores in the affinity mask"
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and 0 < int(share) < aff:
        usable, note = int(share), f"the job's CPU share (OMP_NUM_THREADS={share}) of {aff} cores in the affinity mask"
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return dict(usable=max(1, usable), nproc=nproc, affinity=aff, model=model, note=note)


def _pmc_traffic():
    """HBM bytes per column-update launch (k_chol_update_trsm + k_chol_update, launch-weighted) from
    the committed rocprofv3 --pmc passes (or None)."""
    path = os.path.join(ROOT, "profiles", "pmc_chol_update.json")
    try:
        with open(path) as f:
            return json.load(f)["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def hbm_subphases(kern, n_post, n_s):
    """GB/s of the covariance assembly and the latent sweep over the post-window pass (per-kernel
    HIP events), on algorithmic bytes, as a fraction of the HBM peak."""
    out = {}
    for name, per_subset in (("cov_candidate", lambda n: 4.0 * (n + 1) ** 2), ("w_sweep", lambda n: 4.0 * n * n)):
        ms = kern[name]["ms"]
        if ms > 0:
            gbs = sum(per_subset(n) for n in n_s) * n_post / (ms * 1e-3) / 1e9
            out[name] = {"GB/s": gbs, "frac_of_hbm_peak": gbs / HBM_PEAK_GBS}
    return out


def inverse_roofline(k):
    """k_inv_level's rate over the post-window pass: algorithmic flops (per level the full-by-
    triangular and triangular-by-full products over each accepted factor's extent n_s; with the
    diagonal tiles' inverses inside k_chol_diag they sum to n_s^3 / 3 per factor) over the summed
    launch durations (one stream: the launches do not overlap)."""
    if k["ms"] <= 0:
        return None
    tf = k["flops"] / (k["ms"] * 1e-3) / 1e12
    return {"kernel": "k_inv_level (recursive-doubling W = L^-1 of the accepted factors)", "bound": "mfma",
            "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
            "launches": k["launches"], "avg_launch_ms": k["ms"] / max(1, k["launches"]),
            "algorithmic_flops_per_launch": k["flops"] / max(1, k["launches"]),
            "source": "untimed post-window pass, every kernel kind evented"}


def end_to_end(mk, d, K, devices=(0,)):
    """The whole reference script on this GPU (metakriging.reference_flow -> mk_meta_fit):
    partition (R's stream) -> glm -> 5,000 amcmc iterations of every subset with spPredict on the
    1,251 kept ones -> 200-level grids -> combine -> MK.R:136-165, wall clock per phase.  The
    reference's own timer (MK.R:106-111) covers the foreach only: set-up + chains + quantiles."""
    import time
    marks = []
    t0 = time.perf_counter()

    def progress(it, n):      # spBayes's n.report = 10 batches (MK.R:84)
        if it % 500 == 0:
            marks.append((it, time.perf_counter() - t0))
            print(f"e2e: {it}/{n} iterations, {marks[-1][1]:.1f}s", file=sys.stderr, flush=True)
        return False

    ph, result, result2, summ, cfg = mk.metakriging.reference_flow(d, K, 1, n_batch=100, batch_length=50,
                                                                   seed=20250114, devices=devices, progress=progress)
    return {"phases": ph,
            "reference_timer_s": ph["setup_s"] + ph["chains_s"] + ph["quantiles_combine_s"],
            "chains_subset_iters_per_s": K * cfg.n_samples / ph["chains_s"],
            "devices": list(devices),
            "exchange": ph.get("exchange"),
            "comm_ranks": ph.get("comm_ranks"),     # the ranks mk_meta_fit's RCCL communicators hold
            "workload": f"configs[2] end to end on {len(devices)} GPU(s), one process: n={len(d['coords'])}, K={K}, "
                        f"exponential, q=1, "
                        f"n_test={len(d['coords_test'])}, 100 x 50 amcmc iterations, burn.in 3,750 "
                        f"({cfg.kept} kept with spPredict), sequential-mean combine, 1,000-draw summary",
            "param_median": summ["param_quant"][0].tolist()}


def kriging_leg_process(subsets, sites):
    """bench_kriging.py's configs[4] leg (tiled spPredict of `sites` test sites from `subsets` subsets)
    run as a child process; its JSON line, or the error."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench_kriging.py"), "--subsets", str(subsets), "--n-test", str(sites)]
    env = dict(os.environ)
    if KRIG_SET_HERE:   # the kriging leg chooses its paths itself (the 6-state sample: the exact replay)
        env.pop("MK_KRIG_CHEB", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"bench_kriging.py rc {r.returncode}: {r.stderr[-2000:]}"}
    res = json.loads(lines[-1])
    res["process"] = "child (bench_kriging.py)"
    return res


def node_end_to_end(a, world):
    """N > 1 (strong scaling): the same whole configs[2] script over the node's N GPUs through
    mk_meta_fit (libmk's threads, RCCL combine) -- a fresh child process, started (not exec'd)
    by rank 0 once every rank has closed its session; the other ranks wait on a CPU barrier."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--e2e-only", "--n", str(a.n), "--subsets", str(a.subsets),
           "--n-test", str(a.n_test), "--e2e-devices", ",".join(str(i) for i in range(world))]
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600)   # stderr: progress lines; ~20 s expected on 8 GPUs
        if r.returncode != 0:
            return {"error": f"exit {r.returncode}", "stdout_tail": r.stdout[-500:]}
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:          # the bench line is printed regardless
        return {"error": repr(e)[:500]}


def launcher_cmd(a, argv, port):
    """--gpus N > 1 without a launcher: the torch.distributed.run command that runs this same bench
    as N ranks, one per GPU of this node (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


class _stdout_to_stderr:
    """fd 1 -> fd 2 for a block: process-group setup prints its connection lines ("[Gloo] Rank 0 is
    connected to ...") from C++ onto stdout, where rank 0's one JSON line must stand alone."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def self_launch(a, argv):
    """`python bench.py --gpus N` (N > 1, WORLD_SIZE unset): start torch.distributed.run as a CHILD
    process -- before this process imports torch or libmk or touches a GPU -- let rank 0's JSON
    line through on the shared stdout and exit with the child's code.  Returns None when this
    process is itself a rank (or N = 1); raises when WORLD_SIZE contradicts --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus and not (a.leg or a.e2e_only):
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {a.gpus}: the launcher and the flag disagree")
        return None
    if a.gpus <= 1 or a.leg or a.e2e_only:
        return None
    import subprocess
    env = dict(os.environ, MK_BENCH_LAUNCHER="bench.py (torch.distributed.run child)")
    r = subprocess.run(launcher_cmd(a, argv, _free_port()), env=env)
    return r.returncode


def main():
    a = parse()
    rc = self_launch(a, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if a.leg:
        mk = importlib.import_module(PKG)
        which, sub = {"configs1": (1, None), "configs3": (3, None), "configs3_share7": (3, 7)}[a.leg]
        print(json.dumps(config_leg(mk, which, a.adapt_batches, a.warmup, a.steps, subsets=sub)), flush=True)
        return
    if a.e2e_only:
        mk = importlib.import_module(PKG)
        d = mk.synthetic.generate(a.n, q=1, n_test=a.n_test, seed=20250114)
        print(json.dumps(end_to_end(mk, d, a.subsets, tuple(int(x) for x in a.e2e_devices.split(",")))), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MK_BENCH_REHEARSE=1 (one-GPU boxes only): every rank on device 0, the process group on gloo, no
    # end-to-end leg -- runs the N-rank code path (launcher, sharding, barriers, max-over-ranks) where
    # only one GPU exists; the numbers are not a scaling measurement (the ranks share one GPU)
    rehearse = os.environ.get("MK_BENCH_REHEARSE") == "1" and world > 1
    if rehearse:
        local, a.no_e2e = 0, True
    K, n, n_test = a.subsets, a.n, a.n_test
    want_cpu = rank == 0 and world == 1 and not a.no_cpu_baseline
    host = host_cores() if want_cpu else None

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        with _stdout_to_stderr():
            dist.init_process_group("gloo" if rehearse else "nccl", rank=rank, world_size=world)
            cpu_group = dist.new_group(backend="gloo")   # waits that must not hold a GPU kernel
            dist.barrier()                               # the backend's communicator is created here
        if dist.get_world_size() != a.gpus:
            raise SystemExit(f"bench.py: torch.distributed sees {dist.get_world_size()} ranks, --gpus {a.gpus}")
    ranks_seen = dist.get_world_size() if dist is not None else 1

    mk = importlib.import_module(PKG)
    weak = a.scaling == "weak"
    dseed = 20250114 + (rank if weak else 0)      # weak: each rank's 500k sites are its own draw
    d = mk.synthetic.generate(n, q=1, n_test=n_test, seed=dseed)
    n_part, idx = mk.partition(n, K, seed=dseed)
    beta0, bt = mk.start_values(d["y"], d["x"], 1.0, 1, device=local if world > 1 else 0)
    dmod = importlib.import_module(PKG + ".distributed")
    if weak:
        lo, hi, base, per = 0, K, rank * K, K     # global subset indices rank*K ... (distinct Philox streams)
    else:
        lo, hi = dmod.shard_range(K, world, rank)
        base, per = lo, dmod.shard_capacity(K, world)
    # the chain first runs a.adapt_batches untimed amcmc batches (default 6: 300 iterations), so the
    # window sees adapted proposal scales like the 100-batch job does almost throughout (the first,
    # unadapted batch accepts phi ~0.6 of the time instead of ~0.43: more inverse work per step);
    # the end-to-end leg's whole-job average cross-checks the window's rate
    A = max(0, a.adapt_batches) * 50
    W = max(1, a.warmup) + A
    # amcmc batches of 50 as MK.R:57-58; the timed window holds burn-in and kept (kriging)
    # iterations in the reference's 3:1 ratio (burn.in = 0.75 n.samples, MK.R:85)
    n_burn_timed = int(round(0.75 * a.steps))
    burn_in = W + n_burn_timed + 1               # 1-based first kept iteration
    n_post = 5                                   # untimed post-window pass for the per-kernel breakdown
    n_batch = (W + a.steps + n_post + 49) // 50
    cfg = mk.SamplerConfig(1, 2, beta0, bt, n_batch=n_batch, batch_length=50, burn_in=burn_in, seed=20250114,
                           n_streams=a.streams)
    subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], 1, idx[i]) for i in range(lo, hi)]
    ses = mk.Session(subs, cfg, coords_test=d["coords_test"], subset_base=base, device=local if world > 1 else 0)
    la = ses.lookahead
    ses.run(W)                                    # warmup
    # the CPU baseline resumes the first chains from here: the state at the window's first iteration
    n_cpu = min(host["usable"], hi - lo) if want_cpu else 0
    cpu_states = [ses.chain_state(i) for i in range(n_cpu)]
    # timed window: HIP events bracket only the roofline kernel (the column-update launches) on its stream
    upd_kinds = [mk.session.KS_CHOL_UPDATE, mk.session.KS_CHOL_UPDATE_SUB]   # k_chol_update<128> + <64>/<32>
    ses.profile(not a.no_kernel_events, kinds=upd_kinds, every=a.event_every)

    def barrier():
        if dist is not None:
            dist.barrier()
            import torch
            torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    ses.run(a.steps)                              # returns after the device is idle
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    sts = [ses.kernel_stats(i) for i in upd_kinds]
    sub_share = sts[1]["launches"] / max(1, sts[0]["launches"] + sts[1]["launches"])
    # union of the update launches' event intervals: the split schedule (small shards) runs the
    # bulk and correction updates of a panel concurrently on two streams; each moment counts once
    st = ses.kernel_stats(mk.session.KS_UPDATE_BUSY)
    summed_ms = sts[0]["ms"] + sts[1]["ms"]
    sweep_fallbacks = ses.kernel_stats(mk.session.KS_SWEEP_FALLBACK)["launches"]
    # per-kernel breakdown: a separate untimed pass of n_post (kept) iterations, every kind evented
    kinds = [("chol_update", 0), ("chol_update_sub", 7), ("chol_diag", 1), ("chol_trsm", 2), ("w_sweep", 3),
             ("qblocks", 4), ("inverse", 6), ("cov_candidate", 10)]
    before = {name: ses.kernel_stats(i) for name, i in kinds}
    ses.profile(True)
    ses.run(n_post)
    kern = {name: {"ms": ses.kernel_stats(i)["ms"] - before[name]["ms"],
                   "flops": ses.kernel_stats(i)["flops"] - before[name]["flops"],
                   "launches": ses.kernel_stats(i)["launches"] - before[name]["launches"]} for name, i in kinds}
    dev_window = ses.outputs(quantiles=False, samples=True)["samples"][:n_cpu] if n_cpu else []
    ses.close()
    legs = {}
    if world == 1 and not a.no_legs:
        ls = max(40, a.steps)   # the legs' windows: 40 steps at least (a 20-step window of a small shard is noisy)
        legs["configs[2]_share32"] = shard_leg(mk, d, idx, min(a.shard_subsets, K), beta0, bt, a.adapt_batches, a.warmup, ls)
        legs["configs[1]_matern"] = config_leg(mk, 1, a.adapt_batches, a.warmup, ls)
        legs["configs[3]_lmc_share7"] = config_leg(mk, 3, a.adapt_batches, a.warmup, ls, subsets=7)
    e2e = None
    if world == 1 and not a.no_e2e:
        with _stdout_to_stderr():    # RCCL prints its version banner on stdout at communicator set-up
            e2e = end_to_end(mk, d, K, tuple(int(x) for x in a.e2e_devices.split(",")))
    if world == 1 and not a.no_legs:
        # the 1M-site kriging leg in a fresh process (bench_kriging.py: the same kriging_leg on 32
        # subsets of n_s = 2,000 from the same generator): sessions that follow one another in a process
        # can inherit the HIP runtime's queue state -- in-process, after the other legs
        # and the end-to-end leg, this leg read ~10 % low (16.9 vs 18.7-19.0 M draws/s)
        legs["configs[4]_kriging"] = kriging_leg_process(min(a.krig_subsets, K), a.krig_sites)
    elif world > 1 and not a.no_e2e and not weak:
        if rank == 0:
            e2e = node_end_to_end(a, world)
        dist.barrier(group=cpu_group)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    cpu = None
    if n_cpu:
        cfg_kw = dict(beta_starting=beta0, beta_tuning=bt, n_batch=cfg.n_batch, batch_length=50, burn_in=burn_in,
                      seed=20250114)
        cpu, cpu_window = cpu_baseline(subs, d["coords_test"], cfg_kw, cpu_states, W + a.steps, n_cpu)
        dev = np.stack([smp[W:W + a.steps] for smp in dev_window])
        cpu["window_max_abs_dev_vs_device"] = float(np.max(np.abs(np.stack(cpu_window) - dev)))
        cpu.update(host_nproc=host["nproc"], host_affinity=host["affinity"], cpu_model=host["model"],
                   cores_note=host["note"], host_physical_cores=physical_cores())
    K_job = K * world if weak else K
    value = K_job * a.steps / elapsed
    avg_ms = summed_ms / max(1, st["launches"])   # per-launch duration (what rocprofv3 reports)
    achieved = st["flops"] / (st["ms"] * 1e-3) / 1e12 if st["ms"] > 0 else 0.0
    metric = "MCMC iters/sec (all subsets, whole node) + end-to-end wall-clock, n=500k K=250"
    if weak and world > 1:   # a different (N x larger) job: not the headline metric
        metric = f"MCMC iters/sec (all subsets, whole node), weak scaling: n={n * world // 1000}k K={K_job}"
    out = {
        "metric": metric,
        "value": value,
        "unit": "subset-iters/s",
        "n_gpus": world,
        # what actually ran: the ranks torch.distributed saw (RCCL backend) and who started them
        "ranks_seen": ranks_seen,
        **({"rehearsal": "MK_BENCH_REHEARSE: every rank on GPU 0, gloo process group -- not a scaling measurement"}
           if rehearse else {}),
        "launcher": os.environ.get("MK_BENCH_LAUNCHER", "external torch.distributed.run" if world > 1 else "none"),
        "steps": a.steps,
        "warmup": W - A,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded binary GP field, RFF, SURVEY.md 8d generator)",
        "config": {"workload": (f"configs[2] per GPU (node job n={n * world}, K={K_job})" if weak else
                                f"configs[2] split over {world} GPU(s)") +
                               f": n={n}, K={K} subsets of {n // K}, exponential, q=1, "
                               f"n_test={n_test}, amcmc batches of 50, timed window {n_burn_timed} burn-in + "
                               f"{a.steps - n_burn_timed} kept (fused kriging, "
                               f"{'phi tables made at set-up' if os.environ.get('MK_KRIG_CHEB', '1') != '0' else 'exact X refresh'}"
                               f") iterations at iterations "
                               f"{W + 1}-{W + a.steps} (after {A} untimed adaptation + {W - A} warmup iterations)",
                   "subsets_per_gpu": per, "total_subsets": K_job, "streams_per_gpu": a.streams or 1,
                   "parallelism": f"subset-sharded x{world}"},
        "roofline": {"bound": "mfma", "kernel": "the column-update launches of the left-looking Cholesky (fp64 MFMA): "
                               "k_chol_update_trsm (column k's update of tiles k+1.. with the panel solve fused in "
                               "its epilogue, plus the next diagonal tile's update by panels < k) and, on the unfused "
                               "and split schedules, k_chol_update (128-tile and 64/32-sub-tile instances). The "
                               "fused schedule's rank-128 diagonal correction runs inside k_chol_diag (KS_CHOL_DIAG, "
                               "outside this union)",
                     "flops_definition": "algorithmic: off-diagonal tile updates 2*rows*cols*depth, the diagonal "
                                         "tile's update as a SYRK cols*(cols+1)*depth, the panel solve as a "
                                         "triangular solve rows*cols^2, every factor clipped to its valid extent "
                                         "n_s+1 (the kernels execute more: whole MFMA blocks of the triangles)",
                     "sub_tile_launch_share": sub_share,
                     "busy_ms_union": st["ms"], "launch_ms_summed": summed_ms,
                     "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS,
                     # PMC bytes per launch, profiled on the default workload (N=1, n=500k, K=250) only
                     "traffic": _pmc_traffic() if (world == 1 and K == 250 and n == 500_000) else None,
                     "avg_launch_ms": avg_ms, "launches": st["launches"],
                     "event_sampling": f"the launches of every {a.event_every}-th iteration of the timed window "
                                       f"bracketed by HIP events ({st['launches']} launches)",
                     "algorithmic_flops_per_launch": st["flops"] / max(1, st["launches"]),
                     "schedule": "lookahead" if la else "sequential",
                     "timing_note": ("update launches run beside the candidates' and main streams' other kernels "
                                     "(lookahead schedule, DESIGN.md 4.2): their union interval includes time "
                                     "shared with those kernels, so frac understates the kernel's own rate"
                                     if la else "update launches run alone on the stream (sequential schedule)")},
        "sweep_fallbacks": sweep_fallbacks,   # multi-workgroup sweep only: subsets refused admission
        # the second MFMA kernel: W = L^-1 of the accepted factors (k_inv_level), from the post-window pass
        "roofline_inverse": inverse_roofline(kern["inverse"]),
        "kernels_ms_per_step": {k: v["ms"] / n_post for k, v in kern.items()},
        "kernels_ms_per_step_note": f"untimed post-window pass of {n_post} iterations, every kernel kind evented",
        # the HBM-bound sub-phases in GB/s, on algorithmic bytes per subset-iteration --
        # the candidate's lower triangle written once (4 (n_s+1)^2 B), W read once by the sweep (4 n_s^2 B)
        "hbm_subphases": hbm_subphases(kern, n_post, [len(s_["coords"]) for s_ in subs]),
        "chain_iters_per_s": a.steps / elapsed,
        "end_to_end_estimate_s": elapsed / a.steps * 5000,
    }
    if legs:
        out["legs"] = legs
    if e2e is not None:
        if "phases" in e2e:
            out["end_to_end_s"] = e2e["phases"]["end_to_end_s"]
        out["end_to_end"] = e2e
    if cpu is not None:
        out["cpu_baseline"] = cpu
        out["gpu_over_cpu"] = value / cpu["value"]
        # the port is one process per core (no shared state): its rate scales with PHYSICAL cores (SMT
        # siblings share a core's FP64 units).  Projections, labelled as such -- the job's CPU share on
        # the box is cpu["cores"] cores
        phys = cpu.get("host_physical_cores") or cpu["host_nproc"]
        per_gpu_cores = max(1, phys // 8)
        out["cpu_projection"] = {
            "note": "linear in physical cores (independent subsets, one process per core); not measured beyond "
                    f"the job's {cpu['cores']}-core share",
            "per_gpu_share_cores": per_gpu_cores,
            "per_gpu_share_value": cpu["value"] * per_gpu_cores / cpu["cores"],
            "gpu_over_per_gpu_share": value / (cpu["value"] * per_gpu_cores / cpu["cores"]),
            "node_cores": phys,
            "node_value": cpu["value"] * phys / cpu["cores"],
        }
        if e2e is not None:
            # the CPU port's wall clock for the same 250 x 5,000 subset-iterations (chains only)
            out["cpu_projection"]["e2e_chains_s_at_node_cores"] = K * 5000 / out["cpu_projection"]["node_value"]
            out["cpu_projection"]["e2e_chains_s_at_job_share"] = K * 5000 / cpu["value"]
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
