#!/usr/bin/env python3
"""Experiment: the 32-subset share (the per-GPU work of an 8-GPU run of configs[2]) as G concurrent
sessions of 32/G subsets on one GPU, one host thread each (ctypes releases the GIL inside
mk_session_run), against one session of 32.  Each session keeps its own lookahead pipeline; the
chains are the one-session chains (global subset indices).  Same window as bench.py's share leg:
300 adaptation + 3 warmup iterations, then `--steps` timed with the 3:1 burn-in : kept split.

    GPU_MAX_HW_QUEUES=16 python tools/two_sessions.py --groups 2
"""
import argparse
import importlib
import json
import os
import sys
import threading
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--subsets", type=int, default=32)
    ap.add_argument("--n", type=int, default=64000)
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    mk = importlib.import_module(PKG)
    d = mk.synthetic.generate(a.n, q=1, n_test=1000, seed=20250114)
    _, idx = mk.partition(a.n, 250 if a.n >= 500_000 else a.n // 2000, seed=20250114)
    beta0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)
    S, G = a.subsets, a.groups
    W = 303
    n_burn = int(round(0.75 * a.steps))
    cfg = mk.SamplerConfig(1, 2, beta0, bt, n_batch=(W + a.steps + 49) // 50, batch_length=50,
                           burn_in=W + n_burn + 1, seed=20250114)
    subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], 1, idx[i]) for i in range(S)]
    bounds = [(g * S // G, (g + 1) * S // G) for g in range(G)]
    sessions = [mk.Session(subs[lo:hi], cfg, coords_test=d["coords_test"], subset_base=lo) for lo, hi in bounds]
    go = threading.Barrier(G + 1)
    done = threading.Barrier(G + 1)
    err = []

    def worker(ses):
        try:
            ses.run(W)
            go.wait()
            ses.run(a.steps)
            done.wait()
        except Exception as e:   # noqa: BLE001
            err.append(repr(e))
            go.abort()
            done.abort()

    th = [threading.Thread(target=worker, args=(s_,)) for s_ in sessions]
    for t in th:
        t.start()
    go.wait()
    t0 = time.perf_counter()
    done.wait()
    el = time.perf_counter() - t0
    for t in th:
        t.join()
    la = [s_.lookahead for s_ in sessions]
    samples = [s_.outputs(quantiles=False, samples=True)["samples"] for s_ in sessions]
    for s_ in sessions:
        s_.close()
    if err:
        raise SystemExit(err)
    print(json.dumps({"groups": G, "subsets": S, "value": S * a.steps / el, "ms_per_step": el / a.steps * 1e3,
                      "lookahead": la, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      "sample_checksum": float(sum(np.sum(x) for x in samples))}), flush=True)


if __name__ == "__main__":
    main()
