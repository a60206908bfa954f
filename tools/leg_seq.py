"""Diagnostic: bench legs run one after another in one process (bench.py's window legs), to find
which earlier work slows a later leg.  python tools/leg_seq.py c1 c1 s32 c1 k c1"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import numpy as np  # noqa: E402
import bench  # noqa: E402

import importlib  # noqa: E402

mk = importlib.import_module(bench.PKG)
for tag in sys.argv[1:]:
    if tag == "c1":
        r = bench.config_leg(mk, 1, 6, 3, 40)
    elif tag == "c3":
        r = bench.config_leg(mk, 3, 6, 3, 40, subsets=7)
    elif tag == "s32":
        d = mk.synthetic.generate(64_000, q=1, n_test=1000, seed=20250114)
        _, idx = mk.partition(64_000, 32, seed=20250114, method="R")
        b0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)
        r = bench.shard_leg(mk, d, idx, 32, b0, bt, 6, 3, 40)
    elif tag == "h":
        d = mk.synthetic.generate(500_000, q=1, n_test=1000, seed=20250114)
        _, idx = mk.partition(500_000, 250, seed=20250114, method="R")
        b0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)
        r = bench.shard_leg(mk, d, idx, 250, b0, bt, 6, 3, 20)
    elif tag == "k100":   # the kriging leg with 100,000 sites (a tenth of the buffers)
        import bench_kriging
        d = mk.synthetic.generate(64_000, q=1, n_test=1000, seed=20250114)
        _, idx = mk.partition(64_000, 32, seed=20250114, method="R")
        b0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)
        sites = np.random.default_rng(20250115).uniform(size=(100_000, 2))
        subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], 1, idx[i]) for i in range(32)]
        r = bench_kriging.kriging_leg(mk, subs, sites, b0, bt)
    elif tag == "k":
        import bench_kriging
        d = mk.synthetic.generate(64_000, q=1, n_test=1000, seed=20250114)
        _, idx = mk.partition(64_000, 32, seed=20250114, method="R")
        b0, bt = mk.start_values(d["y"], d["x"], 1.0, 1)
        sites = np.random.default_rng(20250115).uniform(size=(1_000_000, 2))
        subs = [mk.subset_data(d["y"], d["x"], 1.0, d["coords"], 1, idx[i]) for i in range(32)]
        r = bench_kriging.kriging_leg(mk, subs, sites, b0, bt)
    print(tag, round(r["value"]), r.get("ms_per_step"), flush=True)
