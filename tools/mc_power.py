"""Power of the Monte Carlo-error parity test (tests/test_stat_cfg2_cfg4.py) against perturbed
targets on the device: for each perturbation, the criteria and the statistics of the device's
replicates 1..15 against the independent oracle replicates.  Run on a GPU box:
    python tools/mc_power.py > mc_power.json"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_stat_cfg2_cfg4 as t  # noqa: E402

mk = importlib.import_module(t.PKG)
out = []
for case in ("cfg3_exp", "cfg4_lmc"):
    ind = t._load_indep(case)
    perts = [None, ("phi_b", 10.0), ("phi_b", 8.0), ("iw_s", 0.2), ("iw_s", 1.0)]
    if len(sys.argv) > 1:   # e.g. phi_b:6,phi_b:7
        perts = [None] + [(k, float(v)) for k, v in (x.split(":") for x in sys.argv[1].split(","))]
    for pert in perts:
        _, _, res, res2 = t._device_replicates(mk, case, perturb=pert)
        ok, (tp, frac, mt2) = t._mc_criteria(ind, res, res2)
        rec = {"case": case, "perturb": pert, "criteria_pass": ok, "max_abs_t_param": float(np.max(np.abs(tp))),
               "t_param": np.round(tp, 2).tolist(), "w_frac_gt_3.5": frac, "w_mean_t2": mt2}
        out.append(rec)
        print(json.dumps(rec), flush=True)
