"""Helper run as a subprocess by tests/test_gpu_node.py (not a test module): mk_meta_fit over
device 0 in a fresh process must use an RCCL communicator (a group of one) and equal one session
followed by the sequential combine bit for bit.  Prints one JSON line."""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mk = importlib.import_module("laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd")


def main():
    d = mk.synthetic.generate(300, q=1, n_test=7, seed=21)
    subs = [dict(coords=d["coords"][i * 100:(i + 1) * 100], y=d["y"][i * 100:(i + 1) * 100], weights=np.ones(100),
                 x=d["x"][i * 100:(i + 1) * 100]) for i in range(3)]
    cfg = mk.SamplerConfig(1, 2, np.zeros(2), np.full(2, 0.05), n_batch=2, batch_length=3, burn_in=4, seed=8)
    got = mk.meta_fit_node(subs, cfg, coords_test=d["coords_test"], devices=[0])
    with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
        ses.run(cfg.n_samples)
        ref = ses.outputs()
    exact = (np.array_equal(got["result"], mk.combine(ref["parameters"])) and
             np.array_equal(got["result2"], mk.combine(ref["w_predict"])))
    print(json.dumps({"exchange": got["exchange"], "exact": bool(exact)}), flush=True)


if __name__ == "__main__":
    main()
