"""Per-phase timing of the multi-workgroup latent sweep (k_sweep_mg), development probe.

Builds a probe variant of libmk (-DMK_SWEEP_PROBE: the last tile's workgroup of subset 0 stamps
wall_clock64 -- 100 MHz -- at each phase of every block) into tools/libmk_probe.so, runs a
configs[2]-sized shard of S subsets for a few iterations and prints the mean phase durations:
  0->1 partial dots + stores     1->2 Q_BB prefetch     2->3 barrier wait
  3->4 partial sums              4->5 MH steps          5->next 0 z update
    python tools/sweep_probe.py [S]       (on the GPU box; build here first: --build)
"""
import importlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd"
PROBE = os.path.join(ROOT, "tools", "libmk_probe.so")


def build():
    sys.path.insert(0, ROOT)
    b = importlib.import_module(PKG + "._build")
    objs = []
    for src in b.SOURCES:
        obj = os.path.join("/tmp", "probe_" + os.path.splitext(src)[0] + ".o")
        subprocess.check_call(["/opt/rocm/bin/hipcc"] + b.FLAGS + ["-DMK_SWEEP_PROBE", "-c", os.path.join(b.CSRC, src),
                                                                  "-o", obj])
        objs.append(obj)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", PROBE] + objs)


def main(S):
    import ctypes
    os.environ["MK_LIB"] = PROBE
    sys.path.insert(0, ROOT)
    mk = importlib.import_module(PKG)
    lib = mk.load()
    n = 2000 * S
    d = mk.synthetic.generate(n, q=1, n_test=100, seed=3)
    cfg = mk.SamplerConfig(1, 2, [0.5, -0.5], [0.01, 0.01], n_batch=1, batch_length=10, burn_in=8)
    subs = [dict(coords=d["coords"][i * 2000:(i + 1) * 2000], y=d["y"][i * 2000:(i + 1) * 2000],
                 weights=np.ones(2000), x=d["x"][i * 2000:(i + 1) * 2000]) for i in range(S)]
    with mk.Session(subs, cfg, coords_test=d["coords_test"]) as ses:
        ses.run(6)
    ts = (ctypes.c_longlong * 512)()
    lib.mk_debug_sweep_probe.restype = ctypes.c_int
    assert lib.mk_debug_sweep_probe(ts) == 0
    a = np.array(ts[:], dtype=np.int64).reshape(64, 8)[:32, :6] / 100.0     # microseconds (100 MHz)
    ph = np.diff(a, axis=1)
    nxt = a[1:, 0] - a[:-1, 5]
    names = ["dots+store", "Q prefetch", "barrier", "sums", "MH"]
    print(f"S={S}: per block (us), mean over 32 blocks of the last sweep")
    for k, nm in enumerate(names):
        print(f"  {nm:12s} {ph[:, k].mean():7.2f}  (block 0 {ph[0, k]:.2f}, block 31 {ph[31, k]:.2f})")
    print(f"  {'z update':12s} {nxt.mean():7.2f}")
    print(f"  total per block {(a[31, 5] - a[0, 0]) / 31:.2f}")


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
