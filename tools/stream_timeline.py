"""Multi-stream timeline of MCMC iterations from a rocprofv3 kernel trace (SQLite output).

    rocprofv3 --kernel-trace -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline ...
    python tools/stream_timeline.py gpurun_out/prof/run_results.db [first_iteration] [n_iterations]

The lookahead schedule runs the candidates' factorisation on its own stream beside the main
stream, so a per-launch list in start order with the hardware queue of each launch is what shows
the critical path.  Iterations are delimited by `k_theta_mh` launches (one per iteration on the
exponential model).  Prints, per iteration: the span between decisions, busy time per queue, the
launches in start order (relative start, duration, queue, workgroups), and the idle gaps of the
GPU (no kernel on any queue).
"""
import collections
import re
import sqlite3
import subprocess
import sys


def load(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
    qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else "0")
    gx = "grid_size_x" if "grid_size_x" in cols else "0"
    wx = "workgroup_size_x" if "workgroup_size_x" in cols else "1"
    rows = c.execute(f"select s.kernel_name, k.start, k.end, k.{qcol}, k.{gx}, k.{wx} from rocpd_kernel_dispatch k "
                     "join rocpd_info_kernel_symbol s on k.kernel_id = s.id order by k.start").fetchall()
    names = sorted({r[0] for r in rows})
    dm = subprocess.run(["c++filt"], input="\n".join(n.replace(".kd", "") for n in names), capture_output=True,
                        text=True, check=True).stdout.splitlines()
    dm = dict(zip(names, dm))
    short = lambda n: re.sub(r"\(.*", "", dm[n]).replace("void ", "").replace("mk::", "")
    return [(short(r[0]), r[1], r[2], r[3], (r[4] // max(r[5], 1)) if r[5] else r[4]) for r in rows]


def main(db, first=12, n_it=2):
    seq = load(db)
    dec = [i for i, s in enumerate(seq) if s[0] == "k_theta_mh"]
    if len(dec) < first + n_it + 1:
        sys.exit(f"only {len(dec)} decisions in the trace")
    spans = [(seq[dec[i + 1]][2] - seq[dec[i]][2]) / 1e3 for i in range(len(dec) - 1)]
    print("decision-to-decision spans (us):", " ".join(f"{x:.0f}" for x in spans))
    for it in range(first, first + n_it):
        t0, t1 = seq[dec[it]][2], seq[dec[it + 1]][2]
        win = [s for s in seq if s[2] > t0 and s[1] < t1]
        busy = collections.defaultdict(float)
        for name, a, b, q, wg in win:
            busy[q] += (min(b, t1) - max(a, t0)) / 1e3
        print(f"\niteration {it}: span {(t1 - t0) / 1e3:.1f} us; busy per queue (us): " +
              ", ".join(f"q{q} {v:.0f}" for q, v in sorted(busy.items())))
        # GPU idle: union of kernel intervals
        iv = sorted((max(a, t0), min(b, t1)) for _, a, b, _, _ in win)
        idle, cur = 0.0, t0
        for a, b in iv:
            if a > cur:
                idle += (a - cur) / 1e3
            cur = max(cur, b)
        idle += max(0, t1 - cur) / 1e3
        print(f"  no kernel running for {idle:.1f} us")
        for name, a, b, q, wg in win:
            print(f"  {(a - t0) / 1e3:8.1f} {(b - a) / 1e3:7.1f}  q{q}  wg={wg:<6d} {name[:60]}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
