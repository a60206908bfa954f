"""Per-launch timeline of one MCMC iteration from a rocprofv3 kernel trace (SQLite output).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
    python tools/iter_timeline.py gpurun_out/prof/run_results.db [iteration]

Iterations are delimited by `k_beta` launches (the first kernel of run_iteration).  Prints every
launch of the chosen iteration (duration, workgroups) and the per-kernel time averaged over the
iterations after the first eight (warmup, initial factorisation).
"""
import collections
import re
import sqlite3
import sys


def main(db, it=10):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, duration, grid_x, workgroup_x from kernels order by start").fetchall()
    short = lambda n: re.sub(r"\(.*", "", n).replace("void ", "").replace("mk::", "")
    seq = [(short(r[0]), r[2] / 1e3, r[3] // max(r[4], 1), r[1]) for r in rows]
    starts = [i for i, s in enumerate(seq) if s[0] == "k_beta"]
    if len(starts) < 2:
        sys.exit("fewer than two iterations in the trace")
    it = min(it, len(starts) - 2)
    a, b = starts[it], starts[it + 1]
    span = (seq[b][3] - seq[a][3]) / 1e3
    busy = sum(s[1] for s in seq[a:b])
    print(f"iteration {it}: span {span:.1f} us, kernel time {busy:.1f} us, gaps {span - busy:.1f} us, {b - a} launches")
    for name, us, wg, _ in seq[a:b]:
        print(f"  {name:28s} {us:9.1f} us  wg={wg}")
    lo = min(8, len(starts) - 2)
    n = len(starts) - 1 - lo
    agg = collections.defaultdict(float)
    for x, y in zip(starts[lo:-1], starts[lo + 1:]):
        for name, us, _, _ in seq[x:y]:
            agg[name] += us / n
    print(f"mean per iteration over {n} iterations (us):")
    for name, us in sorted(agg.items(), key=lambda kv: -kv[1]):
        print(f"  {name:28s} {us:9.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
