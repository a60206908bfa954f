"""Per-kernel statistics (rocprofv3 --stats layout) from a rocprofv3 kernel-trace database.

    python tools/db_stats.py gpurun_out/<dir>/run_results.db > profiles/<name>_kernel_stats.csv

rocprofv3 7.x writes the kernel trace to SQLite (rocpd) by default; this folds its
kernel-dispatch table into Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs
(template instances kept apart, as rocprofv3 names them)."""
import csv
import sqlite3
import subprocess
import sys
from collections import defaultdict


def _demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(n.replace(".kd", "") for n in names), capture_output=True,
                         text=True, check=True).stdout.splitlines()
    return dict(zip(names, out))


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select s.kernel_name, k.end - k.start from rocpd_kernel_dispatch k "
                     "join rocpd_info_kernel_symbol s on k.kernel_id = s.id").fetchall()
    dm = _demangle(sorted({r[0] for r in rows}))
    agg = defaultdict(list)
    for name, dur in rows:
        agg[dm[name].split("(")[0].replace("void ", "")].append(dur)
    total = sum(sum(v) for v in agg.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
