"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into profiles/pmc_chol_update.json.

usage: python tools/pmc_summary.py <fetch_pass_dir> <write_pass_dir> <out.json> "<command profiled>" [kernel]

[kernel] (default "mk::k_chol_update,mk::k_chol_update_trsm") is a comma-separated list of names:
each name's template instances (k_chol_update<128>, <64>, ...) and the names themselves are folded
into one launch-weighted entry (bench.py's roofline kernel: every column-update launch).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of
16-B/lane coalesced reads -> x2; WRITE_SIZE as reported.  Both are in KB -> x1024.
bench.py reads hbm_bytes_per_launch of KERNEL for roofline.traffic.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "mk::k_chol_update,mk::k_chol_update_trsm"


def _per_kernel(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: [0, 0.0])
    with open(path[0]) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0]
            if name.startswith("void "):
                name = name[5:]
            acc[name][0] += 1
            acc[name][1] += float(row["Counter_Value"])
    return {k: (n, s / n) for k, (n, s) in acc.items()}


def main():
    fetch_dir, write_dir, out, cmd = sys.argv[1:5]
    fetch = _per_kernel(fetch_dir, "FETCH_SIZE")
    write = _per_kernel(write_dir, "WRITE_SIZE")
    allk = {}
    for k in sorted(set(fetch) | set(write)):
        fn, fkb = fetch.get(k, (0, 0.0))
        wn, wkb = write.get(k, (0, 0.0))
        allk[k] = {"launches": max(fn, wn), "fetch_kb_avg": fkb, "write_kb_avg": wkb,
                   "hbm_bytes_per_launch_corrected": (2.0 * fkb + wkb) * 1024.0}
    kernel = sys.argv[5] if len(sys.argv) > 5 else KERNEL
    names = kernel.split(",")
    inst = {k: v for k, v in allk.items() if any(k == nm or k.startswith(nm + "<") for nm in names)}
    if not inst:
        raise SystemExit(f"{kernel} not in the profile")
    n = sum(v["launches"] for v in inst.values())
    main_k = {"launches": n}
    for f in ("fetch_kb_avg", "write_kb_avg", "hbm_bytes_per_launch_corrected"):
        main_k[f] = sum(v[f] * v["launches"] for v in inst.values()) / n
    doc = {"kernel": kernel, "instances": sorted(inst), "command": cmd,
           "correction": "gfx950: FETCH_SIZE counts half the bytes of 16-B/lane coalesced reads "
                         "(MI355X_MICROARCH.md HBM section) -> x2; WRITE_SIZE as reported; units KB -> x1024",
           "fetch_kb_per_launch": main_k["fetch_kb_avg"], "write_kb_per_launch": main_k["write_kb_avg"],
           "hbm_bytes_per_launch": main_k["hbm_bytes_per_launch_corrected"], "launches": main_k["launches"],
           "all_kernels": allk}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"{kernel}: {doc['hbm_bytes_per_launch'] / 1e9:.3f} GB per launch over {doc['launches']} launches")


if __name__ == "__main__":
    main()
