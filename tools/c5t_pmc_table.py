"""Counters of tools/c5t_stride_probe.py's variants from rocprofv3 --pmc passes.

Each pass directory holds the counter_collection (and kernel_trace) CSVs of
`c5t_stride_probe.py --rounds 1 --reps R --variants v1,v2,...`: per variant
2 warm-up dispatches then R timed ones, in variant order.  Prints, per
variant, the median over its timed dispatches of every counter (and of the
kernel duration when the trace is there), plus the ratio to the first variant.

    python tools/c5t_pmc_table.py --variants dense,s+4KiB --reps 3 gpurun_out/r06b_pmc_1 [...]
"""
import argparse
import csv
import glob
import os

import numpy as np


def one_pass(d, variants, reps, kernel="k_transpose"):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    ctr, names = {}, {}
    for r in csv.DictReader(open(cc[0])):
        di = int(r["Dispatch_Id"])
        ctr.setdefault(di, {})
        ctr[di][r["Counter_Name"]] = ctr[di].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[di] = r.get("Kernel_Name", "")
    dur = {}
    if tr:
        for r in csv.DictReader(open(tr[0])):
            di = int(r["Dispatch_Id"])
            dur[di] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            names.setdefault(di, r["Kernel_Name"])
    ds = sorted(di for di in names if kernel in names[di])
    per = 2 + reps
    out = {}
    for i, v in enumerate(variants):
        timed = ds[i * per + 2:(i + 1) * per]
        row = {}
        for c in sorted({c for di in timed for c in ctr.get(di, {})}):
            row[c] = float(np.median([ctr[di][c] for di in timed if c in ctr.get(di, {})]))
        if dur:
            row["ms"] = float(np.median([dur[di] for di in timed if di in dur]))
        out[v] = row
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kernel", default="k_transpose")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    vs = a.variants.split(",")
    rows = {v: {} for v in vs}
    for d in a.dirs:
        for v, r in one_pass(d, vs, a.reps, a.kernel).items():
            for c, x in r.items():
                rows[v].setdefault(c, x)
    cols = sorted({c for r in rows.values() for c in r}, key=lambda c: (c != "ms", c))
    print("| counter (median of the timed dispatches) | " + " | ".join(vs) + " |")
    print("|---" * (len(vs) + 1) + "|")
    for c in cols:
        base = rows[vs[0]].get(c)
        cells = []
        for v in vs:
            x = rows[v].get(c)
            if x is None:
                cells.append("-")
            elif v == vs[0] or not base:
                cells.append("%.4g" % x)
            else:
                cells.append("%.4g (%.2fx)" % (x, x / base))
        print("| %s | %s |" % (c, " | ".join(cells)))


if __name__ == "__main__":
    main()
