"""Counters per call of tools/c2_order_probe.py under rocprofv3 --pmc: every
k_transpose dispatch in order is (placement j, build k, call c) with 2 warm-ups
+ reps timed calls per (j, k); prints the timed calls' medians per (j, k).

    python tools/c2_order_pmc_table.py gpurun_out/r03zj_pmc_1 [--k 6] [--reps 3]
"""
import argparse
import csv
import glob
import os
from collections import OrderedDict

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pass_dir")
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    trace = glob.glob(os.path.join(a.pass_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    cc = glob.glob(os.path.join(a.pass_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    dur, names = {}, {}
    for r in csv.DictReader(open(trace)):
        d = int(r["Dispatch_Id"])
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        names[d] = r["Kernel_Name"]
    ctr = OrderedDict()
    for r in csv.DictReader(open(cc)):
        d = int(r["Dispatch_Id"])
        ctr.setdefault(d, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        names.setdefault(d, r.get("Kernel_Name", ""))
    cnames = sorted({c for v in ctr.values() for c in v})
    ds = sorted(d for d in names if "k_transpose" in names[d])
    per = 2 + a.reps
    print("%3s %-9s %9s  %s" % ("pl", "order", "ms", "  ".join("%16s" % c[:16] for c in cnames)))
    for j in range(a.k):
        for k, label in enumerate(("in-order", "staggered")):
            base = (j * 2 + k) * per
            timed = ds[base + 2:base + per]
            ms = np.median([dur.get(d, np.nan) for d in timed])
            vals = [np.median([ctr.get(d, {}).get(c, np.nan) for d in timed]) for c in cnames]
            print("%3d %-9s %9.4f  %s" % (j, label, ms, "  ".join("%16.4g" % v for v in vals)))


if __name__ == "__main__":
    main()
