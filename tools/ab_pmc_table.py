"""Counters per op and library of an ab_bench.py run under rocprofv3 --pmc.

ab_bench.py with L libraries, --rounds 1 --reps 1 dispatches, per op, 2
warm-up calls of every library, then one timed call of every library (in the
order given); every call launches one kernel whose name contains --kernel.
Prints per op the timed calls' counters (and kernel time if the pass has a
kernel trace), one column per library.

    python tools/ab_pmc_table.py --ops c2_mean_prow,c2_std_prow --libs base,peel --kernel k_red_rows DIR [DIR ...]
"""
import argparse
import csv
import glob
import os


def one_pass(d, ops, nl, kernel):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    ctr, names, dur = {}, {}, {}
    for r in csv.DictReader(open(cc)):
        di = int(r["Dispatch_Id"])
        ctr.setdefault(di, {})
        ctr[di][r["Counter_Name"]] = ctr[di].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[di] = r.get("Kernel_Name", "")
    if tr:
        for r in csv.DictReader(open(tr[0])):
            di = int(r["Dispatch_Id"])
            dur[di] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            names.setdefault(di, r["Kernel_Name"])
    ds = sorted(di for di in names if kernel in names[di])
    per = 3 * nl
    out = {}
    for i, op in enumerate(ops):
        timed = ds[i * per + 2 * nl:(i + 1) * per]
        for k, di in enumerate(timed):
            row = dict(ctr.get(di, {}))
            if di in dur:
                row["ms"] = dur[di]
            out[(op, k)] = row
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", required=True)
    ap.add_argument("--libs", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    ops, libs = a.ops.split(","), a.libs.split(",")
    rows = {}
    for d in a.dirs:
        for key, r in one_pass(d, ops, len(libs), a.kernel).items():
            for c, x in r.items():
                rows.setdefault(key, {}).setdefault(c, x)
    cols = sorted({c for r in rows.values() for c in r}, key=lambda c: (c != "ms", c))
    print("| op | counter | " + " | ".join(libs) + " |")
    print("|---" * (len(libs) + 2) + "|")
    for op in ops:
        for c in cols:
            print("| %s | %s | %s |" % (op, c, " | ".join("%.5g" % rows.get((op, k), {}).get(c, float("nan"))
                                                          for k in range(len(libs)))))


if __name__ == "__main__":
    main()
