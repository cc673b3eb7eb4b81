"""Table of the placement study's counters (tools/gpu_placement_counters.sh).

Reads one rocprofv3 pass directory (counter_collection + kernel_trace CSVs of
`alloc_kind_probe.py --matrix K --rounds 1 --reps 1 --ops c5_T,c5_pack`),
assigns every dispatch of the studied kernels to its (op, source, destination)
pair by dispatch order (per op: K*K pairs x 2 warm-ups, then K*K timed
calls), and prints each timed call's duration with its counters.

    python tools/placement_pmc_table.py gpurun_out/r03h_pmc_1 [--k 4]
"""
import argparse
import csv
import glob
import os
from collections import OrderedDict

KERNELS = (("c5_T", "k_transpose"), ("c5_pack", "k_recmap"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pass_dir")
    ap.add_argument("--k", type=int, default=4)
    a = ap.parse_args()
    K = a.k
    trace = glob.glob(os.path.join(a.pass_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    cc = glob.glob(os.path.join(a.pass_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    dur = {}
    names = {}
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
    print("%-8s %3s %3s %9s  %s" % ("op", "src", "dst", "ms", "  ".join("%14s" % c[:14] for c in cnames)))
    for op, sub in KERNELS:
        ds = sorted(d for d in names if sub in names[d])
        timed = ds[2 * K * K:3 * K * K]
        for n, d in enumerate(timed):
            i, j = divmod(n, K)
            c = ctr.get(d, {})
            print("%-8s %3d %3d %9.4f  %s" % (op, i, j, dur.get(d, float("nan")),
                                             "  ".join("%14.4g" % c.get(x, float("nan")) for x in cnames)))


if __name__ == "__main__":
    main()
