"""Per-kernel statistics from a rocprofv3 kernel trace, every call and the
timed calls only.

rocprofv3 --stats averages every dispatch of a kernel, the warm-up calls
included; the first call of an op writes a freshly allocated destination
and pays its first-touch cost (profiles/r03a_spread_c5.log: C5 chunk 10.9 ms
on the first call, 3.31 ms after).  This prints both views, in dispatch order,
per kernel name (template arguments kept), and for each kernel the per-call
durations so a slow call can be located.

    python tools/trace_stats.py gpurun_out/prof_r03d_C5/run_kernel_trace.csv [--skip N] [--match k_]
"""
import argparse
import csv
from collections import OrderedDict


def short(name):
    """Kernel name without the argument list ('void k_x<...>(args)' -> 'k_x<...>')."""
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=1, help="leading calls per kernel treated as warm-up")
    ap.add_argument("--match", default="k_", help="only kernels whose short name contains this")
    ap.add_argument("--calls", action="store_true", help="print every call's duration")
    a = ap.parse_args()
    calls = OrderedDict()
    for row in csv.DictReader(open(a.trace)):
        k = short(row["Kernel_Name"])
        if a.match not in k:
            continue
        calls.setdefault(k, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    print("%-60s %6s %10s %10s %10s %10s" % ("kernel", "calls", "avg_all_ms", "avg_timed", "min_ms", "max_ms"))
    for k, v in calls.items():
        timed = v[a.skip:] if len(v) > a.skip else v
        print("%-60s %6d %10.4f %10.4f %10.4f %10.4f" % (k[:60], len(v), sum(v) / len(v), sum(timed) / len(timed),
                                                        min(v), max(v)))
        if a.calls:
            print("    " + " ".join("%.3f" % x for x in v))


if __name__ == "__main__":
    main()
