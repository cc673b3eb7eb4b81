"""Per library launch: duration, GRBM_COUNT / GRBM_GUI_ACTIVE and the clock
they imply (counts / duration), from rocprofv3 --pmc csv directories.

    python tools/clock_pmc_table.py DIR [DIR ...]
"""
import csv
import glob
import os
import sys


def rows(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not f:
        return []
    out = {}
    for r in csv.DictReader(open(f[0])):
        k = r["Dispatch_Id"]
        e = out.setdefault(k, {"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]),
                                "end": int(r["End_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return sorted(out.values(), key=lambda e: e["start"])


for d in sys.argv[1:]:
    print("==", d)
    for e in rows(d):
        if "k_" not in e["name"]:
            continue
        ms = (e["end"] - e["start"]) / 1e6
        if ms < 0.05:
            continue
        c, a = e.get("GRBM_COUNT", 0.0), e.get("GRBM_GUI_ACTIVE", 0.0)
        print("%-45s %8.4f ms  COUNT %.4g (%.0f MHz)  GUI_ACTIVE %.4g (%.0f MHz)" % (
            e["name"].split("(")[0][-45:], ms, c, c / (ms * 1e3), a, a / (ms * 1e3)))
