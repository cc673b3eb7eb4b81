"""The C2 step's host turnarounds on one timeline (diagnostic, one GPU): run
under `rocprofv3 --hip-trace --kernel-trace --output-format csv`, then
`--analyze DIR` lines up each statistic kernel's end with the HIP calls
after it (the synchronize that returns, the next launch) and the next
kernel's start, per step.

    rocprofv3 --hip-trace --kernel-trace -d gpurun_out/gap -o run --output-format csv -- python tools/c2_gap_trace.py
    python tools/c2_gap_trace.py --analyze gpurun_out/gap
"""
import glob
import os
import statistics
import sys


def run(steps=30):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np
    import torch
    import bolt_amd as bolt
    from bolt_amd import MI355XContext
    dev = torch.device("cuda", 0)
    ctx = MI355XContext(device=dev)
    shape = (2000, 512, 512)
    x = torch.randn(shape, device=dev).mul_(50).add_(1000)
    b = bolt.ConstructMI355X.fromshards(x, shape, context=ctx, split=1, dtype=np.float32)
    del x
    for _ in range(steps):
        s = b.swap((0,), (0, 1))
        s.mean(axis=2)
        s.std(axis=2)
    torch.cuda.synchronize()


def analyze(d):
    import csv
    kt = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    ht = sorted(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True))[0]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kt))]
    hs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(ht))]
    ks.sort()
    hs.sort()
    lib = [k for k in ks if "k_red_rows" in k[2] or "k_transpose" in k[2]]
    out = {"wake": [], "host": [], "launch": [], "dispatch": [], "gap": []}
    for i in range(len(lib) - 1):
        s0, e0, n0 = lib[i]
        s1, e1, n1 = lib[i + 1]
        if "k_red_rows" not in n0:
            continue
        # the synchronize that returns after this kernel's end, the next launch call
        sync = [h for h in hs if "Synchronize" in h[2] and h[1] >= e0 and h[0] <= e0]
        launch = [h for h in hs if h[2].startswith("hipLaunchKernel") or h[2] == "hipExtLaunchKernel"]
        launch = [h for h in launch if h[0] >= e0 and h[1] <= s1]
        if not sync or not launch:
            continue
        out["wake"].append((sync[0][1] - e0) / 1e3)
        out["host"].append((launch[-1][0] - sync[0][1]) / 1e3)
        out["launch"].append((launch[-1][1] - launch[-1][0]) / 1e3)
        out["dispatch"].append((s1 - launch[-1][1]) / 1e3)
        out["gap"].append((s1 - e0) / 1e3)
    for k, v in out.items():
        if v:
            print("%-9s median %7.2f us  (n=%d, min %.2f, max %.2f)" % (k, statistics.median(v), len(v), min(v), max(v)))
    names = {}
    for h in hs:
        names[h[2]] = names.get(h[2], 0) + 1
    print("HIP calls:", sorted(names.items(), key=lambda kv: -kv[1])[:15])


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
