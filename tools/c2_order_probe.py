"""C2 transpose: the in-order and the staggered tile walk (DESIGN.md §3,
placement-adaptive order) on K placements, for the counter study of the two
placement classes.

Two builds are loaded side by side (BM_TR_AROT=0: always in order;
BM_TR_AROT_FORCE=1: always staggered).  Per placement j and build k (k
fastest): 2 warm-up calls, then `reps` timed calls.  Under rocprofv3 --pmc,
dispatch order identifies each call (tools/c2_order_pmc_table.py).

    python tools/c2_order_probe.py inorder.so stagger.so [--k 6] [--reps 3]
"""
import argparse
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from ab_bench import load, Permute  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    libs = [load(p) for p in a.libs]
    ops = [Permute((2000, 512 * 512), (1, 0), np.float32) for _ in range(a.k)]
    for j, op in enumerate(ops):
        ms = []
        for k, lib in enumerate(libs):
            for _ in range(2):
                op(lib)
            t = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                op(lib)
                e1.record()
                e1.synchronize()
                t.append(e0.elapsed_time(e1))
            ms.append(float(np.median(t)))
        cls = "staggered-class" if ms[1] < 0.99 * ms[0] else "in-order-class"
        print("placement %d  in-order %.4f ms  staggered %.4f ms  %s" % (j, ms[0], ms[1], cls), flush=True)


if __name__ == "__main__":
    sys.exit(main())
