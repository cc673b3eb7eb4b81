"""Host-side cost of the C2 step's calls on the GPU (diagnostic).

Times each call (swap, mean, std) with perf_counter around call + sync,
against the kernel time from hipEvents, and profiles the Python side.
"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402


def main():
    ctx = bolt.MI355XContext()
    shape = (2000, 512, 512)
    raw = (torch.randn(int(np.prod(shape)), device="cuda") * 50 + 1000).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=1, dtype=np.float32)
    s = b.swap((0,), (0, 1))
    for _ in range(5):
        s = b.swap((0,), (0, 1)); s.mean(axis=2); s.std(axis=2)
    torch.cuda.synchronize()
    N = 30
    for name, f in [("swap", lambda: b.swap((0,), (0, 1))), ("mean", lambda: s.mean(axis=2)),
                    ("std", lambda: s.std(axis=2))]:
        ws = []
        for _ in range(N):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f()
            torch.cuda.synchronize()
            ws.append(time.perf_counter() - t)
            del r
        print("%-5s wall %.1f us (median of %d, call + sync)" % (name, np.median(ws) * 1e6, N), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        s2 = b.swap((0,), (0, 1))
        s2.mean(axis=2)
        s2.std(axis=2)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
