"""mean / var / std over every axis of C2's row-padded swap result: read in
place (per-column states over the padded rows, array.py _padded_all_moments)
against what round 6 did before -- compact the rows, then the dense
reduction -- wall ms per call (host result included), best of 5.

    python tools/all_axes_padded_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd.mi355x.construct import ConstructMI355X  # noqa: E402

ctx = bolt.MI355XContext(device="cuda:0")
g = torch.Generator(device="cuda")
g.manual_seed(3)
x = torch.randn((2000, 512, 512), generator=g, device="cuda") * 50 + 1000
b = ConstructMI355X.fromshards(x, (2000, 512, 512), context=ctx, split=1, dtype=np.float32)


def best(f, reps=5):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return min(ts)


s = b.swap((0,), (0, 1))
assert "_pbuf" in s.__dict__
for name in ("mean", "var", "std"):
    in_place = best(lambda: getattr(s, name)())
    assert "_data" not in s.__dict__

    def compact_then():
        t = b.swap((0,), (0, 1))
        t._compact()
        return getattr(t, name)()
    swap_ms = best(lambda: b.swap((0,), (0, 1)))
    old = best(compact_then) - swap_ms
    print("%-4s over every axis: in place %.3f ms, compact + dense %.3f ms" % (name, in_place, old), flush=True)
