"""Wall time of C2's statistics with the result stored by the kernel into
page-locked host memory (transfer.ZERO_COPY, transfer.host_result) vs a
device buffer + D2H copy.  Interleaved rounds, median per call.

    python tools/zero_copy_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd import MI355XContext  # noqa: E402
from bolt_amd.mi355x import transfer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = MI355XContext(device=dev)
    shard = (1000 + 50 * torch.randn(2000 * 512 * 512, device=dev)).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(shard, (2000, 512, 512), context=ctx, split=1, dtype=np.float32)
    s = b.swap((0,), (0, 1))
    ref = {}
    for zc in (False, True):
        transfer.ZERO_COPY = zc
        ref[zc] = (np.asarray(s.mean(axis=2)), np.asarray(s.std(axis=2)))
    assert all(a.tobytes() == c.tobytes() for a, c in zip(ref[False], ref[True]))
    times = {(zc, f): [] for zc in (False, True) for f in ("mean", "std", "step")}
    for _ in range(15):
        for zc in (False, True):
            transfer.ZERO_COPY = zc
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = s.mean(axis=2)
            t1 = time.perf_counter()
            r = s.std(axis=2)
            t2 = time.perf_counter()
            sw = b.swap((0,), (0, 1))
            r = sw.mean(axis=2)
            r = sw.std(axis=2)
            t3 = time.perf_counter()
            del r, sw
            times[(zc, "mean")].append(t1 - t0)
            times[(zc, "std")].append(t2 - t1)
            times[(zc, "step")].append(t3 - t2)
    for k, v in sorted(times.items()):
        print("zero_copy=%-5s %-4s median %8.1f us" % (k[0], k[1], np.median(v) * 1e6), flush=True)


if __name__ == "__main__":
    main()
