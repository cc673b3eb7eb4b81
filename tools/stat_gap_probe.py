"""Where the ~35 us between two statistic kernels of the C2 step go (diagnostic).

The GPU idles from the end of mean's kernel to the start of std's: the host
wakes from the synchronize, returns mean's result, enters std and launches.
Times each piece of that path with perf_counter, median of many calls, on a
small array (kernel ~5 us) so the host path dominates:

    python tools/stat_gap_probe.py
"""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd import MI355XContext  # noqa: E402
from bolt_amd.local import BoltArrayLocal  # noqa: E402
from bolt_amd.mi355x import _lib, transfer  # noqa: E402


def med(f, n=2000):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6


def main():
    dev = torch.device("cuda", 0)
    ctx = MI355XContext(device=dev)
    x = (1000 + 50 * torch.randn(200 * 64 * 64, device=dev))
    b = bolt.ConstructMI355X.fromshards(x, (200, 64, 64), context=ctx, split=1, dtype=np.float32)
    s = b.swap((0,), (0, 1))
    be = s._backend
    for _ in range(50):
        s.mean(axis=2)
    torch.cuda.synchronize()
    out = {}
    out["mean(axis=2) whole call"] = med(lambda: s.mean(axis=2))
    out["std(axis=2) whole call"] = med(lambda: s.std(axis=2))
    nb = 64 * 64 * 4
    out["torch.empty pinned 16 KiB"] = med(lambda: torch.empty(nb, dtype=torch.uint8, pin_memory=True))
    h = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    out["bm_host_writable"] = med(lambda: be.host_writable(h))
    out["host_result (alloc + check)"] = med(lambda: transfer.host_result(be, nb, dev))
    st = torch.cuda.current_stream(dev)
    out["stream.synchronize idle"] = med(lambda: st.synchronize())
    src = s._data

    def launch():
        be.reduce(_lib.STAT_MEAN, src, _lib.BM_F32, 4096, 200, 1, h, _lib.BM_F32)
    launch()
    torch.cuda.synchronize()
    out["be.reduce launch (no sync)"] = med(lambda: (launch(), st.synchronize()), 500) - out["stream.synchronize idle"]
    out["launch + synchronize (tiny kernel)"] = med(lambda: (launch(), st.synchronize()), 500)
    out["current_stream()"] = med(lambda: transfer.current_stream(dev))
    out["finish_host_result"] = med(lambda: transfer.finish_host_result(h, dev, np.float32, (64, 64)))
    arr = h.numpy().view(np.float32).reshape(64, 64)
    out["BoltArrayLocal(arr).toscalar()"] = med(lambda: BoltArrayLocal(arr).toscalar())
    for k, v in out.items():
        print("%-40s %8.2f us" % (k, v), flush=True)


if __name__ == "__main__":
    main()
