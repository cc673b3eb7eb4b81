"""Transpose time with and without padded rows for a few shapes (one GPU):
the array-level swap / transpose, hipEvents, median of N, alternating.

    python tools/pitch_probe.py [N]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bolt_amd as bolt  # noqa: E402
import bolt_amd.mi355x.array as A  # noqa: E402
from bolt_amd import MI355XContext  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 7
ONLY = sys.argv[2].split(",") if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
ctx = MI355XContext(device=dev)
CASES = [("C2 f32 (2000,512,512) swap((0,),(0,1))", (2000, 512, 512), np.float32, lambda b: b.swap((0,), (0, 1))),
         ("f32 (3000,512,512) swap((0,),(0,1))", (3000, 512, 512), np.float32, lambda b: b.swap((0,), (0, 1))),
         ("C4 u16 (10000,1024,1024) .T", (10000, 1024, 1024), np.uint16, lambda b: b.T),
         ("f32 (1100,2048,2048)/4 swap((0,),(0,1))", (1100, 1024, 1024), np.float32, lambda b: b.swap((0,), (0, 1))),
         ("f32 (250,4096,1024) swap: 1000-B rows", (250, 4096, 1024), np.float32, lambda b: b.swap((0,), (0, 1))),
         ("f32 (500,2048,1024) swap: 2000-B rows", (500, 2048, 1024), np.float32, lambda b: b.swap((0,), (0, 1))),
         ("f32 (750,2048,1024) swap: 3000-B rows", (750, 2048, 1024), np.float32, lambda b: b.swap((0,), (0, 1))),
         ("u16 (1000,2048,2048) .T: 2000-B rows", (1000, 2048, 2048), np.uint16, lambda b: b.T),
         ("f64 (1500,1024,1024) swap: 12000-B rows", (1500, 1024, 1024), np.float64, lambda b: b.swap((0,), (0, 1))),
         ("u8 (2000,1024,2048) .T: 2000-B rows", (2000, 1024, 2048), np.uint8, lambda b: b.T),
         ("f64 (300,1024,1024) swap: 2400-B rows", (300, 1024, 1024), np.float64, lambda b: b.swap((0,), (0, 1)))]


def timed(f):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    r = f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), r


for k, (name, shape, dtype, op) in enumerate(CASES):
    if ONLY and str(k) not in ONLY:
        continue
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    x = torch.randint(0, 60000, (nbytes // 2,), dtype=torch.int32, device=dev).to(torch.uint16).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(x, shape, context=ctx, split=1, dtype=dtype)
    del x
    t = {True: [], False: []}
    padded = None
    for i in range(N + 1):
        for p in (True, False):
            A.ROW_PITCH = p
            ms, r = timed(lambda: op(b))
            if i:
                t[p].append(ms)
            if p:
                padded = "_pbuf" in r.__dict__
            del r
    A.ROW_PITCH = True
    gb = 2 * nbytes / 1e9
    print("%-42s padded=%s  padded %.4f ms (%.0f GB/s)  dense %.4f ms (%.0f GB/s)"
          % (name, padded, statistics.median(t[True]), gb / statistics.median(t[True]) * 1e3,
             statistics.median(t[False]), gb / statistics.median(t[False]) * 1e3), flush=True)
    del b
    torch.cuda.empty_cache()
