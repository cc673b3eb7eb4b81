"""Write-side counter probe of the record scatter k_recmap_scatter (diagnostic;
run under rocprofv3 --pmc, one pass per counter group, tools/gpu_scatter_counters.sh).

Ops (each launched 3 times on the same HBM data, after one warm-up):
  c5k2v      C5 chunk((16,16), padding=2).keys_to_values((2,))  [k_recmap_scatter, group 64: 2.6-3.2 KB boxes]
  c5unchunk  the same chunked array .unchunk()                   [k_recmap_scatter, group 1: 128-B rows]
  c4swap     C4 swap (k_rowcopy, 2-KiB rows; reference point at ~0.77)
usage: python tools/scatter_counters.py op [op ...]
"""
import gc
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402

ctx = bolt.MI355XContext()


def arr(shape, dtype, split):
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    raw = torch.randint(0, 255, (n,), device="cuda", dtype=torch.uint8)
    return bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=split, dtype=dtype)


for op in sys.argv[1:]:
    if op in ("c5k2v", "c5unchunk"):
        b = arr((64,) * 5, np.float64, 3)
        c = b.chunk((16, 16), padding=2)
        f = (lambda: c.keys_to_values((2,))) if op == "c5k2v" else (lambda: c.unchunk())
    elif op == "c4swap":
        b = arr((10000, 1024, 1024), np.uint16, 1)
        c = None
        f = lambda: b.swap((0,), (0,))  # noqa: E731
    else:
        raise SystemExit("unknown op %s" % op)
    for _ in range(4):
        r = f()
        del r
    torch.cuda.synchronize()
    del b, c, f
    gc.collect()
    torch.cuda.empty_cache()
print("ok")
