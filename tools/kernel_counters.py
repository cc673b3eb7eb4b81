"""Counter probe for the kernels below roofline (diagnostic; run under
rocprofv3 --pmc, one pass per counter group, see tools/gpu_kernel_counters.sh).

Ops (each launched 3 times on freshly generated HBM data):
  c2swap  k_transpose<u32,64,256>   C2 swap((0,),(0,1)), float32 (2000,512,512)  [0.72-0.75: reference point]
  c4swap  k_rowcopy                 C4 swap, uint16 (10000,1024,1024), 2-KiB rows  [0.77]
  c3swap  k_rowcopy                 C3 swap, float32 (4096,256,256,32), 128-B rows [0.67]
  c5T     k_transpose<u64,32,64>    C5 .T, float64 64^5                            [0.66-0.70]
  c5pack  k_recmap_lds              C5 chunk((16,16), padding=2)                   [0.64-0.79]
  c5v2k   k_recmap_parts            C5 chunk -> values_to_keys((0,))
usage: python tools/kernel_counters.py op [op ...]
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


OPS = {
    "c2swap": (((2000, 512, 512), np.float32, 1), lambda b: b.swap((0,), (0, 1))),
    "c4swap": (((10000, 1024, 1024), np.uint16, 1), lambda b: b.swap((0,), (0,))),
    "c3swap": (((4096, 256, 256, 32), np.float32, 2), lambda b: b.swap((0,), (0,))),
    "c5T": ((((64,) * 5), np.float64, 3), lambda b: b.T),
    "c5pack": ((((64,) * 5), np.float64, 3), lambda b: b.chunk((16, 16), padding=2)),
}

for op in sys.argv[1:]:
    if op == "c5v2k":
        b = arr((64,) * 5, np.float64, 3)
        c = b.chunk((16, 16), padding=2)
        for _ in range(3):
            r = c.values_to_keys((0,))
            del r
        del b, c
    else:
        (shape, dtype, split), f = OPS[op]
        b = arr(shape, dtype, split)
        for _ in range(3):
            r = f(b)
            del r
        del b
    torch.cuda.synchronize()
    gc.collect()
    torch.cuda.empty_cache()
print("ok")
