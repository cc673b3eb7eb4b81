"""Phase timing of keys_to_values / values_to_keys at C5 (diagnostic)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd.mi355x import chunk as C  # noqa: E402


def main():
    ctx = bolt.MI355XContext()
    shape = (64,) * 5
    n = int(np.prod(shape)) * 8
    raw = torch.randint(-128, 127, (n,), device="cuda", dtype=torch.int8).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=3, dtype=np.float64)
    c = b.chunk((16, 16), padding=2)
    orig_unpack, orig_pack = C.ChunkedArrayMI355X._unpack, C.ChunkedArrayMI355X._pack

    def unpack(self):
        torch.cuda.synchronize(); t = time.perf_counter()
        r = orig_unpack(self)
        torch.cuda.synchronize(); print("  unpack %.3f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
        return r

    def pack(*a):
        torch.cuda.synchronize(); t = time.perf_counter()
        r = orig_pack(*a)
        torch.cuda.synchronize(); print("  pack %.3f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
        return r
    C.ChunkedArrayMI355X._unpack = unpack
    C.ChunkedArrayMI355X._pack = staticmethod(pack)
    for it in range(3):
        print("k2v", it, flush=True)
        torch.cuda.synchronize(); t = time.perf_counter()
        k = c.keys_to_values((2,))
        torch.cuda.synchronize(); print(" total %.3f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
        del k
        print("v2k", it, flush=True)
        torch.cuda.synchronize(); t = time.perf_counter()
        v = c.values_to_keys((0,))
        torch.cuda.synchronize(); print(" total %.3f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
        del v


if __name__ == "__main__":
    main()
