"""Chunk pack / unpack throughput of the mi355x mode on the BASELINE chunk configs.

    python tools/chunk_bench.py

C4: uint16 (10000,1024,1024) split 1, chunk('150') (plan (73,1024)) -> unchunk.
C5: float64 64^5 split 3, chunk((16,16), padding=2) -> unchunk, keys_to_values((2,)),
values_to_keys((0,)).  Algorithmic bytes: pack = N*s + packed bytes,
unpack = packed bytes read + N*s written.  Times: hipEvents around the call.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402


def timed(f, reps=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = None
    e0.record()
    for _ in range(reps):
        out = None  # free the previous result first: one live output, no allocator churn
        out = f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, out


def shard(ctx, shape, dtype, split, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    raw = torch.randint(-128, 127, (n,), generator=g, device="cuda", dtype=torch.int8).view(torch.uint8)
    return bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=split, dtype=dtype)


def main():
    ctx = bolt.MI355XContext()
    res = {}
    for name, shape, dtype, split, size, pad in [
            ("C4 chunk('150')", (10000, 1024, 1024), np.uint16, 1, "150", None),
            ("C5 chunk((16,16),padding=2)", (64,) * 5, np.float64, 3, (16, 16), 2)]:
        b = shard(ctx, shape, dtype, split, 1)
        N = int(np.prod(shape)) * np.dtype(dtype).itemsize
        ms, c = timed(lambda: b.chunk(size, padding=pad))
        P = c._packed.numel()
        res[name + " pack"] = {"ms": round(ms, 3), "GB/s": round((N + P) / ms / 1e6, 1),
                               "plan": [int(x) for x in c.plan], "packed_bytes": P}
        ms, u = timed(lambda: c.unchunk())
        res[name + " unchunk"] = {"ms": round(ms, 3), "GB/s": round((N + P) / ms / 1e6, 1)}
        assert torch.equal(u._data, b._data)
        if pad:
            # minimum bytes of a re-chunk: read the old packing, write the new one
            ms, k = timed(lambda: c.keys_to_values((2,)), reps=2)
            res[name + " keys_to_values((2,))"] = {"ms": round(ms, 3),
                                                   "GB/s": round((P + k._packed.numel()) / ms / 1e6, 1)}
            del k
            ms, v = timed(lambda: c.values_to_keys((0,)), reps=2)
            res[name + " values_to_keys((0,))"] = {"ms": round(ms, 3),
                                                   "GB/s": round((P + v._packed.numel()) / ms / 1e6, 1)}
            del v
        del b, c, u
        torch.cuda.empty_cache()
    from bolt_amd.mi355x.chunk import PATHS
    res["paths"] = dict(PATHS)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
