"""Indexing throughput of the mi355x mode at the C2 size (float32 (2000,512,512)).

    python tools/index_bench.py

Algorithmic bytes = bytes read + bytes written of the selection (the output
size twice); times are hipEvents around the call (host planning included).
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
    e0.record()
    out = None
    for _ in range(reps):
        out = None  # free the previous result first: one live output, no allocator churn
        out = f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, out


def main():
    ctx = bolt.MI355XContext()
    shape = (2000, 512, 512)
    raw = (torch.randn(int(np.prod(shape)), device="cuda") * 50 + 1000).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=1, dtype=np.float32)
    rng = np.random.default_rng(0)
    pts = tuple([np.sort(rng.integers(0, 2000, 1 << 22))] + [rng.integers(0, 512, 1 << 22) for _ in range(2)])
    cases = {
        "b[1999:0:-1] (reversed keys)": np.s_[1999:0:-1],
        "b[:, 511:0:-1, 511:0:-1] (reversed values)": np.s_[:, 511:0:-1, 511:0:-1],
        "b[1999:0:-3, 100:400:2] (strided)": np.s_[1999:0:-3, 100:400:2],
        "b[:, :, 7] (int on last axis)": np.s_[:, :, 7],
        "b[perm1000] (key list, 1000 rows)": (rng.permutation(2000)[:1000].tolist(),),
        "b[:, list256] (value list)": (slice(None), rng.permutation(512)[:256].tolist()),
        "b[pts] (4M-point gather)": pts,
    }
    res = {}
    for name, idx in cases.items():
        ms, r = timed(lambda: b[idx])
        nb = r._data.numel()
        res[name] = {"ms": round(ms, 3), "out_bytes": nb, "GB/s": round(2 * nb / ms / 1e6, 1)}
        del r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
