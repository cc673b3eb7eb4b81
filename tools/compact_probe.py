"""What a padded C2 swap result costs its other users (one GPU): the
compaction copy (`_compact`), a transpose back read straight from the
padded rows against the same transpose of the dense result, and swap + map
(records = padded rows) against swap + map on dense rows.  hipEvents on
the current stream, median of N.

    python tools/compact_probe.py [N]
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

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
ctx = MI355XContext(device=dev)
shape = (2000, 512, 512)
g = torch.Generator(device=dev)
g.manual_seed(7)
x = torch.randn(shape, generator=g, device=dev)
b = bolt.ConstructMI355X.fromshards(x, shape, context=ctx, split=1, dtype=np.float32)
del x


def timed(f):
    ts = []
    for _ in range(N + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts[2:])


pad = [None]


def swap_padded():
    pad[0] = b.swap((0,), (0, 1))


print("swap, padded rows        %.4f ms" % timed(swap_padded), flush=True)
assert "_pbuf" in pad[0].__dict__


def compact():
    s = b.swap((0,), (0, 1))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s._compact()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


print("compaction copy          %.4f ms" % statistics.median([compact() for _ in range(N)]), flush=True)
s_pad = b.swap((0,), (0, 1))
A.ROW_PITCH = False
s_dense = b.swap((0,), (0, 1))
A.ROW_PITCH = True
assert "_pbuf" in s_pad.__dict__ and "_pbuf" not in s_dense.__dict__
A.ROW_PITCH = False
print("swap, dense rows         %.4f ms" % timed(lambda: b.swap((0,), (0, 1))), flush=True)
A.ROW_PITCH = True
print("T of the padded result   %.4f ms" % timed(lambda: s_pad.T), flush=True)
assert "_pbuf" in s_pad.__dict__
print("T of the dense result    %.4f ms" % timed(lambda: s_dense.T), flush=True)
assert torch.equal(s_pad.T._data, s_dense.T._data)
print("ok: transposes of the padded and dense results identical", flush=True)


def map_of(make):
    def f():
        make().map(lambda v: v * 2 + 1, axis=(0, 1))
    return f


def padded():
    return b.swap((0,), (0, 1))


def dense():
    A.ROW_PITCH = False
    try:
        return b.swap((0,), (0, 1))
    finally:
        A.ROW_PITCH = True


print("swap + map, padded rows  %.4f ms" % timed(map_of(padded)), flush=True)
print("swap + map, dense rows   %.4f ms" % timed(map_of(dense)), flush=True)
mp = padded().map(lambda v: v * 2 + 1, axis=(0, 1))
md = dense().map(lambda v: v * 2 + 1, axis=(0, 1))
assert torch.equal(mp._data, md._data)
print("ok: maps identical", flush=True)
