"""Host-side pieces of one C2 statistic call (diagnostic, one GPU).

Each piece is timed alone, many times, with the GPU idle: the pinned result
allocation, the host-writable check, the reduction launch (ctypes + runtime),
the stream synchronize of an empty stream, the result wrapping, and the whole
mean(axis=2) call minus its kernel time (hipEvents).  Medians in microseconds.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd.local import BoltArrayLocal  # noqa: E402
from bolt_amd.mi355x import _lib  # noqa: E402
from bolt_amd.mi355x.transfer import host_result  # noqa: E402


def med(f, n=300):
    ws = []
    for _ in range(n):
        t = time.perf_counter()
        f()
        ws.append(time.perf_counter() - t)
    return np.median(ws) * 1e6


def main():
    ctx = bolt.MI355XContext()
    shape = (2000, 512, 512)
    raw = (torch.randn(int(np.prod(shape)), device="cuda") * 50 + 1000).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=1, dtype=np.float32)
    s = b.swap((0,), (0, 1))
    for _ in range(5):
        s.mean(axis=2)
    torch.cuda.synchronize()
    dev = s._data.device
    be = s._backend
    stream = torch.cuda.current_stream(dev)
    nb = 512 * 512 * 4
    print("pinned torch.empty(1 MiB)      %7.1f us" % med(lambda: torch.empty(nb, dtype=torch.uint8, pin_memory=True)))
    h = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    print("host_writable                   %7.1f us" % med(lambda: be.host_writable(h)))
    print("host_result (alloc + check)     %7.1f us" % med(lambda: host_result(be, nb, dev)))
    print("current_stream()                %7.1f us" % med(lambda: torch.cuda.current_stream(dev)))
    print("stream.synchronize (idle)       %7.1f us" % med(lambda: stream.synchronize()))
    arr = h.numpy().view(np.float32).reshape(512, 512)
    print("BoltArrayLocal(arr).toscalar()  %7.1f us" % med(lambda: BoltArrayLocal(arr).toscalar()))
    # one launch of the reduction into the pinned buffer, the GPU otherwise idle
    from bolt_amd.mi355x.plan import reduce_layout
    perm, O, R, I = reduce_layout((512, 512, 2000), [2])
    code = _lib.BM_F32

    def launch():
        be.reduce(_lib.STAT_MEAN, s._data, code, O, R, I, h, code)
    ws = []
    for _ in range(100):
        torch.cuda.synchronize()
        t = time.perf_counter()
        launch()
        ws.append(time.perf_counter() - t)
    print("reduce launch (host side)       %7.1f us" % (np.median(ws) * 1e6))
    # whole call: wall minus the kernel's own event time
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ws, ks = [], []
    for _ in range(100):
        torch.cuda.synchronize()
        t = time.perf_counter()
        e0.record(stream)
        launch()
        e1.record(stream)
        stream.synchronize()
        ws.append(time.perf_counter() - t)
        ks.append(e0.elapsed_time(e1) * 1e3)
    print("launch + sync wall - kernel     %7.1f us  (kernel %.1f us)" % (np.median(ws) * 1e6 - np.median(ks),
                                                                           np.median(ks)))
    ws = []
    for _ in range(100):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.mean(axis=2)
        ws.append(time.perf_counter() - t)
    print("s.mean(axis=2) wall - kernel    %7.1f us" % (np.median(ws) * 1e6 - np.median(ks)))
    ws = []
    for _ in range(100):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = b.swap((0,), (0, 1))
        ws.append(time.perf_counter() - t)
        del r
    print("b.swap call (host side)         %7.1f us" % (np.median(ws) * 1e6))


if __name__ == "__main__":
    main()
