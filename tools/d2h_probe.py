"""Latency of small device -> host result transfers after a kernel (diagnostic).

Mimics a statistic: a ~300 us reduction kernel followed by a 1 MiB result
copied to pinned host memory, then a host wait.  Variants: the runtime copy +
stream.synchronize; the runtime copy + event spin; our copy kernel writing
straight into the pinned buffer (device-mapped host memory) + synchronize /
spin.  Reports median wall time per call and checks the bytes.
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bolt_amd.mi355x._ops import backend_for  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    be = backend_for(dev)
    x = torch.randn(2000 * 512 * 512, device=dev)
    res = torch.randn(512 * 512, device=dev).view(torch.uint8)
    n = res.numel()
    stream = torch.cuda.current_stream(dev)

    def work():
        x.sum()  # ~ a reduction's worth of HBM reading

    def copy_rt(spin):
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        host.copy_(res, non_blocking=True)
        if spin:
            ev = torch.cuda.Event()
            ev.record(stream)
            while not ev.query():
                pass
        else:
            stream.synchronize()
        return host

    def copy_kernel(spin):
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        be.lib.bm_copy_strided(ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(host.data_ptr()), 1,
                               (ctypes.c_int64 * 1)(n), (ctypes.c_int64 * 1)(1), (ctypes.c_int64 * 1)(1), 1,
                               ctypes.c_void_p(stream.cuda_stream))
        if spin:
            ev = torch.cuda.Event()
            ev.record(stream)
            while not ev.query():
                pass
        else:
            stream.synchronize()
        return host

    want = res.cpu().numpy().tobytes()
    for name, f in [("runtime copy + synchronize", lambda: copy_rt(False)),
                    ("runtime copy + event spin", lambda: copy_rt(True)),
                    ("copy kernel to pinned + synchronize", lambda: copy_kernel(False)),
                    ("copy kernel to pinned + event spin", lambda: copy_kernel(True))]:
        ws, ok = [], True
        for i in range(40):
            torch.cuda.synchronize()
            work()
            t = time.perf_counter()
            h = f()
            ws.append(time.perf_counter() - t)
            ok = ok and (h.numpy().tobytes() == want)
        print("%-40s median %.1f us (includes the reduction kernel)  %s" % (name, np.median(ws) * 1e6,
                                                                            "ok" if ok else "MISMATCH"), flush=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        work()
    torch.cuda.synchronize()
    print("reduction kernel alone: %.1f us" % ((time.perf_counter() - t) / 20 * 1e6))


if __name__ == "__main__":
    main()
