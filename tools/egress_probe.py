"""Device -> host egress of large results (diagnostic for toarray, array.py:1006-1014).

For 2.1 GB (C2) and 8.6 GB (C5) device buffers, times:
  staged     transfer.to_host as shipped (two pinned 64-MiB chunks, 8 host
             copy threads, into a fresh numpy array: first-touch bound)
  pinned     the result allocated from torch's caching pinned-host allocator
             and DMA'd into directly; the numpy result views it (first call
             pays the pinning, later same-size calls reuse the block)
  register   a fresh numpy array hipHostRegister'ed, one DMA, unregistered
Each variant runs 3 times; GB/s per call are printed and the bytes checked.
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bolt_amd.mi355x import transfer  # noqa: E402

dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")


def staged(t):
    return transfer.to_host(t, np.uint8, (t.numel(),))


def pinned(t):
    host = torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(t, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    return host.numpy()


def register(t):
    out = np.empty(t.numel(), dtype=np.uint8)
    rc = hip.hipHostRegister(ctypes.c_void_p(out.ctypes.data), ctypes.c_size_t(out.nbytes), 0)
    assert rc == 0, rc
    torch.from_numpy(out).copy_(t, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    hip.hipHostUnregister(ctypes.c_void_p(out.ctypes.data))
    return out


for gb in (2.1, 8.6):
    n = int(gb * 1e9) // 16 * 16
    t = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    probe = t[::max(1, n // 4096)].cpu().numpy()
    for name, f in (("staged", staged), ("pinned", pinned), ("register", register)):
        for i in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            h = f(t)
            dt = time.perf_counter() - t0
            ok = np.array_equal(h[::max(1, n // 4096)], probe)
            print("%.1f GB %-9s call %d: %6.1f GB/s %s" % (gb, name, i, n / dt / 1e9, "ok" if ok else "MISMATCH"),
                  flush=True)
            del h
    del t
    torch.cuda.empty_cache()
