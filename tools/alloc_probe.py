"""Does the buffer's allocator change a permute's speed?  The product's
bm_permute (C5 .T and C2 swap) on torch caching-allocator tensors vs on raw
hipMalloc buffers, interleaved in one process (hipEvents on one stream).

    python tools/alloc_probe.py [--rounds 5]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from bolt_amd.mi355x import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--hip-first", action="store_true", help="hipMalloc the raw buffers before torch allocates")
    ap.add_argument("--cases", default="c5_T,c2_swap")
    args = ap.parse_args()
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    torch.cuda.init()
    st = torch.cuda.current_stream()
    cases = {"c5_T": ((64, 64, 64, 64, 64), (4, 3, 2, 1, 0), 8),
             "c2_swap": ((2000, 512 * 512), (1, 0), 4),
             "c3_T": ((1024, 256, 256, 32), (3, 2, 1, 0), 4),
             "c3_swap": ((1024, 256, 256, 32), (1, 2, 0, 3), 4)}
    for name, (shape, perm, es) in cases.items():
        if name not in args.cases.split(","):
            continue
        nbytes = int(np.prod(shape)) * es
        hs, hd = ctypes.c_void_p(), ctypes.c_void_p()
        if args.hip_first:
            assert hip.hipMalloc(ctypes.byref(hs), nbytes) == 0 and hip.hipMalloc(ctypes.byref(hd), nbytes) == 0
        ts = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        td = torch.empty_like(ts)
        ts.fill_(7)
        if not args.hip_first:
            assert hip.hipMalloc(ctypes.byref(hs), nbytes) == 0 and hip.hipMalloc(ctypes.byref(hd), nbytes) == 0
        assert hip.hipMemset(hs, 7, nbytes) == 0
        torch.cuda.synchronize()
        shp = (ctypes.c_int64 * len(shape))(*shape)
        prm = (ctypes.c_int32 * len(perm))(*perm)
        # a 1-GiB-aligned pair carved out of over-sized hipMalloc blocks
        G = 1 << 30
        gs, gd = ctypes.c_void_p(), ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(gs), nbytes + G) == 0 and hip.hipMalloc(ctypes.byref(gd), nbytes + G) == 0
        als, ald = (gs.value + G - 1) // G * G, (gd.value + G - 1) // G * G
        assert hip.hipMemset(ctypes.c_void_p(als), 7, nbytes) == 0
        torch.cuda.synchronize()
        # the same carve-out from torch's caching allocator
        tgs = torch.empty(nbytes + G, dtype=torch.uint8, device="cuda")
        tgd = torch.empty(nbytes + G, dtype=torch.uint8, device="cuda")
        tas, tad = (tgs.data_ptr() + G - 1) // G * G, (tgd.data_ptr() + G - 1) // G * G
        bufs = {"torch": (ts.data_ptr(), td.data_ptr()), "hipMalloc": (hs.value, hd.value),
                "torch_1G": (tas, tad),
                "t_src/h_dst": (ts.data_ptr(), hd.value), "h_src/t_dst": (hs.value, td.data_ptr()),
                "hip_1G": (als, ald)}
        print("%s: torch src 0x%x dst 0x%x | hipMalloc src 0x%x dst 0x%x" %
              (name, ts.data_ptr(), td.data_ptr(), hs.value, hd.value), flush=True)
        times = {k: [] for k in bufs}
        for r in range(args.rounds):
            for k, (s, d) in bufs.items():
                evs = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    rc = lib.bm_permute(ctypes.c_void_p(s), ctypes.c_void_p(d), len(shape), shp, prm, es,
                                        ctypes.c_void_p(st.cuda_stream))
                    assert rc == 0
                    e1.record(st)
                    evs.append((e0, e1))
                torch.cuda.synchronize()
                times[k].append(float(np.median([a.elapsed_time(b) for a, b in evs])))
        for k, v in times.items():
            med = float(np.median(v))
            print("%-8s %-12s median %.4f ms  %.1f GB/s  rounds %s" % (name, k, med, 2 * nbytes / med / 1e6,
                                                                     " ".join("%.4f" % x for x in v)), flush=True)
        del ts, td, tgs, tgd
        for p in (hs, hd, gs, gd):
            hip.hipFree(p)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
