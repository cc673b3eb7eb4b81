"""End-to-end time of one C2 statistic (launch -> the host sees the result)
with the result stored straight into page-locked host memory (zero-copy) or
into HBM, per libbolt_mi355x build (diagnostic).

The kernel trace shows the GPU idle ~35 us between the mean's and the std's
kernel.  Part of it may be the 1 MiB of zero-copy results draining over PCIe
after the last wave (the completion signal waits for them).  For each library
and each output kind: median host wall time of bm_reduce + stream synchronize
over many calls, and the kernel time from hipEvents.

    python tools/zero_copy_drain_probe.py lib_a.so [lib_b.so ...]
"""
import ctypes
import statistics
import sys
import time

import torch

STAT_MEAN, STAT_STD, BM_F32 = 0, 2, 10


def load(path):
    lib = ctypes.CDLL(path)
    lib.bm_reduce.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_size_t, ctypes.c_void_p]
    lib.bm_last_error.restype = ctypes.c_char_p
    return lib


def main():
    libs = [(p.split("/")[-1], load(p)) for p in sys.argv[1:]]
    O, R = 512 * 512, 2000
    src = (1000 + 50 * torch.randn(O * R, device="cuda")).contiguous()
    dev_out = torch.empty(O, device="cuda")
    host_out = torch.empty(O, pin_memory=True)
    st = torch.cuda.current_stream()
    raw = ctypes.c_void_p(st.cuda_stream)
    for stat, sname in ((STAT_MEAN, "mean"), (STAT_STD, "std")):
        for name, lib in libs:
            for kind, out in (("host", host_out), ("hbm", dev_out)):
                def call():
                    rc = lib.bm_reduce(stat, ctypes.c_void_p(src.data_ptr()), BM_F32, O, R, 1,
                                       ctypes.c_void_p(out.data_ptr()), BM_F32, None, 0, raw)
                    assert rc == 0, lib.bm_last_error()
                for _ in range(10):
                    call()
                st.synchronize()
                walls, kern = [], []
                for _ in range(60):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    t0 = time.perf_counter()
                    e0.record()
                    call()
                    e1.record()
                    st.synchronize()
                    walls.append(time.perf_counter() - t0)
                    kern.append(e0.elapsed_time(e1))
                print("%-5s %-22s %-4s wall %8.1f us   events %8.1f us" % (
                    sname, name, kind, statistics.median(walls) * 1e6, statistics.median(kern) * 1e3), flush=True)


if __name__ == "__main__":
    main()
