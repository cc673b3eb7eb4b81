"""C5 `.T` (64^5 float64, all axes reversed): does the 128-MiB row stride itself
hold the transpose below the copy ceiling?  (VERDICT r05 "next" item 2.)

The product's bm_copy_strided runs the same k_transpose<u64,32,64> on the
same logical transpose while the probe pads ONE outer stride of the layout:
the source's leading axis (the tile's 64 read rows, 128 MiB apart) by
delta_s elements, or the destination's leading axis (the tile's 32 write
rows) by delta_d.  Tiles, walk, loads and stores are unchanged; only the
physical distance between the rows of a tile moves off the power of two.
If the rows of a tile camp on one DRAM channel / bank set, a skew of a few
hundred bytes to a few KiB speeds the kernel up.

One source and one destination buffer (sized for the largest skew) serve
every variant, interleaved over rounds, so placement is common to all.
Under rocprofv3 --pmc, dispatches come in variant order per round
(2 warm-ups + reps timed per variant per round).

    python tools/c5t_stride_probe.py [--rounds 3] [--reps 3] [--variants ...]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_bench import load, i64, stream  # noqa: E402

N = 64
E = N ** 4  # elements between leading-axis planes (128 MiB of float64)
VARIANTS = {  # name: (delta_s, delta_d) in elements
    "dense": (0, 0),
    "s+256B": (32, 0), "s+512B": (64, 0), "s+4KiB": (512, 0), "s+64KiB": (8192, 0), "s+2MiB": (262144, 0),
    "d+256B": (0, 32), "d+4KiB": (0, 512), "d+64KiB": (0, 8192),
    "sd+4KiB": (512, 512), "sd+256B": (32, 32),
}


def strides(ds, dd):
    # destination axes k = 0..4 take source axis 4 - k; the source's axis 0
    # (stride E + ds) is the destination's axis 4 (its contiguous one)
    sst = [1, N, N * N, N ** 3, E + ds]
    dst = [E + dd, N ** 3, N * N, N, 1]
    return sst, dst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "bolt_amd", "libbolt_mi355x.so"))
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--check", action="store_true", help="compare every variant's output with torch")
    a = ap.parse_args()
    lib = load(a.lib)
    names = a.variants.split(",")
    ms_ = max(VARIANTS[n][0] for n in names)
    md_ = max(VARIANTS[n][1] for n in names)
    src = torch.randint(-2 ** 62, 2 ** 62, (N * (E + ms_),), dtype=torch.int64, device="cuda")
    dst = torch.empty(N * (E + md_), dtype=torch.int64, device="cuda")
    shape = i64([N] * 5)
    nbytes = 2 * N ** 5 * 8
    res = {n: [] for n in names}

    def run(n):
        ds, dd = VARIANTS[n]
        sst, dstr = strides(ds, dd)
        rc = lib.bm_copy_strided(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), 5, shape,
                                 i64(sst), i64(dstr), 8, stream())
        assert rc == 0, lib.bm_last_error()

    for r in range(a.rounds):
        for n in names:
            for _ in range(2):
                run(n)
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(n)
                e1.record()
                e1.synchronize()
                res[n].append(e0.elapsed_time(e1))
            if a.check and r == 0:
                ds, dd = VARIANTS[n]
                sv = torch.as_strided(src, (N,) * 5, strides(ds, dd)[0])
                dv = torch.as_strided(dst, (N,) * 5, strides(ds, dd)[1])
                ok = bool(torch.equal(sv, dv))
                print("check %-8s %s" % (n, "exact" if ok else "MISMATCH"), flush=True)
                assert ok
    base = float(np.median(res[names[0]]))
    for n in names:
        m = float(np.median(res[n]))
        print("%-8s ds=%-7d dd=%-7d  median %.4f ms  min %.4f  %.1f GB/s  frac %.3f  vs %s %+.1f%%"
              % (n, VARIANTS[n][0], VARIANTS[n][1], m, min(res[n]), nbytes / m / 1e6, nbytes / m / 1e6 / 8000,
                 names[0], 100 * (base / m - 1)), flush=True)


if __name__ == "__main__":
    sys.exit(main())
