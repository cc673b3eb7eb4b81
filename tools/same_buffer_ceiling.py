"""Every BASELINE permute against a plain copy of ITS OWN buffers (diagnostic,
one GPU).

A kernel's fraction of 8 TB/s moves with where its buffers land (boxes and
processes differ by up to ~25% on the same kernel, profiles/r06zk, r06zm).
Here each permute the bench measures runs on one source / destination pair,
interleaved with the library's contiguous copy of the same bytes from that
source into that destination (bm_copy_strided -> the 16-B rowcopy), so the
ratio permute / copy is free of placement:
  C2 swap     (2000,512,512) f32 swap((0,),(0,1)): padded rows (pitch 2048)
  C3 swap     (4096,256,256,32) f32 swap((0,),(0,))
  C3 .T       the same array reversed
  C4 swap     (10000,1024,1024) u16 swap((0,),(0,))
  C5 .T       64^5 f64 reversed
  C5 perm     64^5 f64 transpose(2,0,4,1,3)
  t64 swap    (8192,256,256,32) f32 swap((0,),(0,))
Each op exactly as the product launches it (array._move: the pitched copy when
_pitch_plan pads the result, else bm_permute).  ms per call, median of 7
rounds x 3 calls.

    python tools/same_buffer_ceiling.py [C2,C3s,...]
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bolt_amd.mi355x import array as A  # noqa: E402
from bolt_amd.mi355x._ops import backend_for  # noqa: E402
from bolt_amd.mi355x.plan import swap_perm  # noqa: E402

CASES = {
    "C2": ((2000, 512, 512), np.float32, 1, ("swap", (0,), (0, 1))),
    "C3s": ((4096, 256, 256, 32), np.float32, 2, ("swap", (0,), (0,))),
    "C3T": ((4096, 256, 256, 32), np.float32, 2, ("perm", (3, 2, 1, 0))),
    "C4": ((10000, 1024, 1024), np.uint16, 1, ("swap", (0,), (0,))),
    "C5T": ((64,) * 5, np.float64, 3, ("perm", (4, 3, 2, 1, 0))),
    "C5p": ((64,) * 5, np.float64, 3, ("perm", (2, 0, 4, 1, 3))),
    "t64": ((8192, 256, 256, 32), np.float32, 2, ("swap", (0,), (0,))),
}


def run(name, dev, be):
    shape, dt, split, op = CASES[name]
    es = np.dtype(dt).itemsize
    perm = swap_perm(len(shape), split, op[1], op[2])[0] if op[0] == "swap" else op[1]
    mv = A._move_plan(shape, perm, split)
    pp = A._pitch_plan(mv, shape, es)
    n = int(np.prod(shape))
    nbytes = n * es
    dbytes = nbytes if pp is None else pp[1] * pp[0] * es
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    src.view(torch.int32)[: nbytes // 4].random_(0, 1 << 30) if nbytes % 4 == 0 else src.random_(0, 255)
    dst = torch.empty(dbytes, dtype=torch.uint8, device=dev)
    if pp is None:
        kern = lambda: be.permute(src, list(shape), list(perm), es, dst)  # noqa: E731
        how = "bm_permute"
    else:
        P, rows, oshape, psstr, dstr = pp
        kern = lambda: be.copy_strided(src, 0, dst, 0, oshape, psstr, dstr, es)  # noqa: E731
        how = "pitched copy (pitch %d)" % P
    n4 = nbytes // 4
    copy = lambda: be.copy_strided(src, 0, dst, 0, [n4], [1], [1], 4)  # noqa: E731
    ops = {"permute": kern, "copy": copy}
    for f in ops.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in ops}
    for _ in range(7):
        for k, f in ops.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 3)
    ms = {k: statistics.median(v) for k, v in times.items()}
    b = 2 * nbytes
    print("%-4s %-26s permute %8.4f ms (%.3f of 8 TB/s)  copy %8.4f ms (%.3f)  permute/copy speed %.3f"
          % (name, how, ms["permute"], b / ms["permute"] / 8e9, ms["copy"], b / ms["copy"] / 8e9,
             ms["copy"] / ms["permute"]), flush=True)
    del src, dst
    torch.cuda.empty_cache()


def main():
    dev = torch.device("cuda", 0)
    be = backend_for(dev)
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CASES)
    for name in names:
        run(name, dev, be)


if __name__ == "__main__":
    main()
