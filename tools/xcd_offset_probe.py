"""Does a kernel's speed depend on which XCD its block 0 lands on?

The dispatcher deals blocks round-robin over the 8 XCDs and, as observed,
carries on from where the previous launch stopped, so the XCD of block 0
moves with the block counts of everything launched before.  This probe
first checks that model (an empty 1-block launch reports its XCD; a 16-block
launch that follows reports every block's), then times each op with block 0
steered to each of the 8 XCDs (tools/microbench/xcd_shift.hip pads the
dispatch with empty blocks), interleaved over rounds.

    python tools/xcd_offset_probe.py [--ops c5_pack,c5_T,c5_v2k,c2_swap] [--rounds 5] [--lib bolt_amd/libbolt_mi355x.so]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import ab_bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="c5_pack,c5_T,c5_v2k,c2_swap")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(HERE), "bolt_amd", "libbolt_mi355x.so"))
    a = ap.parse_args()
    torch.cuda.init()
    lib = ab_bench.load(a.lib)
    xs = ctypes.CDLL(os.path.join(HERE, "ab_libs", "xcd_shift.so"))
    xs.xcd_shift.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    xs.xcd_map.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    buf = torch.full((64,), -1, dtype=torch.int32, device="cuda")
    bp = ctypes.c_void_p(buf.data_ptr())

    def where():
        """XCD the NEXT launch's block 0 will land on (per the round-robin model)."""
        buf.fill_(-1)   # torch's fill is itself a launch: read after it
        xs.xcd_shift(1, bp, ab_bench.stream())
        torch.cuda.synchronize()
        return (int(buf[0].item()) + 1) % 8

    def steer(target):
        c = where()
        k = (target - c) % 8
        if k:
            xs.xcd_shift(k, None, ab_bench.stream())

    # the model, checked: after steering, a 16-block map
    for target in range(8):
        steer(target)
        xs.xcd_map(16, bp, ab_bench.stream())
        torch.cuda.synchronize()
        print("steer %d -> blocks 0..15 on XCDs %s" % (target, buf[:16].tolist()), flush=True)

    ops = [(name, ab_bench.OPS[name]()) for name in a.ops.split(",")]
    for name, op in ops:
        op(lib)
        torch.cuda.synchronize()
        times = {t: [] for t in range(8)}
        for _ in range(a.rounds):
            for t in range(8):
                for _ in range(a.reps):
                    steer(t)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    op(lib)
                    e1.record()
                    e1.synchronize()
                    times[t].append(e0.elapsed_time(e1))
        med = {t: float(np.median(v)) for t, v in times.items()}
        lo, hi = min(med.values()), max(med.values())
        print("%-10s block0 XCD: %s   spread %.1f%%" % (
            name, "  ".join("%d:%.4f" % (t, med[t]) for t in range(8)), 100.0 * (hi - lo) / lo), flush=True)
        print("%-10s GB/s at best / worst: %.1f / %.1f" % (name, op.bytes / lo / 1e6, op.bytes / hi / 1e6), flush=True)
        del op
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
