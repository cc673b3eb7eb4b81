"""Within-process spread of the record-map and permute kernels.

Runs a config's bench step (bench.steps_of) for --steps steps and times every
backend launch (bm_permute, bm_record_gather, bm_copy_strided) with its own
hipEvent pair, recording the source and destination addresses.  Prints, per
op and launch kind, each call's duration with its buffers, so a slow call can
be tied to a particular allocation (or not).

    python tools/spread_probe.py [--config C5] [--steps 8] [--reuse]

--reuse keeps every op's output alive across steps (the caching allocator then
cannot hand a step's output block to the next op of the step).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402
import bolt_amd as bolt  # noqa: E402
from bolt_amd.mi355x._ops import backend_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = bolt.MI355XContext(device=dev)
    shape, dtype, split, _, _ = bench.CONFIGS[args.config]
    shard = bench.synth_shard(torch, shape, dtype, dev, 1234)
    b = bolt.ConstructMI355X.fromshards(shard, shape, context=ctx, split=split, dtype=dtype)
    del shard
    be = backend_for(dev)
    log = []
    cur = {"op": None, "step": -1}

    def wrap(name, fn, src_i, dst_i):
        def w(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **k)
            e1.record()
            log.append((cur["step"], cur["op"], name, int(a[src_i].data_ptr()), int(a[dst_i].data_ptr()),
                        int(a[dst_i].numel()), e0, e1))
            return r
        return w

    be.permute = wrap("permute", be.permute, 0, 4)
    be.record_gather = wrap("record_gather", be.record_gather, 0, 2)
    be.copy_strided = wrap("copy_strided", be.copy_strided, 0, 2)
    ops = bench.steps_of(args.config, b)
    for s in range(args.steps):
        cur["step"] = s
        for name, call, _ in ops:
            cur["op"] = name
            r = call()
            del r
    torch.cuda.synchronize()
    rows = [(st, op, k, hex(sp), hex(dp), nb, a.elapsed_time(z)) for st, op, k, sp, dp, nb, a, z in log]
    by = {}
    for st, op, k, sp, dp, nb, ms in rows:
        by.setdefault((op, k), []).append((st, sp, dp, ms))
    out = {}
    for (op, k), v in by.items():
        ms = [x[3] for x in v]
        print("%-16s %-14s n=%-3d min %.4f  med %.4f  max %.4f ms  (+%.1f%%)"
              % (op, k, len(ms), min(ms), float(np.median(ms)), max(ms), 100 * (max(ms) / min(ms) - 1)))
        for st, sp, dp, m in v:
            print("    step %2d  src %s  dst %s  %.4f ms" % (st, sp, dp, m))
        out["%s/%s" % (op, k)] = v
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
