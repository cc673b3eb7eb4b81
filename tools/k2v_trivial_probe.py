"""C5 keys_to_values((2,)) against its own kernel on a trivial runs table
(diagnostic, one GPU).

bm_record_runs walks the destination of C5's keys_to_values (12.1 GB in,
12.1 GB out: 16 chunk boxes of 2.6-3.2 KB per record regrouped by chunk id,
k_record_runs_dst).  Here, in one process and on the same buffers,
interleaved:
  k2v      the product's runs table (16 runs; each destination region is
           filled from 64 records in turn)
  trivial  the same kernel and bytes with ONE run per record laid out in
           record order (group 64): a copy through the destination walk
  runs1    the product's 16 run boundaries with group 1 (each record copied
           onto itself run by run): the k2v's lookups, sequential reads
  copy     torch copy_ of the source into the destination
ms per call, median of 7 rounds x 3 calls; both outputs checked.

    python tools/k2v_trivial_probe.py
"""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bolt_amd.mi355x import _lib, plan  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    g = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
    new = plan.ChunkGeometry((64, 64, 64), (64, 16, 16), (0, 2, 2))
    nrec, src_rec, group, gstride = 64 ** 3, g.size, 64, new.size
    map_a, map_b = plan.copies_to_scatter(plan.k2v_copies(g, new, [1, 1, 64], np.array([False, False, True])),
                                          64 * g.size, group=64, src_rec=g.size)
    runs, vb = plan.scatter_to_runs(map_a, map_b, g.size, new.size, 8)
    runs = runs[np.argsort(runs[:, 2], kind="stable")]
    assert group * src_rec == gstride, (group, src_rec, gstride)
    rv = src_rec * 8 // vb
    trivial = np.array([[0, rv, 0, rv]], dtype=np.int64)
    bys = runs[np.argsort(runs[:, 0], kind="stable")]
    assert bys[0, 0] == 0 and np.all(bys[1:, 0] == bys[:-1, 0] + bys[:-1, 1]) and bys[-1, 0] + bys[-1, 1] == rv
    runs1 = np.stack([bys[:, 0], bys[:, 1], bys[:, 0], bys[:, 1]], axis=1).astype(np.int64)
    src = torch.randint(0, 255, (nrec * src_rec * 8,), dtype=torch.uint8, device=dev)
    dst = torch.empty(nrec // group * gstride * 8, dtype=torch.uint8, device=dev)
    tabs = {"k2v": torch.from_numpy(runs.reshape(-1).copy()).to(dev),
            "trivial": torch.from_numpy(trivial.reshape(-1).copy()).to(dev),
            "runs1": torch.from_numpy(runs1.reshape(-1).copy()).to(dev)}
    nruns = {"k2v": runs.shape[0], "trivial": 1, "runs1": runs1.shape[0]}
    geo = {"k2v": (group, gstride), "trivial": (group, gstride), "runs1": (1, src_rec)}

    def call(name):
        grp, gs = geo[name]
        rc = lib.bm_record_runs(src.data_ptr(), dst.data_ptr(), nrec, src_rec, grp, gs, nruns[name],
                                tabs[name].data_ptr(), vb, 1, 8, st)  # 1: BM_RUNS_TILED
        assert rc == 0, lib.bm_last_error()

    ops = {"k2v": lambda: call("k2v"), "trivial": lambda: call("trivial"), "runs1": lambda: call("runs1"),
           "copy": lambda: dst.copy_(src)}
    nbytes = src.numel() + dst.numel()
    # checks
    call("trivial")
    torch.cuda.synchronize()
    ok_t = torch.equal(dst, src)
    dst.zero_()
    call("runs1")
    torch.cuda.synchronize()
    ok_t = ok_t and torch.equal(dst, src)
    call("k2v")
    torch.cuda.synchronize()
    s = src.view(torch.int64).view(nrec, src_rec)
    d = dst.view(torch.int64).view(nrec // group, gstride)
    rh = runs * (vb // 8)
    ok_k = all(torch.equal(d[:, a + k * m:a + k * m + ln], s[k::group, s0:s0 + ln])
               for s0, ln, a, m in rh for k in range(0, group, 9))
    print("vec %d B, %d runs; checks: trivial / runs1 %s, k2v %s" % (vb, runs.shape[0], "exact" if ok_t else "MISMATCH",
                                                           "exact" if ok_k else "MISMATCH"), flush=True)
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
    for k in ops:
        ms = statistics.median(times[k])
        print("%-8s %7.4f ms  %7.1f GB/s  %.3f of 8 TB/s  (min %.4f)" % (k, ms, nbytes / ms / 1e6,
                                                                      nbytes / ms / 8e9, min(times[k])), flush=True)


if __name__ == "__main__":
    main()
