"""C5 chunk pack against the same kernel with trivial maps (diagnostic, one GPU).

The C5 pack (bm_record_gather, k_recmap_lds: 64^3 records of 64x64 float64,
(16,16) chunks with 2-cell halos) reads 8.6 GB and writes 12.1 GB and runs in
one of two states, 3.2-3.4 ms or 4.0-4.1 ms, per box and process
(profiles/r06_pack_slow_state.md), while a plain copy into the same
destination does not slow down.  Here, in one process and on the same
buffers, interleaved:
  pack     the product's pack map (halos re-read from LDS)
  expand   the same kernel and byte counts with a sequential map: each
           destination record is its source record followed by its first
           1680 elements again (the pack's write:read ratio, no halo pattern)
  ident    the same kernel with a 1:1 map (dst_rec = src_rec: 8.6 GB each way)
  copy     torch copy_ of the 8.6 GB source into the destination's front
ms per call, median of 7 rounds x 3 calls; outputs of expand / ident checked.

    python tools/pack_expand_probe.py [churn_gib]

churn_gib: first allocate and free that many GiB (torch's caching allocator
hands them back to the driver), as the bench's earlier configs do before C5
(the 64 GiB target alone holds 128 GiB), so the C5 buffers land on the pages
a long process is given.
"""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bolt_amd.mi355x import _lib, _ops, plan  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    churn = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
    if churn > 0:
        blocks = [torch.empty(16 << 30, dtype=torch.uint8, device=dev) for _ in range(int(churn // 16))]
        for t in blocks:
            t.fill_(7)
        torch.cuda.synchronize()
        del blocks
        torch.cuda.empty_cache()
        print("churned %.0f GiB" % churn, flush=True)
    st = torch.cuda.current_stream(dev).cuda_stream
    nrec, src_rec = 64 ** 3, 64 * 64
    geom = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
    pack_map = geom.record_map(unpack=False)
    dst_rec = pack_map.size                       # 5776
    exp_map = (np.arange(dst_rec) % src_rec).astype(np.int32)
    id_map = np.arange(src_rec, dtype=np.int32)
    src = torch.randint(0, 255, (nrec * src_rec * 8,), dtype=torch.uint8, device=dev)
    dst = torch.empty(nrec * dst_rec * 8, dtype=torch.uint8, device=dev)

    def gather(rmap, drec, split=True):
        # the product's parts for the pack; the trivial maps run whole-record
        # tiles, the kernel the pack's empty part list selects (k_recmap_lds)
        parts = _ops.record_parts(rmap, src_rec, 8, None) if split else []
        print("map of %d: %d parts" % (drec, len(parts) // 4), flush=True)
        p = (ctypes.c_int64 * max(1, len(parts)))(*[int(v) for v in parts]) if parts else None
        dmap = torch.from_numpy(rmap).to(dev)

        def run():
            rc = lib.bm_record_gather(src.data_ptr(), dst.data_ptr(), nrec, src_rec, drec, dmap.data_ptr(),
                                      len(parts) // 4, p, 8, st)
            assert rc == 0, lib.bm_last_error()
        run.keep = (dmap, p)
        return run

    ops = {
        "pack": (gather(pack_map, dst_rec), nrec * (src_rec + dst_rec) * 8),
        "expand": (gather(exp_map, dst_rec, False), nrec * (src_rec + dst_rec) * 8),
        "ident": (gather(id_map, src_rec, False), nrec * src_rec * 16),
        "copy": (lambda: dst[:src.numel()].copy_(src), nrec * src_rec * 16),
    }
    # checks: expand and ident move the bytes they should
    ops["expand"][0]()
    torch.cuda.synchronize()
    s64 = src.view(torch.int64).view(nrec, src_rec)
    d64 = dst.view(torch.int64).view(nrec, dst_rec)
    ok_e = torch.equal(d64[:, :src_rec], s64) and torch.equal(d64[:, src_rec:], s64[:, :dst_rec - src_rec])
    ops["ident"][0]()
    torch.cuda.synchronize()
    ok_i = torch.equal(dst.view(torch.int64)[:nrec * src_rec], src.view(torch.int64))
    print("checks: expand %s, ident %s" % ("exact" if ok_e else "MISMATCH", "exact" if ok_i else "MISMATCH"),
          flush=True)
    times = {k: [] for k in ops}
    for _ in range(7):
        for k, (f, _) in ops.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 3)
    for k, (_, b) in ops.items():
        ms = statistics.median(times[k])
        print("%-7s %7.4f ms  %7.1f GB/s  %.3f of 8 TB/s  (min %.4f)" % (k, ms, b / ms / 1e6, b / ms / 8e9,
                                                                      min(times[k])), flush=True)


if __name__ == "__main__":
    main()
