"""Kernel builds A/B over destination placements, with the placement's own
copy ceiling beside every kernel.

K source and K destination buffers are allocated (kinds cycled from --kinds:
hipmalloc, contiguous = hipExtMallocWithFlags(hipDeviceMallocContiguous),
vmm = hipMemCreate/hipMemMap chunks; see tools/alloc_kind_probe.py); every
(source, destination) pair runs every op with every library, interleaved over
rounds.  Ops ending in "_copy" are a plain 16-B copy of the op's source bytes
into the same destination buffer (bm_copy_strided, 1-D): the ceiling of that
placement.  With --check each library's first run on every pair is compared
byte for byte with the first library's.

    python tools/dst_placement_ab.py LIB [LIB ...] [--ops c5_pack,c5_pack_copy,c5_T,c5_T_copy]
                                     [--k 3] [--kinds hipmalloc,contiguous,vmm] [--rounds 3] [--reps 3]
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
import alloc_kind_probe as akp  # noqa: E402
from bolt_amd.mi355x import _ops, plan  # noqa: E402


def st():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def make_op(name):
    """(source bytes, destination bytes, algorithmic bytes, run(lib, s, d))."""
    base = name[:-5] if name.endswith("_copy") else name
    if base in ("c5_pack", "c5_v2k"):
        geom = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        nrec = 64 ** 3
        if base == "c5_pack":
            rmap, src_rec = geom.record_map(unpack=False), 64 * 64
        else:
            new = plan.ChunkGeometry((64,), (16,), (2,))
            rmap = plan.copies_to_map(plan.v2k_copies(geom, new, [], np.array([True, False])), 64 * new.size)
            src_rec = geom.size
        parts = _ops.record_parts(rmap, src_rec, 8)
        pp = ab_bench.i64(parts) if parts else None
        dmap = torch.from_numpy(rmap).cuda()
        sb, db = nrec * src_rec * 8, nrec * rmap.size * 8

        def run(lib, s, d, dmap=dmap):
            rc = lib.bm_record_gather(ctypes.c_void_p(s), ctypes.c_void_p(d), nrec, src_rec, rmap.size,
                                      ctypes.c_void_p(dmap.data_ptr()), len(parts) // 4, pp, 8, st())
            assert rc == 0, lib.bm_last_error()
    elif base in ("c5_T", "c3_T", "c2_swap"):
        shape, perm, es = {"c5_T": ((64,) * 5, (4, 3, 2, 1, 0), 8),
                           "c3_T": ((4096, 256, 256, 32), (3, 2, 1, 0), 4),
                           "c2_swap": ((2000, 512 * 512), (1, 0), 4)}[base]
        sb = db = int(np.prod(shape)) * es

        def run(lib, s, d):
            rc = lib.bm_permute(ctypes.c_void_p(s), ctypes.c_void_p(d), len(shape), ab_bench.i64(shape),
                                ab_bench.i32(perm), es, st())
            assert rc == 0, lib.bm_last_error()
    else:
        raise ValueError(name)
    if name.endswith("_copy"):
        n16 = min(sb, db) // 16

        def run(lib, s, d):  # noqa: F811
            rc = lib.bm_copy_strided(ctypes.c_void_p(s), ctypes.c_void_p(d), 1, ab_bench.i64([n16]),
                                     ab_bench.i64([1]), ab_bench.i64([1]), 16, st())
            assert rc == 0, lib.bm_last_error()
        return sb, db, 2 * n16 * 16, run
    return sb, db, sb + db, run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--ops", default="c5_pack,c5_pack_copy,c5_T,c5_T_copy")
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--kinds", default="hipmalloc,contiguous,vmm")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--vmm-chunk", type=int, default=1 << 30)
    a = ap.parse_args()
    torch.cuda.init()
    hip = akp.hip
    hip.hipMemGetAllocationGranularity.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p, ctypes.c_int]
    hip.hipMemAddressReserve.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_ulonglong]
    hip.hipMemCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_void_p,
                                 ctypes.c_ulonglong]
    hip.hipMemMap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                              ctypes.c_ulonglong]
    hip.hipMemSetAccess.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    hip.hipMemUnmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    hip.hipMemRelease.argtypes = [ctypes.c_void_p]
    hip.hipMemAddressFree.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libs = [(os.path.basename(p), ab_bench.load(p)) for p in a.libs]
    kinds = (a.kinds.split(",") * a.k)[:a.k]
    names = a.ops.split(",")
    ops = {n: make_op(n) for n in names}
    sb = max(o[0] for o in ops.values())
    db = max(o[1] for o in ops.values())
    srcs, dsts = [], []
    for kind in kinds:
        s, ns = akp.alloc(kind, sb, a.vmm_chunk)
        d, nd = akp.alloc(kind, db, a.vmm_chunk)
        assert s and d, (kind, ns, nd)
        assert hip.hipMemset(ctypes.c_void_p(s), 7, sb) == 0 and hip.hipMemset(ctypes.c_void_p(d), 0, db) == 0
        srcs.append(s)
        dsts.append(d)
    hip.hipDeviceSynchronize()
    if a.check and len(libs) > 1:
        # every library's result on pair (0, j) against the first library's
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        for name in names:
            if name.endswith("_copy"):
                continue
            sbo, dbo, _, run = ops[name]
            src = torch.randint(0, 255, (sbo,), dtype=torch.uint8, device="cuda", generator=g)
            hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            assert hip.hipMemcpy(ctypes.c_void_p(srcs[0]), ctypes.c_void_p(src.data_ptr()), sbo, 3) == 0
            ref = None
            for lname, lib in libs:
                for j in range(a.k):
                    hip.hipMemset(ctypes.c_void_p(dsts[j]), 0, dbo)
                    run(lib, srcs[0], dsts[j])
                    out = torch.empty(dbo, dtype=torch.uint8, device="cuda")
                    assert hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(dsts[j]), dbo, 3) == 0
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = out
                    elif not torch.equal(ref, out):
                        print("CHECK MISMATCH %s %s dst %d" % (name, lname, j), flush=True)
                        sys.exit(1)
                    del out
            print("check %s: %d libraries x %d destinations identical" % (name, len(libs), a.k), flush=True)
            del ref, src
            torch.cuda.empty_cache()
    for name in names:
        _, _, algo, run = ops[name]
        for _, lib in libs:
            for j in range(a.k):
                run(lib, srcs[j % a.k], dsts[j])
        torch.cuda.synchronize()
        res = {}
        for _ in range(a.rounds):
            for i in range(a.k):
                for j in range(a.k):
                    for lname, lib in libs:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(a.reps):
                            run(lib, srcs[i], dsts[j])
                        e1.record()
                        e1.synchronize()
                        res.setdefault((lname, i, j), []).append(e0.elapsed_time(e1) / a.reps)
        print("%s: ms by (source kind row, destination kind column), frac of 8 TB/s in brackets" % name, flush=True)
        for lname, _ in libs:
            print("  %s" % lname, flush=True)
            for i in range(a.k):
                cells = []
                for j in range(a.k):
                    ms = float(np.median(res[(lname, i, j)]))
                    cells.append("%.4f (%.3f)" % (ms, algo / ms / 1e6 / 8000))
                print("    src %-10s " % kinds[i] + "  ".join(cells), flush=True)
        print("    dst kinds: %s" % ", ".join(kinds), flush=True)
    for kind, s, d in zip(kinds, srcs, dsts):
        akp.free(kind, s)
        akp.free(kind, d)


if __name__ == "__main__":
    main()
