"""Does HOW a buffer is allocated change the TLB-heavy kernels' speed?

The same kernels (C5 chunk pack / values_to_keys record gathers, C5 .T, C3
.T, C2 swap) run interleaved in one process on source / destination pairs
made four ways:

  hipmalloc      plain hipMalloc (what torch's caching allocator does)
  hipmalloc2     a second plain hipMalloc pair, made after the others
  contiguous     hipExtMallocWithFlags(hipDeviceMallocContiguous = 0x4), if the runtime takes it
  vmm            hipMemCreate + hipMemMap in chunks of --vmm-chunk bytes (physical
                 handles of the largest granularity the runtime accepts)

Each op reports the median kernel time per kind (hipEvents, 10 reps x rounds).

    python tools/alloc_kind_probe.py [--rounds 5] [--ops c5_pack,c5_v2k,c5_T,c3_T1024,c2_swap]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from bolt_amd.mi355x import _lib, _ops, plan  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
hip.hipDeviceSynchronize.argtypes = []


class MemProp(ctypes.Structure):
    # hipMemAllocationProp (hip_runtime_api.h): type, requestedHandleType, location{type,id},
    # win32HandleMetaData, allocFlags{compressionType, gpuDirectRDMACapable, usage}
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int),
                ("loc_type", ctypes.c_int), ("loc_id", ctypes.c_int),
                ("win32HandleMetaData", ctypes.c_void_p),
                ("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class AccessDesc(ctypes.Structure):
    _fields_ = [("loc_type", ctypes.c_int), ("loc_id", ctypes.c_int), ("flags", ctypes.c_int)]


_VMM = {}  # base -> (size, [handles]) for vmm_free


def vmm_free(base):
    size, handles, ch = _VMM.pop(base)
    hip.hipMemUnmap(ctypes.c_void_p(base), ctypes.c_size_t(size))
    for h in handles:
        hip.hipMemRelease(h)
    hip.hipMemAddressFree(ctypes.c_void_p(base), ctypes.c_size_t(size))


def free(kind, p):
    if kind == "vmm":
        vmm_free(p)
    else:
        hip.hipFree(ctypes.c_void_p(p))


def alloc(kind, nbytes, chunk):
    p = ctypes.c_void_p()
    if kind.startswith("hipmalloc"):
        rc = hip.hipMalloc(ctypes.byref(p), nbytes)
        return (p.value, None) if rc == 0 else (None, "hipMalloc rc %d" % rc)
    if kind == "contiguous":
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, 0x4)
        return (p.value, None) if rc == 0 else (None, "hipExtMallocWithFlags(contiguous) rc %d" % rc)
    # vmm: reserve, create chunk handles, map, set access
    prop = MemProp(type=1, requestedHandleType=0, loc_type=1, loc_id=0)
    gran = ctypes.c_size_t()
    if hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 1) != 0:  # recommended
        return None, "granularity query failed"
    ch = max(int(chunk) // gran.value * gran.value, gran.value)
    size = (nbytes + ch - 1) // ch * ch
    if hip.hipMemAddressReserve(ctypes.byref(p), ctypes.c_size_t(size), ctypes.c_size_t(ch), None,
                                ctypes.c_ulonglong(0)) != 0:
        return None, "reserve failed"
    off = 0
    handles = []
    while off < size:
        h = ctypes.c_void_p()
        rc = hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(ch), ctypes.byref(prop), ctypes.c_ulonglong(0))
        if rc != 0:
            return None, "hipMemCreate rc %d (chunk %d)" % (rc, ch)
        rc = hip.hipMemMap(ctypes.c_void_p(p.value + off), ctypes.c_size_t(ch), ctypes.c_size_t(0), h,
                           ctypes.c_ulonglong(0))
        if rc != 0:
            return None, "hipMemMap rc %d" % rc
        handles.append(h)
        off += ch
    _VMM[p.value] = (size, handles, ch)
    acc = AccessDesc(loc_type=1, loc_id=0, flags=3)
    if hip.hipMemSetAccess(p, ctypes.c_size_t(size), ctypes.byref(acc), ctypes.c_size_t(1)) != 0:
        return None, "hipMemSetAccess failed"
    return p.value, "granularity %d, chunk %d" % (gran.value, ch)


def i64(v):
    return (ctypes.c_int64 * len(v))(*v)


def i32(v):
    return (ctypes.c_int32 * len(v))(*v)


def make_ops():
    lib = _lib.load()
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    ops = {}

    def permute(shape, perm, es):
        n = int(np.prod(shape)) * es

        def run(s, d):
            rc = lib.bm_permute(ctypes.c_void_p(s), ctypes.c_void_p(d), len(shape), i64(shape), i32(perm), es, st())
            assert rc == 0, lib.bm_last_error()
        return n, n, 2 * n, run

    def recgather(kind):
        geom = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        nrec = 64 ** 3
        if kind == "pack":
            rmap, src_rec = geom.record_map(unpack=False), 64 * 64
        else:
            new = plan.ChunkGeometry((64,), (16,), (2,))
            rmap = plan.copies_to_map(plan.v2k_copies(geom, new, [], np.array([True, False])), 64 * new.size)
            src_rec = geom.size
        parts = _ops.record_parts(rmap, src_rec, 8)
        pp = i64(parts) if parts else None
        dmap = torch.from_numpy(rmap).cuda()
        ops.setdefault("_keep", []).append(dmap)

        def run(s, d):
            rc = lib.bm_record_gather(ctypes.c_void_p(s), ctypes.c_void_p(d), nrec, src_rec, rmap.size,
                                      ctypes.c_void_p(dmap.data_ptr()), len(parts) // 4, pp, 8, st())
            assert rc == 0, lib.bm_last_error()
        return nrec * src_rec * 8, nrec * rmap.size * 8, nrec * (src_rec + rmap.size) * 8, run

    ops["c5_pack"] = lambda: recgather("pack")
    ops["c5_v2k"] = lambda: recgather("v2k")
    ops["c5_T"] = lambda: permute((64, 64, 64, 64, 64), (4, 3, 2, 1, 0), 8)
    ops["c3_T1024"] = lambda: permute((1024, 256, 256, 32), (3, 2, 1, 0), 4)
    ops["c2_swap"] = lambda: permute((2000, 512 * 512), (1, 0), 4)
    return ops


def matrix(a, ops):
    """--matrix K: K source and K destination hipMalloc buffers, every (source,
    destination) pair timed: is a slow placement a property of one buffer or
    of the pair?"""
    for name in a.ops.split(","):
        sb, db, algo, run = ops[name]()
        srcs, dsts = [], []
        kinds = (a.matrix_kinds.split(",") * a.matrix)[:a.matrix]
        for kind in kinds:
            s, _n = alloc(kind, sb, a.vmm_chunk)
            d, _n = alloc(kind, db, a.vmm_chunk)
            assert s and d, (kind, _n)
            assert hip.hipMemset(ctypes.c_void_p(s), 7, sb) == 0 and hip.hipMemset(ctypes.c_void_p(d), 0, db) == 0
            srcs.append(s)
            dsts.append(d)
        hip.hipDeviceSynchronize()
        K = a.matrix
        t = np.zeros((K, K))
        for i in range(K):
            for j in range(K):
                run(srcs[i], dsts[j])
                run(srcs[i], dsts[j])
        torch.cuda.synchronize()
        res = [[[] for _ in range(K)] for _ in range(K)]
        for _ in range(a.rounds):
            for i in range(K):
                for j in range(K):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.reps):
                        run(srcs[i], dsts[j])
                    e1.record()
                    e1.synchronize()
                    res[i][j].append(e0.elapsed_time(e1) / a.reps)
        for i in range(K):
            for j in range(K):
                t[i, j] = np.median(res[i][j])
        print("%s: ms by (source row, destination column); frac of 8 TB/s in brackets; kinds %s"
              % (name, ",".join(kinds)), flush=True)
        for i in range(K):
            print("  src 0x%x  " % srcs[i] + "  ".join("%.4f (%.3f)" % (t[i, j], algo / t[i, j] / 1e6 / 8000)
                                                     for j in range(K)), flush=True)
        print("  dst " + "  ".join("0x%x" % d for d in dsts), flush=True)
        for k_, (s_, d_) in zip(kinds, zip(srcs, dsts)):
            free(k_, s_)
            free(k_, d_)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--ops", default="c5_pack,c5_v2k,c5_T,c3_T1024,c2_swap")
    ap.add_argument("--kinds", default="hipmalloc,contiguous,vmm,hipmalloc2")
    ap.add_argument("--vmm-chunk", type=int, default=1 << 30)
    ap.add_argument("--matrix", type=int, default=0, help="K sources x K destinations per op")
    ap.add_argument("--matrix-kinds", default="hipmalloc", help="allocation kinds of the matrix buffers, cycled")
    a = ap.parse_args()
    torch.cuda.init()
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
    ops = make_ops()
    if a.matrix:
        return matrix(a, ops)
    for name in a.ops.split(","):
        sb, db, algo, run = ops[name]()
        bufs = {}
        for kind in a.kinds.split(","):
            s, note_s = alloc(kind, sb, a.vmm_chunk)
            d, note_d = alloc(kind, db, a.vmm_chunk) if s else (None, None)
            if not s or not d:
                print("%-10s %-12s unavailable: %s" % (name, kind, note_s if not s else note_d), flush=True)
                continue
            assert hip.hipMemset(ctypes.c_void_p(s), 7, sb) == 0 and hip.hipMemset(ctypes.c_void_p(d), 0, db) == 0
            bufs[kind] = (s, d, note_s)
        hip.hipDeviceSynchronize()
        times = {k: [] for k in bufs}
        for k, (s, d, _) in bufs.items():  # warm-up: first touch
            run(s, d)
            run(s, d)
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for k, (s, d, _) in bufs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run(s, d)
                e1.record()
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.reps)
        for k, (s, d, note) in bufs.items():
            ms = float(np.median(times[k]))
            print("%-10s %-12s %8.4f ms  %7.1f GB/s  frac %.3f  (min %.4f, max %.4f)  src 0x%x dst 0x%x  %s"
                  % (name, k, ms, algo / ms / 1e6, algo / ms / 1e6 / 8000, min(times[k]), max(times[k]), s, d,
                     note or ""), flush=True)
        for k, (s, d, _) in bufs.items():
            free(k, s)
            free(k, d)


if __name__ == "__main__":
    main()
