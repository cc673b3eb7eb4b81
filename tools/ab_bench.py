"""Interleaved A/B timing of libbolt_mi355x builds on the BASELINE shapes.

    python tools/ab_bench.py libA.so [libB.so ...] [--ops c2_swap,c2_mean_rows,...] [--rounds 5]

Every library is loaded side by side in ONE process and the variants run in
interleaved rounds on the same buffers (cdna_hip_programming.md §5.4 rule 24);
each op reports the median kernel time (hipEvents) and GB/s of algorithmic
bytes.  Build variants with  make -C bolt_amd/csrc OUT=/tmp/x.so BUILD=/tmp/bx EXTRA=-D...
"""
import argparse
import ctypes
import sys

import numpy as np
import torch

I64P = ctypes.POINTER(ctypes.c_int64)


def load(path):
    lib = ctypes.CDLL(path)
    lib.bm_permute.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, I64P,
                               ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_void_p]
    lib.bm_copy_strided.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, I64P, I64P, I64P,
                                    ctypes.c_int, ctypes.c_void_p]
    lib.bm_reduce.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_size_t, ctypes.c_void_p]
    if hasattr(lib, "bm_reduce_rows"):
        lib.bm_reduce_rows.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_void_p]
    lib.bm_reduce_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, ctypes.POINTER(ctypes.c_size_t)]
    lib.bm_record_gather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, I64P, ctypes.c_int,
                                     ctypes.c_void_p]
    if hasattr(lib, "bm_record_scatter"):
        lib.bm_record_scatter.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    if hasattr(lib, "bm_record_runs"):
        lib.bm_record_runs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    if hasattr(lib, "bm_record_gather_masked"):
        lib.bm_record_gather_masked.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                                ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, I64P,
                                                ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.bm_last_error.restype = ctypes.c_char_p
    return lib


def i64(v):
    return (ctypes.c_int64 * len(v))(*[int(x) for x in v])


def i32(v):
    return (ctypes.c_int32 * len(v))(*[int(x) for x in v])


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Permute(object):
    def __init__(self, shape, perm, dtype):
        self.shape, self.perm, self.es = shape, perm, np.dtype(dtype).itemsize
        n = int(np.prod(shape)) * self.es
        self.src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
        self.dst = torch.empty_like(self.src)
        self.bytes = 2 * n

    def __call__(self, lib):
        rc = lib.bm_permute(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()),
                            len(self.shape), i64(self.shape), i32(self.perm), self.es, stream())
        assert rc == 0, lib.bm_last_error()

    def check(self):
        """dst == src.permute(perm) byte for byte (torch reference, same element size)."""
        tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[self.es]
        ref = self.src.view(tdt).view(self.shape).permute(self.perm).contiguous()
        return bool(torch.equal(ref.view(-1), self.dst.view(tdt)))


class Reduce(object):
    CODES = {np.dtype(np.float32): 10, np.dtype(np.float64): 11, np.dtype(np.uint16): 3}

    def __init__(self, stat, O, R, I, dtype, out_dtype):
        self.stat, self.O, self.R, self.I = stat, O, R, I
        self.code = self.CODES[np.dtype(dtype)]
        self.ocode = self.CODES[np.dtype(out_dtype)]
        n = O * R * I * np.dtype(dtype).itemsize
        self.src = (torch.randn(n // 4, device="cuda") * 50 + 1000).view(torch.uint8) \
            if np.dtype(dtype) == np.float32 else torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
        self.out = torch.empty(O * I * np.dtype(out_dtype).itemsize, dtype=torch.uint8, device="cuda")
        self.ws = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        self.bytes = n + self.out.numel()

    def __call__(self, lib):
        rc = lib.bm_reduce(self.stat, ctypes.c_void_p(self.src.data_ptr()), self.code, self.O, self.R, self.I,
                           ctypes.c_void_p(self.out.data_ptr()), self.ocode,
                           ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(), stream())
        assert rc == 0, lib.bm_last_error()


class ReduceRows(Reduce):
    """bm_reduce_rows: O rows of R elements at a pitch of P elements (the
    statistics of a row-padded swap result: C2 is 262144 rows of 2000 float32
    at 2048)."""

    def __init__(self, stat, O, R, P, dtype, out_dtype):
        Reduce.__init__(self, stat, O, P, 1, dtype, out_dtype)
        self.R, self.P = R, P
        self.bytes = O * R * np.dtype(dtype).itemsize + self.out.numel()

    def __call__(self, lib):
        rc = lib.bm_reduce_rows(self.stat, ctypes.c_void_p(self.src.data_ptr()), self.code, self.O, self.R, self.P,
                                ctypes.c_void_p(self.out.data_ptr()), self.ocode,
                                ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(), stream())
        assert rc == 0, lib.bm_last_error()


class Copy(object):
    def __init__(self, nbytes):
        self.n = nbytes
        self.src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
        self.dst = torch.empty_like(self.src)
        self.bytes = 2 * nbytes

    def __call__(self, lib):
        rc = lib.bm_copy_strided(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()), 1,
                                 i64([self.n // 4]), i64([1]), i64([1]), 4, stream())
        assert rc == 0, lib.bm_last_error()


class RecGather(object):
    """C5's chunk pack ((16,16), padding 2 on 64x64 float64 records) or its
    values_to_keys((0,)) repack, as one bm_record_gather (parts as _ops picks)."""

    def __init__(self, kind, nparts_off=False, part_bytes=None, masked=False):
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bolt_amd.mi355x import plan, _ops
        geom = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        self.nrec = 64 ** 3
        if kind == "pack":
            rmap, self.src_rec = geom.record_map(unpack=False), 64 * 64
        else:
            vmask = np.array([True, False])
            new = plan.ChunkGeometry((64,), (16,), (2,))
            rmap = plan.copies_to_map(plan.v2k_copies(geom, new, [], vmask), 64 * new.size)
            self.src_rec = geom.size
        self.dst_rec = rmap.size
        parts = [] if nparts_off else _ops.record_parts(rmap, self.src_rec, 8, part_bytes)
        self.nparts, self.parts = len(parts) // 4, (i64(parts) if parts else None)
        self.mask, self.words = None, 0
        if masked:
            m, self.words = _ops.stage_mask(rmap, parts, 8)
            self.mask = torch.from_numpy(m).cuda()
        self.map = torch.from_numpy(rmap).cuda()
        self.src = torch.randint(0, 255, (self.nrec * self.src_rec * 8,), dtype=torch.uint8, device="cuda")
        self.dst = torch.empty(self.nrec * self.dst_rec * 8, dtype=torch.uint8, device="cuda")
        self.bytes = self.src.numel() + self.dst.numel()

    def __call__(self, lib):
        if self.mask is not None:
            rc = lib.bm_record_gather_masked(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()),
                                             self.nrec, self.src_rec, self.dst_rec,
                                             ctypes.c_void_p(self.map.data_ptr()), self.nparts, self.parts,
                                             ctypes.c_void_p(self.mask.data_ptr()), self.words, 8, stream())
        else:
            rc = lib.bm_record_gather(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()),
                                      self.nrec, self.src_rec, self.dst_rec, ctypes.c_void_p(self.map.data_ptr()),
                                      self.nparts, self.parts, 8, stream())
        assert rc == 0, lib.bm_last_error()

    def check(self):
        """dst[r, o] == src[r, map[o]] for every record (torch gather, in record blocks)."""
        s = self.src.view(torch.int64).view(self.nrec, self.src_rec)
        d = self.dst.view(torch.int64).view(self.nrec, self.dst_rec)
        idx = self.map.long()
        for r0 in range(0, self.nrec, 1 << 14):
            if not torch.equal(s[r0:r0 + (1 << 14)].index_select(1, idx), d[r0:r0 + (1 << 14)]):
                return False
        return True


class RecScatter(object):
    """C5's unchunk, keys_to_values((2,)) or values_to_keys((0,)) of the
    (16,16) padding-2 chunking as one bm_record_scatter (chunk.py's plan)."""

    def __init__(self, kind):
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bolt_amd.mi355x import plan
        g = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        self.nrec, self.src_rec, self.group = 64 ** 3, g.size, 1
        if kind == "unchunk":
            maps = plan.copies_to_scatter([(sh, ps, ds, po, do) for sh, ds, ps, do, po in g.copies(unpack=True)],
                                          g.size)
            self.gstride = 64 * 64
        elif kind == "k2v":
            new = plan.ChunkGeometry((64, 64, 64), (64, 16, 16), (0, 2, 2))
            self.group = 64
            maps = plan.copies_to_scatter(plan.k2v_copies(g, new, [1, 1, 64], np.array([False, False, True])),
                                          64 * g.size, group=64, src_rec=g.size)
            self.gstride = new.size
        else:
            new = plan.ChunkGeometry((64,), (16,), (2,))
            maps = plan.copies_to_scatter(plan.v2k_copies(g, new, [], np.array([True, False])), g.size)
            self.gstride = 64 * new.size
        map_a, map_b = maps
        self.vec = plan.scatter_vec(map_a, map_b, g.size, self.gstride, 8)
        self.ma = torch.from_numpy(map_a).cuda()
        self.mb = torch.from_numpy(map_b).cuda()
        self.src = torch.randint(0, 255, (self.nrec * g.size * 8,), dtype=torch.uint8, device="cuda")
        ndst = self.nrec // self.group * self.gstride
        self.dst = torch.empty(ndst * 8, dtype=torch.uint8, device="cuda")
        self.bytes = self.src.numel() + self.dst.numel()

    def __call__(self, lib):
        rc = lib.bm_record_scatter(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()),
                                   self.nrec, self.src_rec, self.group, self.gstride,
                                   ctypes.c_void_p(self.ma.data_ptr()),
                                   ctypes.c_void_p(self.mb.data_ptr()) if self.group > 1 else None,
                                   self.vec, 8, stream())
        assert rc == 0, lib.bm_last_error()


class RecRuns(object):
    """C5's keys_to_values((2,)) as bm_record_runs: one wave per chunk box
    (plan.scatter_to_runs of the scatter plan)."""

    def __init__(self):
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bolt_amd.mi355x import plan
        g = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        new = plan.ChunkGeometry((64, 64, 64), (64, 16, 16), (0, 2, 2))
        self.nrec, self.src_rec, self.group, self.gstride = 64 ** 3, g.size, 64, new.size
        map_a, map_b = plan.copies_to_scatter(plan.k2v_copies(g, new, [1, 1, 64], np.array([False, False, True])),
                                              64 * g.size, group=64, src_rec=g.size)
        runs, self.vb = plan.scatter_to_runs(map_a, map_b, g.size, new.size, 8)
        runs = runs[np.argsort(runs[:, 2], kind="stable")]
        self.runs_host = runs * (self.vb // 8)
        self.n = runs.shape[0]
        self.flags = int(os.environ.get("AB_RUNS_FLAGS", "1"))  # BM_RUNS_TILED (C5's boxes tile the records)
        self.table = torch.from_numpy(runs.reshape(-1).copy()).cuda()
        self.src = torch.randint(0, 255, (self.nrec * g.size * 8,), dtype=torch.uint8, device="cuda")
        self.dst = torch.empty(self.nrec // 64 * new.size * 8, dtype=torch.uint8, device="cuda")
        self.bytes = self.src.numel() + self.dst.numel()

    def __call__(self, lib):
        rc = lib.bm_record_runs(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()),
                                self.nrec, self.src_rec, self.group, self.gstride, self.n,
                                ctypes.c_void_p(self.table.data_ptr()), self.vb, self.flags, 8, stream())
        assert rc == 0, lib.bm_last_error()

    def check(self):
        s = self.src.view(torch.int64).view(self.nrec, self.src_rec)
        d = self.dst.view(torch.int64).view(self.nrec // self.group, self.gstride)
        for s0, ln, a, m in self.runs_host:
            for k in range(self.group):
                if not torch.equal(d[:, a + k * m:a + k * m + ln], s[k::self.group, s0:s0 + ln]):
                    return False
        return True


class Unchunk(object):
    """C5's unchunk as the strided copies of the chunk geometry (one per run combination)."""

    def __init__(self):
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bolt_amd.mi355x import plan
        g = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        nrec = 64 ** 3
        self.src = torch.randint(0, 255, (nrec * g.size * 8,), dtype=torch.uint8, device="cuda")
        self.dst = torch.empty(nrec * 4096 * 8, dtype=torch.uint8, device="cuda")
        self.bytes = self.src.numel() + self.dst.numel()
        self.args = [(ctypes.c_void_p(self.src.data_ptr() + po * 8), ctypes.c_void_p(self.dst.data_ptr() + do * 8),
                      len(sh) + 1, i64([nrec] + sh), i64([g.size] + ps), i64([4096] + ds))
                     for sh, ds, ps, do, po in g.copies(unpack=True)]

    def __call__(self, lib):
        for a in self.args:
            rc = lib.bm_copy_strided(*a, 8, stream())
            assert rc == 0, lib.bm_last_error()


class K2V(object):
    """C5's chunked keys_to_values((2,)) as the strided copies chunk.py runs
    (plan.k2v_copies, packed -> packed: 3200-B rows of old chunk boxes)."""

    def __init__(self):
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bolt_amd.mi355x import plan
        old = plan.ChunkGeometry((64, 64), (16, 16), (2, 2))
        new = plan.ChunkGeometry((64, 64, 64), (64, 16, 16), (0, 2, 2))
        self.copies = plan.k2v_copies(old, new, [64, 64, 64], np.array([False, False, True]))
        self.src = torch.randint(0, 255, (64 ** 3 * old.size * 8,), dtype=torch.uint8, device="cuda")
        self.dst = torch.empty(64 ** 2 * new.size * 8, dtype=torch.uint8, device="cuda")
        self.bytes = self.src.numel() + self.dst.numel()
        self.args = [(ctypes.c_void_p(self.src.data_ptr() + so * 8), ctypes.c_void_p(self.dst.data_ptr() + do * 8),
                      len(sh), i64(sh), i64(ss), i64(ds)) for sh, ss, ds, so, do in self.copies]

    def __call__(self, lib):
        for a in self.args:
            rc = lib.bm_copy_strided(*a, 8, stream())
            assert rc == 0, lib.bm_last_error()


OPS = {
    "c5_k2v": lambda: K2V(),
    "c5_k2v_scatter": lambda: RecScatter("k2v"),
    "c5_k2v_runs": lambda: RecRuns(),
    "c5_v2k_scatter": lambda: RecScatter("v2k"),
    "c5_unchunk": lambda: Unchunk(),
    "c5_unchunk_scatter": lambda: RecScatter("unchunk"),
    "c5_pack": lambda: RecGather("pack"),
    "c5_pack_whole": lambda: RecGather("pack", True),
    "c5_v2k": lambda: RecGather("v2k"),
    "c5_v2k_whole": lambda: RecGather("v2k", True),
    "c5_v2k_masked": lambda: RecGather("v2k", masked=True),
    "c5_v2k_pb16k": lambda: RecGather("v2k", part_bytes=16 << 10),
    "c5_v2k_pb24k": lambda: RecGather("v2k", part_bytes=24 << 10),
    "c2_copy": lambda: Copy(2097152000),
    "c2_swap": lambda: Permute((2000, 512 * 512), (1, 0), np.float32),
    "c2_mean_rows": lambda: Reduce(0, 512 * 512, 2000, 1, np.float32, np.float32),
    "c2_std_rows": lambda: Reduce(2, 512 * 512, 2000, 1, np.float32, np.float32),
    "c2_sum_rows": lambda: Reduce(3, 512 * 512, 2000, 1, np.float32, np.float32),
    "c2_max_rows": lambda: Reduce(4, 512 * 512, 2000, 1, np.float32, np.float32),
    "c2_mean_prow": lambda: ReduceRows(0, 512 * 512, 2000, 2048, np.float32, np.float32),
    "c2_std_prow": lambda: ReduceRows(2, 512 * 512, 2000, 2048, np.float32, np.float32),
    "c2_sum_prow": lambda: ReduceRows(3, 512 * 512, 2000, 2048, np.float32, np.float32),
    "c2_max_prow": lambda: ReduceRows(4, 512 * 512, 2000, 2048, np.float32, np.float32),
    "c2q_mean_prow": lambda: ReduceRows(0, 128 * 512, 2000, 2048, np.float32, np.float32),
    "c2q_std_prow": lambda: ReduceRows(2, 128 * 512, 2000, 2048, np.float32, np.float32),
    "c2_mean_cols": lambda: Reduce(0, 1, 2000, 512 * 512, np.float32, np.float32),
    "c2_std_cols": lambda: Reduce(2, 1, 2000, 512 * 512, np.float32, np.float32),
    "c3_swap": lambda: Permute((1024, 256, 256, 32), (1, 2, 0, 3), np.float32),
    "c3_T": lambda: Permute((1024, 256, 256, 32), (3, 2, 1, 0), np.float32),
    "runs32": lambda: Permute((4096, 4096, 8), (1, 0, 2), np.float32),
    "runs64": lambda: Permute((4096, 2048, 16), (1, 0, 2), np.float32),
    "runs128": lambda: Permute((2048, 2048, 32), (1, 0, 2), np.float32),
    "c3_full": lambda: Permute((4096, 256, 256, 32), (1, 2, 0, 3), np.float32),
    "t64_swap": lambda: Permute((8192, 256, 256, 32), (1, 2, 0, 3), np.float32),
    "c3T_full": lambda: Permute((4096, 256, 256, 32), (3, 2, 1, 0), np.float32),
    "c4_full": lambda: Permute((10000, 1024, 1024), (1, 0, 2), np.uint16),
    "u16_T": lambda: Permute((2000, 1024, 1024), (2, 1, 0), np.uint16),
    "u8_T": lambda: Permute((2000, 1024, 2048), (2, 1, 0), np.uint8),
    "u16_2d": lambda: Permute((2000, 1048576), (1, 0), np.uint16),
    "c4_swap": lambda: Permute((2000, 1024, 1024), (1, 0, 2), np.uint16),
    "rc_512": lambda: Permute((8192, 2048, 128), (1, 0, 2), np.float32),
    "rc_1k": lambda: Permute((8192, 1024, 256), (1, 0, 2), np.float32),
    "rc_4k": lambda: Permute((4096, 512, 1024), (1, 0, 2), np.float32),
    "rc_16k": lambda: Permute((2048, 256, 4096), (1, 0, 2), np.float32),
    "rc_c4half": lambda: Permute((5008, 1024, 1024), (1, 0, 2), np.uint16),
    "t64_mean_cols": lambda: Reduce(0, 1, 4096, 2097152, np.float32, np.float32),
    "t64_std_cols": lambda: Reduce(2, 1, 4096, 2097152, np.float32, np.float32),
    "t64f_mean_cols": lambda: Reduce(0, 1, 8192, 2097152, np.float32, np.float32),
    "t64f_std_cols": lambda: Reduce(2, 1, 8192, 2097152, np.float32, np.float32),
    "c4_var_cols": lambda: Reduce(1, 1, 2000, 1024 * 1024, np.uint16, np.float64),
    "c4_var_full": lambda: Reduce(1, 1, 10000, 1024 * 1024, np.uint16, np.float64),
    "u16_var_rows": lambda: Reduce(1, 1024 * 1024, 2000, 1, np.uint16, np.float64),
    "c5_T": lambda: Permute((64, 64, 64, 64, 64), (4, 3, 2, 1, 0), np.float64),
    # statistics over every axis: a rows pass into chunk partials + the block combine
    "c1_mean_all": lambda: Reduce(0, 1, 100 * 64 * 64, 1, np.float64, np.float64),
    "c1_var_all": lambda: Reduce(1, 1, 100 * 64 * 64, 1, np.float64, np.float64),
    "c1_sum_all": lambda: Reduce(3, 1, 100 * 64 * 64, 1, np.float64, np.float64),
    "c2_mean_all": lambda: Reduce(0, 1, 2000 * 512 * 512, 1, np.float32, np.float32),
    "c2_var_all": lambda: Reduce(1, 1, 2000 * 512 * 512, 1, np.float32, np.float32),
    "c5_perm": lambda: Permute((64, 64, 64, 64, 64), (2, 0, 4, 1, 3), np.float64),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--ops", default=",".join(OPS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--placements", type=int, default=1, help="separate buffer allocations per op")
    ap.add_argument("--check", action="store_true", help="compare every library's permute output with torch's")
    a = ap.parse_args()
    libs = [load(p) for p in a.libs]
    for name in a.ops.split(","):
        # --placements K: K separate allocations of the op's buffers (buffer
        # placement moves these kernels by up to ~25%, profiles/r03d_alloc_kind.log),
        # every library timed on every one, interleaved
        insts = [OPS[name]() for _ in range(a.placements)]
        times = [[[] for _ in libs] for _ in insts]
        for j, op in enumerate(insts):
            for _ in range(2):
                for k, lib in enumerate(libs):
                    op(lib)
                    if a.check and hasattr(op, "check") and _ == 0 and j == 0:
                        op.dst.fill_(0)
                        op(lib)
                        torch.cuda.synchronize()
                        if not op.check():
                            print("%-14s %-40s OUTPUT MISMATCH" % (name, a.libs[k].split("/")[-1]), flush=True)
        for _ in range(a.rounds):
            for j, op in enumerate(insts):
                for k, lib in enumerate(libs):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.reps):
                        op(lib)
                    e1.record()
                    e1.synchronize()
                    times[j][k].append(e0.elapsed_time(e1) / a.reps)
        for j, op in enumerate(insts):
            for k, p in enumerate(a.libs):
                ms = float(np.median(times[j][k]))
                tag = name if a.placements == 1 else "%s#%d" % (name, j)
                print("%-14s %-40s %8.4f ms  %8.1f GB/s  (min %.4f)" % (tag, p.split("/")[-1], ms,
                      op.bytes / ms / 1e6, min(times[j][k])), flush=True)
        del insts, op
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
