"""Device operations of the MI355X backend, on byte buffers (torch tensors).

Every array of the backend stores its local shard as a flat ``torch.uint8``
tensor in HBM; the numpy dtype and shape are host metadata.  The operations
here launch the libbolt_mi355x kernels on the current HIP stream of the
tensor's device (torch's stream: hipEvents on it time the kernels).

The backend is chosen per device: HIP for 'cuda' devices.  There is no CPU
fallback; a non-GPU device raises unless a backend has been registered for
it explicitly (the multi-process CPU tests register a reference executor to
check the distributed orchestration -- see tests/cpu_backend.py).
"""
import ctypes

import numpy as np

from bolt_amd.mi355x import _lib

_DTYPE_CODES = {
    np.dtype(np.bool_): _lib.BM_BOOL,
    np.dtype(np.uint8): _lib.BM_U8,
    np.dtype(np.int8): _lib.BM_I8,
    np.dtype(np.uint16): _lib.BM_U16,
    np.dtype(np.int16): _lib.BM_I16,
    np.dtype(np.uint32): _lib.BM_U32,
    np.dtype(np.int32): _lib.BM_I32,
    np.dtype(np.uint64): _lib.BM_U64,
    np.dtype(np.int64): _lib.BM_I64,
    np.dtype(np.float16): _lib.BM_F16,
    np.dtype(np.float32): _lib.BM_F32,
    np.dtype(np.float64): _lib.BM_F64,
}


def dtype_code(dtype):
    dt = np.dtype(dtype)
    if dt.byteorder == '>':
        raise NotImplementedError("big-endian dtype %s is not supported on MI355X" % dt)
    try:
        return _DTYPE_CODES[dt.newbyteorder('=')]
    except KeyError:
        raise NotImplementedError("statistics over dtype %s are not supported by the mi355x mode" % dt)


# Records up to PART_BYTES are staged whole (5 blocks per CU); larger ones are
# split into (record, part) tiles.  C5: the 32-KiB pack record whole 3.26 ms
# vs parts 3.45; the 46-KiB values_to_keys record parts 3.72 vs whole 3.85
# (profiles/r01_ab_recmap2.log)
PART_BYTES = 32768


def record_parts(rmap, src_rec, es, part_bytes=None):
    """Split a record map into <= 8 destination ranges whose source ranges fit
    ``part_bytes`` of LDS, as a flat [dlo, dhi, slo, shi, ...] list ([] = one
    whole-record tile).  Ranges are 16-B aligned; the split is taken only if
    the staged bytes stay within 1.25x of the record (halo rows re-read)."""
    part_bytes = PART_BYTES if part_bytes is None else part_bytes
    if src_rec * es <= part_bytes:
        return []
    al = max(1, 16 // es)
    n = rmap.size
    for k in range(2, 9):
        cut = [(n * i // k) // al * al for i in range(k)] + [n]
        if any(b <= a for a, b in zip(cut[:-1], cut[1:])):
            break
        out, staged, widest = [], 0, 0
        for a, b in zip(cut[:-1], cut[1:]):
            seg = rmap[a:b]
            slo = int(seg.min()) // al * al
            shi = min(src_rec, -(-(int(seg.max()) + 1) // al) * al)
            out += [a, b, slo, shi]
            staged += shi - slo
            widest = max(widest, shi - slo)
        if widest * es <= part_bytes and staged <= 1.25 * src_rec:
            return out
    return []


STAGE_MASK_MIN_SKIP = 0.05  # stage masks only when they keep at least this share of units in HBM


def stage_mask(rmap, parts, es):
    """(uint32 mask [nparts x words], words) of the 16-B units of each part's
    source range [slo, shi) that its map entries read, or (None, 0) when there
    are no parts or the mask would skip less than STAGE_MASK_MIN_SKIP of the
    staged units (values_to_keys skips the moved axis' halo rows: ~16% on C5)."""
    if not parts:
        return None, 0
    p4 = np.asarray(parts, dtype=np.int64).reshape(-1, 4)
    units = [(-(-(int(shi - slo) * es) // 16)) for _, _, slo, shi in p4]
    words = max(1, -(-max(units) // 32))
    mask = np.zeros((len(p4), words * 32), dtype=bool)
    for k, (dlo, dhi, slo, shi) in enumerate(p4):
        mask[k, ((np.asarray(rmap[dlo:dhi], dtype=np.int64) - slo) * es) // 16] = True
    if 1.0 - mask.sum() / float(sum(units)) < STAGE_MASK_MIN_SKIP:
        return None, 0
    # bit j of word w is unit 32 w + j
    m = mask.reshape(len(p4), words, 32).astype(np.uint64)
    words32 = (m << np.arange(32, dtype=np.uint64)).sum(axis=2).astype(np.uint32)
    return np.ascontiguousarray(words32.reshape(-1)), words


def raw_stream(device):
    """Handle of torch's current HIP stream on ``device`` (what
    ``torch.cuda.current_stream(device).cuda_stream`` returns, without building
    a Stream object: ~2 us less per launch, profiles/r01_host_breakdown.log)."""
    global _raw_stream_of
    if _raw_stream_of is None:
        import torch
        _raw_stream_of = torch._C._cuda_getCurrentRawStream
    idx = device.index
    if idx is None:
        import torch
        idx = torch.cuda.current_device()
    return _raw_stream_of(idx)


_raw_stream_of = None  # torch._C._cuda_getCurrentRawStream, bound on first use


class HipBackend(object):
    """Launches libbolt_mi355x kernels on torch's current stream.  Between GPUs
    its records move over the library's own RCCL communicator only."""

    name = "hip"
    transport = "rccl"

    def __init__(self):
        self.lib = _lib.load()
        self._maps = {}  # (device, geometry key) -> resident int32 record map
        self._args = {}  # (shape, perm) -> ctypes arguments of bm_permute
        self._cargs = {}  # (shape, strides, strides) -> ctypes arrays of bm_copy_strided
        self._ws = {}    # reduction -> workspace bytes

    # Pointer and stream arguments go to ctypes as plain ints (the argtypes
    # are c_void_p): no c_void_p object per argument on the launch path.
    @staticmethod
    def _stream(t):
        return raw_stream(t.device)

    @staticmethod
    def _ptr(t, off=0):
        return t.data_ptr() + int(off)

    def host_writable(self, t):
        """True if kernels can store into host tensor ``t`` at its own address."""
        ok = ctypes.c_int(0)
        _lib.check(self.lib.bm_host_writable(self._ptr(t), t.numel() * t.element_size(), ctypes.byref(ok)),
                   "bm_host_writable")
        return bool(ok.value)

    def copy_strided(self, src, src_off, dst, dst_off, shape, sstrides, dstrides, es):
        """dst[dst_off + idx . dstrides] = src[src_off + idx . sstrides] (offsets in bytes)."""
        nd = len(shape)
        if nd == 0:
            shape, sstrides, dstrides, nd = [1], [1], [1], 1
        # the swap's launch path repeats one (shape, strides) per call: its
        # three int64 arrays are built once (~5 us of ctypes per call)
        key = (tuple(shape), tuple(sstrides), tuple(dstrides))
        args = self._cargs.get(key)
        if args is None:
            args = (_lib.i64_array(shape), _lib.i64_array(sstrides), _lib.i64_array(dstrides))
            if len(self._cargs) > 4096:
                self._cargs.clear()
            self._cargs[key] = args
        rc = self.lib.bm_copy_strided(self._ptr(src, src_off), self._ptr(dst, dst_off), nd,
                                      args[0], args[1], args[2], int(es), self._stream(src))
        if rc:
            _lib.check(rc, "bm_copy_strided")

    def permute(self, src, shape, perm, es, dst):
        key = (tuple(shape), tuple(perm))
        args = self._args.get(key)
        if args is None:
            args = (len(shape), _lib.i64_array(shape), _lib.i32_array(perm))
            if len(self._args) > 4096:
                self._args.clear()
            self._args[key] = args
        rc = self.lib.bm_permute(src.data_ptr(), dst.data_ptr(), args[0], args[1], args[2], es,
                                 raw_stream(src.device))
        if rc:
            _lib.check(rc, "bm_permute")

    def gather_rows(self, src, src_off, dst, dst_off, n_outer, src_rows, row_bytes, idx):
        """dst[a, j, :] = src[a, idx[j], :] (byte offsets; idx a host int64 array, bounds-checked)."""
        import torch
        idx = np.ascontiguousarray(idx, dtype=np.int64).reshape(-1)
        if idx.size == 0 or n_outer == 0:
            return
        if idx.min() < 0 or idx.max() >= src_rows:
            raise IndexError("gather index out of range [0, %d)" % src_rows)
        # page-locked + non-blocking: the upload queues behind earlier kernels
        # without blocking the host (the caching host allocator keeps the
        # pinned block until the copy has run)
        didx = torch.from_numpy(idx).pin_memory().to(src.device, non_blocking=True)
        _lib.check(self.lib.bm_gather_rows(self._ptr(src, src_off), self._ptr(dst, dst_off), int(n_outer),
                                           int(src_rows), int(row_bytes), ctypes.c_void_p(didx.data_ptr()),
                                           int(idx.size), self._stream(src)), "bm_gather_rows")
        # the caching allocator must not hand the index buffer out before the kernel has read it
        didx.record_stream(torch.cuda.current_stream(src.device))

    def _drop_maps(self, device):
        """Forget the resident maps.  Kernels queued on any stream may still read
        them, and the caching allocator would hand their blocks out again as
        soon as the last reference goes: wait for the device first (rare: the
        cache holds 256 geometries)."""
        import torch
        torch.cuda.synchronize(device)
        self._maps.clear()

    def record_gather(self, src, src_off, dst, dst_off, nrec, src_rec, dst_rec, rmap, key, es):
        """dst[r*dst_rec + o] = src[r*src_rec + rmap[o]] (elements; offsets in bytes).

        rmap: host int32 array of dst_rec entries in [0, src_rec), uploaded once
        per (device, key) and kept resident.
        """
        import torch
        ck = (src.device, key)
        hit = self._maps.get(ck)
        if hit is None:
            rmap = np.ascontiguousarray(rmap, dtype=np.int32)
            if rmap.size != dst_rec or rmap.min() < 0 or rmap.max() >= src_rec:
                raise ValueError("record map does not match the record sizes")
            parts = record_parts(rmap, int(src_rec), int(es))
            mask, words = stage_mask(rmap, parts, int(es))
            hit = (torch.from_numpy(rmap).to(src.device), len(parts) // 4,
                   _lib.i64_array(parts) if parts else None,
                   torch.from_numpy(mask).to(src.device) if mask is not None else None, words)
            if len(self._maps) >= 256:  # bounded: maps of at most 64-KiB records each
                self._drop_maps(src.device)
            self._maps[ck] = hit
        dmap, nparts, parts, dmask, words = hit
        _lib.check(self.lib.bm_record_gather_masked(self._ptr(src, src_off), self._ptr(dst, dst_off), int(nrec),
                                                    int(src_rec), int(dst_rec), ctypes.c_void_p(dmap.data_ptr()),
                                                    nparts, parts,
                                                    ctypes.c_void_p(dmask.data_ptr()) if dmask is not None else None,
                                                    words, int(es), self._stream(src)), "bm_record_gather_masked")

    def record_scatter(self, src, src_off, dst, dst_off, nrec, src_rec, group, gstride, plan, key, es):
        """dst[(r//group)*gstride + map_a[p] + (r%group)*map_b[p]] = src[r*src_rec + p]
        (elements; offsets in bytes).  plan = (map_a, map_b, vec) on the host,
        uploaded once per (device, key) and kept resident."""
        import torch
        ck = (src.device, key)
        hit = self._maps.get(ck)
        if hit is None:
            map_a, map_b, vec = plan
            if map_a.size != src_rec or map_b.size != src_rec:
                raise ValueError("scatter maps do not match the record size")
            da = torch.from_numpy(np.ascontiguousarray(map_a, dtype=np.int32)).to(src.device)
            db = (torch.from_numpy(np.ascontiguousarray(map_b, dtype=np.int32)).to(src.device)
                  if group > 1 else None)
            hit = (da, db, int(vec))
            if len(self._maps) >= 256:  # bounded: maps of at most 64-KiB records each
                self._drop_maps(src.device)
            self._maps[ck] = hit
        da, db, vec = hit
        _lib.check(self.lib.bm_record_scatter(self._ptr(src, src_off), self._ptr(dst, dst_off), int(nrec),
                                              int(src_rec), int(group), int(gstride),
                                              ctypes.c_void_p(da.data_ptr()),
                                              ctypes.c_void_p(db.data_ptr()) if db is not None else None,
                                              vec, int(es), self._stream(src)), "bm_record_scatter")

    def record_runs(self, src, src_off, dst, dst_off, nrec, src_rec, group, gstride, runs, key, es):
        """Run b of record r = g*group + k: dst[g*gstride + a_b + k*m_b + j] =
        src[r*src_rec + s_b + j], j < len_b (bm_record_runs; runs = (table
        [s, len, a, m] in vec_bytes vectors, vec_bytes) from
        plan.scatter_to_runs, checked here against the record and destination
        sizes and uploaded once per (device, key))."""
        import torch
        ck = (src.device, key)
        hit = self._maps.get(ck)
        if hit is None:
            table, vb = runs
            t = np.ascontiguousarray(table, dtype=np.int64).reshape(-1, 4)
            per = vb // int(es)
            s0, ln, a, m = t[:, 0] * per, t[:, 1] * per, t[:, 2] * per, t[:, 3] * per
            if (t.size == 0 or (ln <= 0).any() or (s0 < 0).any() or (s0 + ln > src_rec).any() or (a < 0).any()
                    or (m < 0).any() or (a + (group - 1) * m + ln > gstride).any()):
                raise ValueError("record runs do not fit the records")
            t = t[np.argsort(t[:, 2], kind="stable")]
            ends = t[:, 2] + int(group) * t[:, 1]
            tiled = (t.shape[0] <= 64 and np.array_equal(t[:, 1], t[:, 3]) and t[0, 2] == 0 and
                     np.array_equal(t[1:, 2], ends[:-1]) and ends[-1] * vb == int(gstride) * int(es))
            hit = (torch.from_numpy(t.reshape(-1).copy()).to(src.device), t.shape[0], int(vb),
                   _lib.RUNS_TILED if tiled else 0)
            if len(self._maps) >= 256:
                self._drop_maps(src.device)
            self._maps[ck] = hit
        table, n, vb, flags = hit
        _lib.check(self.lib.bm_record_runs(self._ptr(src, src_off), self._ptr(dst, dst_off), int(nrec), int(src_rec),
                                           int(group), int(gstride), int(n), ctypes.c_void_p(table.data_ptr()),
                                           vb, flags, int(es), self._stream(src)), "bm_record_runs")

    def _workspace(self, stat, code, O, R, I, device):
        import torch
        key = (stat, code, O, R, I)
        nb = self._ws.get(key)
        if nb is None:
            n = ctypes.c_size_t(0)
            _lib.check(self.lib.bm_reduce_workspace_bytes(stat, code, O, R, I, ctypes.byref(n)),
                       "bm_reduce_workspace_bytes")
            nb = self._ws[key] = n.value
        if nb == 0:
            return None, 0
        return torch.empty(nb, dtype=torch.uint8, device=device), nb

    def reduce(self, stat, src, code, O, R, I, out, out_code):
        ws, nws = self._workspace(stat, code, O, R, I, src.device)
        rc = self.lib.bm_reduce(stat, src.data_ptr(), code, O, R, I, out.data_ptr(), out_code,
                                ws.data_ptr() if ws is not None else None, nws, raw_stream(src.device))
        if rc:
            _lib.check(rc, "bm_reduce")

    def reduce_rows(self, stat, src, code, O, R, pitch, out, out_code):
        """reduce over O rows of R elements that start ``pitch`` elements apart."""
        ws, nws = self._workspace(stat, code, O, R, 1, src.device)
        rc = self.lib.bm_reduce_rows(stat, src.data_ptr(), code, O, R, pitch, out.data_ptr(), out_code,
                                     ws.data_ptr() if ws is not None else None, nws, raw_stream(src.device))
        if rc:
            _lib.check(rc, "bm_reduce_rows")

    def state_bytes(self, stat, code, nout):
        n = ctypes.c_size_t(0)
        _lib.check(self.lib.bm_reduce_state_bytes(stat, code, nout, ctypes.byref(n)), "bm_reduce_state_bytes")
        return n.value

    def reduce_state(self, stat, src, code, O, R, I, state):
        ws, nws = self._workspace(stat, code, O, R, I, src.device)
        _lib.check(self.lib.bm_reduce_state(stat, self._ptr(src), code, O, R, I, self._ptr(state),
                                            self._ptr(ws) if ws is not None else None, nws,
                                            self._stream(src)), "bm_reduce_state")

    def reduce_combine(self, stat, code, states, counts, nout, out, out_code):
        _lib.check(self.lib.bm_reduce_combine(stat, code, self._ptr(states), _lib.i64_array(counts),
                                              len(counts), nout, self._ptr(out), out_code,
                                              self._stream(states)), "bm_reduce_combine")


_BACKENDS = {}


def register_backend(device_type, backend):
    """Install a backend for a torch device type (test executors only: the numpy
    executor on 'cpu', the host-staged one-GPU rehearsal on 'cuda').  A
    backend's ``transport`` attribute names how its contexts exchange records
    across ranks ("rccl", or "torch" / "host" for test executors)."""
    if backend is None:
        _BACKENDS.pop(device_type, None)
    else:
        _BACKENDS[device_type] = backend


def backend_for(device):
    kind = device.type
    if kind in _BACKENDS:
        return _BACKENDS[kind]
    if kind == "cuda":
        _BACKENDS["cuda"] = HipBackend()
        return _BACKENDS["cuda"]
    raise RuntimeError("bolt_amd: device %s has no backend; the mi355x mode runs on MI355X GPUs "
                       "(HIP) and has no CPU fallback" % device)
