"""BoltArrayMI355X: the 'mi355x' mode array (drop-in for BoltArraySpark's hot path).

Data layout.  The logical array is C-order (keys..., values...) -- one record
is one contiguous value block, exactly the order of the Spark path's sorted
records (bolt/spark/array.py:1006-1014).  Each rank holds a slab of the
leading key axis as a flat uint8 tensor in HBM; shape/split/dtype are host
metadata (array.py:15-28).

Operations and what replaces the Spark machinery:
  swap / transpose / T / swapaxes / Keys.transpose / Values.transpose:
      the net permutation (plan.swap_perm, array.py:716-808) as ONE permute
      kernel (bm_permute); across GPUs pack -> RCCL all-to-all -> unpack.
  chunk: ChunkedArrayMI355X (chunk.py), the packed chunk layout in HBM.
  sum / mean / var / std: one reduction kernel over the aligned layout
      (array.py:243-395 + statcounter.py), float64 accumulation; across GPUs
      per-rank states -> all_gather -> ordered Chan combine.
  toarray / tolocal: D2H (+ all_gather of the slabs).
"""
import functools
import os

import numpy as np

from bolt_amd.mi355x import _lib
from bolt_amd.mi355x._ops import backend_for, dtype_code
from bolt_amd.base import BoltArray
from bolt_amd.mi355x.context import local_shape
from bolt_amd.mi355x.dist import all_gather_bytes, concat_rows_sharded, gather_to_host, permute_sharded, redistribute_rows, select_sharded, _empty
from bolt_amd.mi355x.transfer import finish_host_result, host_result, to_device, to_host
from bolt_amd.local import BoltArrayLocal
from bolt_amd.mi355x.plan import getplan, check_plan, padded_strides, swap_perm, swap_shape, reduce_layout, stat_dtype
from bolt_amd.utils import tupleize, argpack, inshape, istransposeable, isreshapeable

_STAT_CODES = {'mean': _lib.STAT_MEAN, 'variance': _lib.STAT_VAR, 'stdev': _lib.STAT_STD}


def _ufunc_stats():
    """reduce(func) functions that run as one bm_reduce mode (array.py:243-282)."""
    import operator
    return {operator.add: _lib.STAT_SUM, np.add: _lib.STAT_SUM,
            np.maximum: _lib.STAT_MAX, np.minimum: _lib.STAT_MIN,
            operator.mul: _lib.STAT_PROD, np.multiply: _lib.STAT_PROD,
            np.logical_and: _lib.STAT_LAND, np.logical_or: _lib.STAT_LOR,
            np.bitwise_and: _lib.STAT_BAND, operator.and_: _lib.STAT_BAND,
            np.bitwise_or: _lib.STAT_BOR, operator.or_: _lib.STAT_BOR,
            np.bitwise_xor: _lib.STAT_BXOR, operator.xor: _lib.STAT_BXOR,
            np.fmax: _lib.STAT_FMAX, np.fmin: _lib.STAT_FMIN}


_UFUNC_STATS = _ufunc_stats()


def _hashable(f):
    try:
        hash(f)
        return True
    except TypeError:
        return False


def _tree(func, recs):
    """((r0 f r1) f (r2 f r3)) ... over the leading axis of a device tensor."""
    import torch
    from bolt_amd.mi355x.functional import apply_pairs
    while recs.shape[0] > 1:
        n = recs.shape[0]
        nxt = apply_pairs(func, recs[0:n - 1:2], recs[1:n:2])
        if n % 2:
            nxt = torch.cat([nxt, recs[n - 1:].to(nxt.dtype)])
        recs = nxt
    return recs[0]
# reductions whose result keeps the input dtype (numpy's same-dtype ufunc rule)
_MOMENTS = (_lib.STAT_MEAN, _lib.STAT_VAR, _lib.STAT_STD)
_KEEP_DTYPE = (_lib.STAT_SUM, _lib.STAT_MAX, _lib.STAT_MIN, _lib.STAT_PROD, _lib.STAT_BAND,
               _lib.STAT_BOR, _lib.STAT_BXOR, _lib.STAT_FMAX, _lib.STAT_FMIN)


@functools.lru_cache(maxsize=256)
def _plan_ok(vshape, dtype, size):
    try:
        plan, pad = getplan(vshape, dtype, size, None, None)
        check_plan(plan, pad, vshape)
    except Exception as e:  # cache the failure too; re-raised below
        return e
    return None


def _check_swap_plan(vshape, dtype, size):
    """getplan + _chunk's checks for the swap's chunk size (chunk.py:120-129), cached."""
    try:
        err = _plan_ok(tuple(vshape), np.dtype(dtype), size)
    except TypeError:  # unhashable size: validate uncached
        plan, pad = getplan(vshape, dtype, size, None, None)
        check_plan(plan, pad, vshape)
        return
    if err is not None:
        raise type(err)(*err.args)


_SWAP_PLANS = {}   # (shape, split, dtype, kaxes, vaxes, size) -> (_move_plan, squeezed shape | None) | _NOOP
_NOOP = object()


def _move_plan(shape, perm, split):
    """What x.transpose(perm) with the given split needs, from the shape alone:
    (perm, split, new shape, identity, only unit axes move)."""
    perm = tuple(int(p) for p in perm)
    moved = [p for p in perm if shape[p] != 1]
    return (perm, int(split), tuple(shape[p] for p in perm), perm == tuple(range(len(shape))),
            moved == sorted(moved))


# Row pitch of transposed results.  A transpose writes its destination rows in
# 256-B tile segments; rows whose length is not a multiple of the 128-B line
# start mid-line (C2's 2000 float32 = 8000 B: every other row), so
# neighbouring tiles write parts of the same lines.  Such a result is stored
# with its rows padded to a 256-B multiple (C2: 8192 B): the C2 transpose
# 0.729 -> 0.675 ms, its time-axis statistics 0.298 -> 0.301-0.305 ms, the
# step -2.8% (profiles/r05s_pitch_prof.txt, r05s_pitch_ab.log; pitch sweep
# r05t_pitch_sweep.txt); other shapes gain more: float32 rows of 4400 B
# 2.26 -> 1.65 ms, of 12000 B 1.34 -> 1.18, C4's uint16 .T (20000-B rows)
# 9.2 -> 8.1 ms (r05zw_pitch_align.log: 256-B steps are the best or near it
# everywhere; 1 KiB steps lose 8% on the uint16 rows); rows of 2000 / 3000 B
# +10-16%, but 1000-B rows padded to 1024 lose 16%, hence the 1536-B floor
# (r05zz_short_rows.log).  Statistics over the
# last axis read the padded rows in place (bm_reduce_rows); swaps,
# transposes, indexing, map / filter / chunk of single-row records, column
# statistics and elementwise ops read them too; the rest compacts the rows
# once (_compact).  ROW_PITCH = False turns padding off (the tests' switch;
# the sweeps that chose the constants ran on round-5 builds with them as
# environment knobs: tools/pitch_sweep.sh, tools/pitch_align_sweep.sh).
ROW_PITCH = True
_PITCH_MIN_ROW = 1536   # bytes: shorter rows are not padded
_PITCH_ALIGN = 256      # bytes: padded rows start on this boundary
_PITCH_LINE = 128       # bytes: rows of a multiple of this stay dense
_PITCH_PAD_DIV = 16     # at most 1/16 of a row is padding
_PITCH_PLANS = {}  # (_move_plan, itemsize) -> None | pitched copy plan


def _pitch_plan(mv, shape, es):
    """The pitched copy for _move_plan ``mv`` of an array of ``shape``, or None:
    (pitch in elements, rows, output shape, source strides, pitched
    destination strides), all in elements."""
    perm, _, new_shape, _, _ = mv
    nd = len(new_shape)
    if nd < 2 or perm[-1] == nd - 1:
        return None
    R = new_shape[-1]
    rb = R * es
    if rb < _PITCH_MIN_ROW or rb % _PITCH_LINE == 0:
        return None
    pb = -(-rb // _PITCH_ALIGN) * _PITCH_ALIGN
    if (pb - rb) * _PITCH_PAD_DIV > rb or pb % es:
        return None
    P = pb // es
    rows = int(np.prod(new_shape[:-1], dtype=np.int64))
    if rows < 2:
        return None
    sstr = [1] * len(shape)
    for k in range(len(shape) - 2, -1, -1):
        sstr[k] = sstr[k + 1] * shape[k + 1]
    return P, rows, list(new_shape), [sstr[p] for p in perm], _padded_strides(new_shape, P)


_DEVICE_BYTES = {}  # device index -> total HBM bytes


def _pitch_fits(pp, es, device):
    """Room for the padded result AND a later dense compaction of it (a
    consumer that needs dense records copies them once, see _compact): checked
    against the device's free memory (plus what torch's allocator holds
    unused) only when the two together exceed 1/8 of the device, so the small
    results of a hot loop never query the driver."""
    if device.type != "cuda":
        return True
    import torch
    P, rows, oshape = pp[0], pp[1], pp[2]
    need = rows * (P + oshape[-1]) * es
    idx = device.index if device.index is not None else torch.cuda.current_device()
    total = _DEVICE_BYTES.get(idx)
    if total is None:
        total = _DEVICE_BYTES[idx] = torch.cuda.get_device_properties(idx).total_memory
    if need * 8 <= total:
        return True
    free = torch.cuda.mem_get_info(idx)[0] + torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
    return need <= free


_padded_strides = padded_strides


@functools.lru_cache(maxsize=1024)
def _aligned_vshape_of(shape, split, axis):
    """BoltArrayMI355X._aligned_vshape for (shape, split, axes)."""
    tokeys = [a - split for a in axis if a >= split]
    tovalues = [a for a in range(split) if a not in axis]
    if not (tokeys or tovalues):
        return None
    ref = swap_shape(shape, split, tovalues, tokeys)
    if ref is None:
        return None
    vs = ref[0][ref[1]:]
    kept = tuple(d for i, d in enumerate(shape) if i not in set(axis))
    return None if vs == kept else vs


_REDUCE_PLANS = {}  # (local shape, axes, stat, dtype, world) -> device reduction plan
_STAT_AXES = {}  # (shape, split, axis as given) -> (validated axes, records after _align, record shape | None)


class BoltArrayMI355X(BoltArray):

    _metadata = {
        '_shape': None,
        '_split': None,
        '_dtype': None,
        '_ordered': True,
    }

    def __init__(self, data, shape=None, split=None, dtype=None, ordered=True, context=None,
                 npartitions=None):
        self._data = data
        self._shape = tuple(int(s) for s in shape)
        self._split = int(split)
        self._dtype = np.dtype(dtype)
        self._mode = 'mi355x'
        self._ordered = ordered
        self._ctx = context
        self._npartitions = npartitions

    # ------------------------------------------------------------ creation
    @property
    def _constructor(self):
        return BoltArrayMI355X

    @classmethod
    def _ingest(cls, arry, permutation, shape, split, dtype, ctx, npartitions):
        """Host ndarray -> sharded device array (spark/construct.py:43-70).

        Records are ``arry.transpose(permutation)`` in C order while the array
        keeps ``shape`` -- the reference takes the shape before transposing
        (construct.py:48 vs :55), so non-leading key axes come back as
        ``x.transpose(perm).reshape(x.shape)``; this is kept for parity.
        """
        import torch
        dev = ctx.device
        es = dtype.itemsize
        arry = np.ascontiguousarray(arry)
        identity = list(permutation) == list(range(len(shape)))
        lo, hi = ctx.local_bounds(shape[0])
        rowbytes = int(np.prod(shape[1:], dtype=np.int64)) * es
        if identity:
            data = to_device(arry[lo:hi].reshape(-1).view(np.uint8), dev)
        elif ctx.world_size == 1:
            # whole array to HBM, permuted on the GPU (the reference's records
            # are x.transpose(perm) reshaped to the old shape)
            full = to_device(arry.reshape(-1).view(np.uint8), dev)
            data = _empty(full.numel(), dev)
            if full.numel():
                backend_for(dev).permute(full, arry.shape, permutation, es, data)
        else:
            # this rank's slab is the flat element range [s, e) of
            # x.transpose(perm): upload only the source planes along axis
            # perm[0] that cover it, permute them on the GPU, cut the range
            pshape = tuple(arry.shape[i] for i in permutation)
            inner0 = int(np.prod(pshape[1:], dtype=np.int64))
            s0, e0 = lo * (rowbytes // es), hi * (rowbytes // es)
            if e0 == s0 or inner0 == 0:
                data = _empty(0, dev)
            else:
                i_lo, i_hi = s0 // inner0, min(pshape[0], -(-e0 // inner0))
                idx = [slice(None)] * arry.ndim
                idx[permutation[0]] = slice(i_lo, i_hi)
                sub = np.ascontiguousarray(arry[tuple(idx)])
                part = to_device(sub.reshape(-1).view(np.uint8), dev)
                perm_bytes = _empty(part.numel(), dev)
                backend_for(dev).permute(part, sub.shape, permutation, es, perm_bytes)
                off = (s0 - i_lo * inner0) * es
                data = perm_bytes[off:off + (e0 - s0) * es]
                if data.numel() != perm_bytes.numel():
                    data = data.clone()
        return cls(data, shape=shape, split=split, dtype=dtype, context=ctx, npartitions=npartitions)

    @classmethod
    def _filled(cls, value, shape, split, dtype, ctx, npartitions):
        """ones/zeros: one record built on the host, broadcast on the GPU (spark/construct.py:207-222)."""
        import torch
        dev = ctx.device
        es = dtype.itemsize
        lshape = local_shape(ctx, shape)
        n = int(np.prod(lshape, dtype=np.int64))
        data = _empty(n * es, dev)
        if n:
            unit = to_device(np.full(1, value, dtype=dtype).view(np.uint8), dev)
            backend_for(dev).copy_strided(unit, 0, data, 0, [n], [0], [1], es)
        return cls(data, shape=shape, split=split, dtype=dtype, context=ctx, npartitions=npartitions)

    @classmethod
    def _from_shard(cls, shard, shape, split, dtype, ctx, npartitions):
        import torch
        dev = ctx.device
        if isinstance(shard, np.ndarray):
            dtype = np.dtype(dtype or shard.dtype)
            data = to_device(np.ascontiguousarray(shard, dtype=dtype).reshape(-1).view(np.uint8), dev)
        else:
            if dtype is None:
                raise ValueError("dtype is required for a device shard")
            dtype = np.dtype(dtype)
            t = shard.contiguous()
            data = t.view(torch.uint8).reshape(-1) if t.dtype != torch.uint8 else t.reshape(-1)
            if data.device != dev:
                data = data.to(dev)
        want = int(np.prod(local_shape(ctx, shape), dtype=np.int64)) * dtype.itemsize
        if data.numel() != want:
            raise ValueError("shard holds %d bytes, rank %d of %s needs %d"
                             % (data.numel(), ctx.rank, str(shape), want))
        if split < 1 or split > len(shape):
            raise ValueError("split axis must be in [1, %d], got %d" % (len(shape), split))
        return cls(data, shape=shape, split=split, dtype=dtype, context=ctx, npartitions=npartitions)

    def _like(self, data, shape, split, dtype=None):
        return BoltArrayMI355X(data, shape=shape, split=split, dtype=self._dtype if dtype is None else dtype,
                               context=self._ctx, npartitions=self._npartitions)

    def _derive(self, data, shape, split):
        """_like for a ``shape`` that is already a tuple of ints and the same
        dtype: the constructor's coercions skipped (the swap's launch path)."""
        new = object.__new__(BoltArrayMI355X)
        new.__dict__.update(_data=data, _shape=shape, _split=split, _dtype=self._dtype, _mode='mi355x',
                            _ordered=True, _ctx=self._ctx, _npartitions=self._npartitions)
        return new

    def __getattr__(self, name):
        # only reached for attributes not set: a row-padded array's records
        # (see ROW_PITCH) are compacted the first time anything needs them dense
        if name == "_data" and "_pbuf" in self.__dict__:
            return self._compact()
        raise AttributeError("'%s' object has no attribute '%s'" % (type(self).__name__, name))

    def _compact(self):
        """Dense records of a row-padded array (one strided copy on the GPU)."""
        d = self.__dict__
        pbuf, P = d["_pbuf"], d["_pitch"]
        es = self._dtype.itemsize
        R = self._shape[-1]
        rows = int(np.prod(self._local_shape[:-1], dtype=np.int64))
        data = _empty(rows * R * es, pbuf.device)
        if rows and R:
            backend_for(pbuf.device).copy_strided(pbuf, 0, data, 0, [rows, R], [P, 1], [R, 1], es)
        d["_data"] = data
        del d["_pbuf"], d["_pitch"]
        return data

    def _derive_padded(self, pbuf, pitch, shape, split):
        """_derive for records stored with padded rows (see ROW_PITCH)."""
        new = self._derive(None, shape, split)
        nd = new.__dict__
        del nd["_data"]
        nd["_pbuf"], nd["_pitch"] = pbuf, pitch
        return new

    @property
    def _device(self):
        d = self.__dict__
        return (d["_pbuf"] if "_pbuf" in d else d["_data"]).device

    @property
    def _backend(self):
        return backend_for(self._device)

    @property
    def _local_shape(self):
        # shape and context never change after construction: computed once
        ls = self.__dict__.get("_lshape")
        if ls is None:
            ls = self.__dict__["_lshape"] = local_shape(self._ctx, self._shape)
        return ls

    # ---------------------------------------------------------- properties
    @property
    def shape(self):
        return self._shape

    @property
    def size(self):
        return int(np.prod(self._shape))

    @property
    def ndim(self):
        return len(self._shape)

    @property
    def split(self):
        return self._split

    @property
    def dtype(self):
        return self._dtype

    @property
    def context(self):
        return self._ctx

    @property
    def mask(self):
        return tuple([1] * self._split + [0] * (self.ndim - self._split))

    @property
    def keys(self):
        from bolt_amd.mi355x.shapes import Keys
        return Keys(self)

    @property
    def values(self):
        from bolt_amd.mi355x.shapes import Values
        return Values(self)

    def cache(self):
        """Records are resident in HBM already (array.py:37-41); only the flag
        the record view reports changes."""
        self._cached = True

    def unpersist(self):
        """(array.py:43-47) -- the records stay in HBM; clears the flag."""
        self._cached = False

    # ------------------------------------------------------------ movement
    def _permute(self, perm, split):
        """x.transpose(perm) as a new array with the given split (one kernel / one all-to-all)."""
        return self._move(_move_plan(self._shape, perm, split))

    def _move(self, mv):
        """Run a _move_plan on this array."""
        perm, split, new_shape, relabel, units_only = mv
        if relabel or (units_only and (perm[0] == 0 or self._ctx.world_size == 1)):
            # no bytes move: the identity, or only unit axes move, so the C-order
            # bytes are already the result's (across GPUs the leading axis,
            # hence every slab, stays put)
            data = self._data
        elif ROW_PITCH and self._ctx.world_size == 1:
            es = self._dtype.itemsize
            pp = self._pitch_of(mv, es)
            d = self.__dict__
            if "_pbuf" in d:
                # a padded source is read in place: its strides, permuted
                src, pstr = d["_pbuf"], _padded_strides(self._shape, d["_pitch"])
                sstr = [pstr[p] for p in perm]
            else:
                src, sstr = self._data, None
            be = backend_for(src.device)
            if pp is not None:
                P, rows, oshape, psstr, dstr = pp
                pbuf = _empty(rows * P * es, src.device)
                be.copy_strided(src, 0, pbuf, 0, oshape, psstr if sstr is None else sstr, dstr, es)
                return self._derive_padded(pbuf, P, new_shape, split)
            if sstr is None:
                data = permute_sharded(self._ctx, be, src, self._shape, perm, es)
            else:
                n = int(np.prod(new_shape, dtype=np.int64))
                data = _empty(n * es, src.device)
                be.copy_strided(src, 0, data, 0, list(new_shape), sstr, _padded_strides(new_shape, new_shape[-1]), es)
        else:
            # across GPUs: the exchange's pack reads a padded source in place
            # and its unpack writes the result's rows at the same pitch rule
            # as on one GPU
            es = self._dtype.itemsize
            pp = self._pitch_of(mv, es) if ROW_PITCH else None
            d = self.__dict__
            src = d["_pbuf"] if "_pbuf" in d else self._data
            data = permute_sharded(self._ctx, backend_for(src.device), src, self._shape, perm, es,
                                   src_pitch=d.get("_pitch"), out_pitch=None if pp is None else pp[0])
            if pp is not None:
                return self._derive_padded(data, pp[0], new_shape, split)
        return self._derive(data, new_shape, split)

    def _pitch_of(self, mv, es):
        """The pitched copy plan of move ``mv`` (cached, see _pitch_plan), or
        None when the result stays dense or the device lacks room for it."""
        key = (mv, es)
        pp = _PITCH_PLANS.get(key, False)
        if pp is False:
            pp = _pitch_plan(mv, self._shape, es)
            if len(_PITCH_PLANS) > 4096:
                _PITCH_PLANS.clear()
            _PITCH_PLANS[key] = pp
        if pp is not None and not _pitch_fits(pp, es, self._device):
            return None
        return pp

    def chunk(self, size="150", axis=None, padding=None):
        """Chunk the values of every record (array.py:678-714) -> ChunkedArrayMI355X."""
        if type(size) is not str:
            size = tupleize((size))
        axis = tupleize((axis))
        padding = tupleize((padding))
        from bolt_amd.mi355x.chunk import ChunkedArrayMI355X
        return ChunkedArrayMI355X._from_array(self, size, axis, padding)

    def swap(self, kaxes, vaxes, size="150"):
        """Move key axes to the values and value axes to the keys (array.py:716-763).

        Same validation and result as the reference: x.transpose(P) with
        P = [keys kept] + [moved values] + [moved keys] + [values kept] and
        split' = split - #kaxes + #vaxes.  ``size`` only chooses the Spark
        chunking; it is validated the same way (getplan + _chunk checks) and
        does not change the result.  Executed as one permute kernel.
        """
        # host plan of an already validated (shape, split, dtype, axes, size):
        # first under the arguments as given, then canonicalised
        try:
            raw = (self._shape, self._split, self._dtype, kaxes, vaxes, size)
            hit = _SWAP_PLANS.get(raw)
        except TypeError:  # unhashable arguments (lists)
            raw = hit = None
        if hit is None:
            try:
                key = (self._shape, self._split, self._dtype, tuple(int(k) for k in tupleize(kaxes)),
                       tuple(int(v) for v in tupleize(vaxes)), size if type(size) is str else tupleize(size))
                hash(key)
            except (TypeError, ValueError):
                key = None
            hit = _SWAP_PLANS.get(key) if key is not None else None
            if hit is None:
                plan = self._swap_plan(kaxes, vaxes, size)
                if plan is None:
                    hit = _NOOP
                else:
                    mv = _move_plan(self._shape, *plan[:2])
                    ref = swap_shape(self._shape, self._split, *plan[2:])
                    # the reference's unit-axis squeezes (plan.swap_shape): a relabel
                    hit = (mv, ref[0] if ref is not None and ref[0] != mv[2] else None)
            if len(_SWAP_PLANS) > 4096:
                _SWAP_PLANS.clear()
            for k in (key, raw):
                if k is not None:
                    _SWAP_PLANS[k] = hit
        if hit is _NOOP:
            return self
        mv, squeezed = hit
        out = self._move(mv)
        return out if squeezed is None else out._relabel(squeezed)

    def _relabel(self, shape):
        """The same records under ``shape`` -- this shape with unit axes
        dropped, split unchanged (the reference's swap squeezes)."""
        d = self.__dict__
        if "_pbuf" in d and len(shape) >= 2 and shape[-1] == self._shape[-1]:
            return self._derive_padded(d["_pbuf"], d["_pitch"], shape, self._split)
        return self._derive(self._data, shape, self._split)

    def _swap_plan(self, kaxes, vaxes, size):
        """Validation and net permutation of swap: (perm, newsplit), or None for a no-op."""
        kaxes = np.asarray(tupleize(kaxes), 'int')
        vaxes = np.asarray(tupleize(vaxes), 'int')
        if type(size) is not str:
            size = tupleize(size)

        if len(kaxes) == self.keys.ndim and len(vaxes) == 0:
            raise ValueError('Cannot perform a swap that would '
                             'end up with all data on a single key')

        if len(kaxes) == 0 and len(vaxes) == 0:
            return None

        # the chunk plan the reference would build (errors surface the same way)
        if not (self._split == self.ndim):
            _check_swap_plan(self._shape[self._split:], self._dtype, size)
        # axes index boolean masks in the reference (chunk.py:224, :293):
        # negative axes count from the end, out-of-range ones raise IndexError
        nv = self.ndim - self._split
        for k in kaxes:
            if not -self._split <= k < self._split:
                raise IndexError("key axis %d out of range for %d keys" % (k, self._split))
        for v in vaxes:
            if not -nv <= v < nv:
                raise IndexError("value axis %d out of range for %d values" % (v, nv))
        kaxes = [int(k) % self._split for k in kaxes]
        vaxes = [int(v) % nv for v in vaxes] if nv else []

        return swap_perm(self.ndim, self._split, kaxes, vaxes) + (kaxes, vaxes)

    def transpose(self, *axes):
        """Permute the axes, split unchanged (array.py:765-808)."""
        if len(axes) == 0:
            p = np.arange(self.ndim - 1, -1, -1)
        else:
            p = np.asarray(argpack(axes))
        istransposeable(p, range(self.ndim))
        return self._permute([int(x) for x in p], self._split)

    @property
    def T(self):
        """Reverse the axes (array.py:810-815)."""
        return self.transpose()

    def swapaxes(self, axis1, axis2):
        """Interchange two axes (array.py:817-833)."""
        p = list(range(self.ndim))
        p[axis1] = axis2
        p[axis2] = axis1
        return self.transpose(p)

    def reshape(self, *shape):
        """Same data, new shape (array.py:835-877): only reshapes that split into
        an independent reshape of the keys and one of the values
        (NotImplementedError otherwise, as the reference).  On the dense
        layout both are metadata, plus a re-slab across GPUs when the leading
        key axis changes (shapes.py:40-64, :111-134)."""
        new = argpack(shape)
        isreshapeable(new, self.shape)
        if new == self.shape:
            return self
        i = self._reshapebasic(new)
        if i == -1:
            raise NotImplementedError("Currently no support for reshaping between "
                                      "keys and values for BoltArraySpark")
        return self.keys.reshape(new[:i]).values.reshape(new[i:])

    def _reshapebasic(self, shape):
        """Index in ``shape`` splitting it into key and value parts of the old
        key and value sizes, or -1 (array.py:861-877)."""
        new = tupleize(shape)
        old_key = int(np.prod(self.keys.shape, dtype=np.int64))
        old_val = int(np.prod(self.values.shape, dtype=np.int64))
        for i in range(len(new)):
            if int(np.prod(new[:i], dtype=np.int64)) == old_key and \
                    int(np.prod(new[i:], dtype=np.int64)) == old_val:
                return i
        return -1

    def astype(self, dtype, casting='unsafe'):
        """Cast every record to ``dtype`` (array.py:920-930), on the device.

        numpy's casting rule is checked on the host (np.can_cast raises the
        same TypeError numpy's astype would); the conversion itself is torch's
        elementwise cast, numpy's values for every finite in-range input."""
        from bolt_amd.mi355x import functional as F
        dtype = np.dtype(dtype)
        if not np.can_cast(self._dtype, dtype, casting):
            raise TypeError("Cannot cast array data from %r to %r according to the rule %r"
                            % (self._dtype, dtype, casting))
        d = self.__dict__
        if dtype == self._dtype:
            if "_pbuf" in d:
                return self._derive_padded(d["_pbuf"].clone(), d["_pitch"], self._shape, self._split)
            return self._like(self._data.clone(), self._shape, self._split)
        src = self._elements()
        out = F.as_bytes(src.to(F.torch_dtype(dtype)))
        return self._like(out, self._shape, self._split, dtype=dtype)

    def _elements(self, shape=None):
        """This rank's elements, in C order, as a torch view of ``shape``
        (default: flat -- for a row-padded array (rows, row length), a strided
        view of the padded rows, so elementwise work reads them in place)."""
        from bolt_amd.mi355x import functional as F
        d = self.__dict__
        if "_pbuf" in d:
            R = self._shape[-1]
            rows = int(np.prod(self._local_shape[:-1], dtype=np.int64))
            v = F.view(d["_pbuf"], (rows, d["_pitch"]), self._dtype)[:, :R]
            return v if shape is None else v.view(tuple(shape))
        n = self._data.numel() // max(1, self._dtype.itemsize)
        return F.view(self._data, (n,) if shape is None else tuple(shape), self._dtype)

    def clip(self, min=None, max=None):
        """Clip values below ``min`` / above ``max`` (array.py:932-945), on the device.

        The result dtype is numpy's for ``record.clip(min, max)`` (numpy is asked
        on a 1-element record, so its errors are numpy's too): a float bound on an
        integer array promotes.  torch has no max/min kernels for uint16/32/64,
        so unsigned records are compared in a wider signed type (uint64: with
        the sign bit flipped, which maps unsigned order onto signed order)."""
        import torch
        from bolt_amd.mi355x import functional as F
        rdt = np.zeros(1, self._dtype).clip(min=min, max=max).dtype
        x = self._elements(self._local_shape)
        vs = tuple(self._shape[self._split:])
        wide = {1: torch.int16, 2: torch.int32, 4: torch.int64}
        if rdt != self._dtype:
            x = x.to(F.torch_dtype(rdt))
        if rdt.kind == "u" and rdt.itemsize < 8:
            out, back = x.to(wide[rdt.itemsize]), F.torch_dtype(rdt)
        elif rdt.kind == "u":
            flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=x.device)
            out, back = x.view(torch.int64) ^ flip, None
        else:
            out, back = x.clone(), None
        for bound, fn in ((min, torch.maximum), (max, torch.minimum)):
            if bound is None:
                continue
            nb = np.asarray(bound).astype(rdt)
            if nb.ndim > len(vs):
                raise ValueError("clip bound of shape %s does not broadcast to records %s" % (nb.shape, vs))
            if rdt.kind == "u" and rdt.itemsize < 8:
                b = torch.as_tensor(nb.astype(np.int64), device=out.device).to(out.dtype)
            elif rdt.kind == "u":
                b = torch.as_tensor(nb.view(np.int64), device=out.device) ^ flip
            else:
                b = torch.as_tensor(nb, device=out.device)
            out = fn(out, b)
        if rdt.kind == "u":
            out = out.to(back) if back is not None else (out ^ flip).view(torch.uint64)
        return self._like(F.as_bytes(out.contiguous()), self._shape, self._split, dtype=rdt)

    def repartition(self, npartitions):
        """Records stay sharded one slab per GPU; only the partition count the
        array reports changes, and, as after Spark's repartition, the array is
        marked unordered (array.py:49-60)."""
        out = self._like(self._data, self._shape, self._split)
        out._npartitions = npartitions
        out._ordered = False
        return out

    # ---------------------------------------------------------- functional
    def stack(self, size=None):
        """Group each partition's records into stacks of up to ``size`` (array.py:62-83)."""
        from bolt_amd.mi355x.stack import StackedArrayMI355X
        return StackedArrayMI355X._from_array(self, size)

    def _align(self, axis):
        """Swap so that ``axis`` are exactly the keys (array.py:85-115)."""
        inshape(self.shape, axis)
        tokeys = [(a - self._split) for a in axis if a >= self._split]
        tovalues = [a for a in range(self._split) if a not in axis]
        if tokeys or tovalues:
            return self.swap(tovalues, tokeys)
        return self

    def first(self):
        """The first record's value, on the host (array.py:117-123)."""
        from bolt_amd.mi355x.dist import all_gather_bytes
        es = self._dtype.itemsize
        rec = int(np.prod(self._shape[self._split:], dtype=np.int64))
        rb = rec * es
        d = self.__dict__
        if "_pbuf" in d and rec > self._shape[-1]:
            # padded rows: gather the first record's rows, no compaction
            R = self._shape[-1]
            buf = _empty(rb, d["_pbuf"].device)
            self._backend.copy_strided(d["_pbuf"], 0, buf, 0, [rec // R, R], [d["_pitch"], 1], [R, 1], es)
        elif "_pbuf" in d:
            buf = d["_pbuf"][:rb]  # within the first row
        else:
            buf = self._data[:rb]
        if self._ctx.world_size > 1:
            lo, hi = self._ctx.bounds(self._shape[0])[0]
            sizes = [rb if r == 0 else 0 for r in range(self._ctx.world_size)]
            buf = all_gather_bytes(self._ctx, buf if self._ctx.rank == 0 else buf[:0], sizes)
        return BoltArrayLocal(to_host(buf, self._dtype, self._shape[self._split:]))

    def _records_tensor(self):
        """This rank's records as a (records, *value shape) torch view."""
        from bolt_amd.mi355x import functional as F
        lshape = self._local_shape
        nrec = int(np.prod(lshape[:self._split], dtype=np.int64))
        vshape = tuple(self._shape[self._split:])
        d = self.__dict__
        if "_pbuf" in d and vshape and int(np.prod(vshape[:-1], dtype=np.int64)) == 1:
            # padded rows, one row per record: each record is still contiguous
            # (only the records are P elements apart), so the functions that
            # see them cannot tell; no compaction
            rows = F.view(d["_pbuf"], (nrec, d["_pitch"]), self._dtype)[:, :vshape[-1]]
            return rows.view((nrec,) + vshape)
        return F.view(self._data, (nrec,) + vshape, self._dtype)

    def map(self, func, axis=(0,), value_shape=None, dtype=None, with_keys=False):
        """Apply ``func`` to every record along ``axis`` (array.py:125-191).

        The array is aligned (swapped) so ``axis`` are the keys, then ``func``
        runs on every record -- a torch tensor on the GPU -- vmapped over all
        of this rank's records at once (record by record with keys when
        ``with_keys``: func((key tuple, value))).  Shape inference, checks and
        the result's shape/split follow the reference.
        """
        from bolt_amd.mi355x import functional as F
        axis = tupleize(axis)
        swapped = self._align(axis)
        dev = swapped._device
        func = F.user_fn(func)
        test_func = (lambda x: func((F.KeyTuple((0,) * len(axis)), x))) if with_keys else func
        if value_shape is None or dtype is None:
            try:
                mapped = F.to_device(test_func(F.random_like(swapped.values.shape, self._dtype, dev)), dev)
            except Exception:
                mapped = F.to_device(test_func(swapped._records_tensor()[0]), dev)
            if value_shape is None:
                value_shape = tuple(mapped.shape)
            if dtype is None:
                dtype = F.numpy_dtype(mapped.dtype)
        value_shape = tupleize(value_shape)
        dtype = np.dtype(dtype)
        shape = tuple([swapped._shape[ax] for ax in range(len(axis))]) + value_shape
        recs = swapped._records_tensor()
        if with_keys:
            import torch
            lo, _ = swapped._ctx.local_bounds(swapped._shape[0]) if swapped._shape else (0, 0)
            kshape = swapped._shape[:swapped._split]
            base = lo * int(np.prod(kshape[1:], dtype=np.int64))
            outs = [F.to_device(func((F.KeyTuple(int(k) for k in np.unravel_index(base + i, kshape)), recs[i])), dev)
                    for i in range(recs.shape[0])]
            out = torch.stack(outs) if outs else None
        else:
            out = F.apply_batched(func, recs)
        if out is not None and len(out.shape) > 1 and tuple(out.shape[1:]) != value_shape:
            raise Exception("Map operation did not produce values of uniform shape.")
        data = F.as_bytes(out.to(F.torch_dtype(dtype))) if out is not None else _empty(0, dev)
        return self._like(data, shape, swapped.split, dtype=dtype)

    def filter(self, func, axis=(0,), sort=False):
        """Keep the records along ``axis`` for which ``func`` is true (array.py:193-241).

        ``func`` runs on every record (a torch tensor, vmapped) and returns a
        boolean; the kept records are compacted with one gather kernel (and an
        all-to-all across GPUs) and re-keyed 0..count-1 in key order.
        """
        from bolt_amd.mi355x import functional as F
        from bolt_amd.mi355x.indexing import gather_units_sharded
        axis = tupleize(axis)
        swapped = self._align(axis)
        recs = swapped._records_tensor()
        func = F.user_fn(func)
        keep = F.apply_batched(lambda v: F.to_device(func(v), v.device).reshape(()).to(bool), recs)
        mask = keep.cpu().numpy().reshape(-1) if keep is not None else np.zeros(0, bool)
        ctx = swapped._ctx
        local_idx = np.nonzero(mask)[0].astype(np.int64)
        if ctx.world_size > 1:
            # every rank's mask (one byte per record, rank order) on every rank
            import torch
            per = int(np.prod(swapped.shape[1:swapped.split], dtype=np.int64))
            sizes = [(hi - lo) * per for lo, hi in ctx.bounds(swapped.shape[0])]
            mb = torch.from_numpy(mask.astype(np.uint8)).to(swapped._device)
            allm = all_gather_bytes(ctx, mb, sizes).cpu().numpy()
            glob = np.nonzero(allm)[0].astype(np.int64)
        else:
            glob = local_idx
        remaining = list(swapped.shape[len(axis):])
        count = int(glob.size)
        es = self._dtype.itemsize
        rowbytes = int(np.prod(remaining, dtype=np.int64)) * es
        nrec = int(np.prod(swapped.shape[:swapped.split], dtype=np.int64))
        if count == 0:
            return self._like(_empty(0, swapped._device), (0,), 1)
        # records are rows of the flattened key space; ragged per rank
        flat_rows_per_lead = int(np.prod(swapped.shape[1:swapped.split], dtype=np.int64))
        d = swapped.__dict__
        if "_pbuf" in d and remaining:
            # padded rows (one GPU): whole padded records move, the result keeps the pitch
            P = d["_pitch"]
            prb = rowbytes // (remaining[-1] * es) * P * es
            data = gather_units_sharded(ctx, swapped._backend, d["_pbuf"], swapped.shape[0],
                                        prb, flat_rows_per_lead, glob, count, 1)
            return self._derive_padded(data, P, tuple([count] + remaining), 1)
        data = gather_units_sharded(ctx, swapped._backend, swapped._data, swapped.shape[0],
                                    rowbytes, flat_rows_per_lead, glob, count, 1)
        return self._like(data, tuple([count] + remaining), 1)

    # ------------------------------------------------------------ indexing
    def __getitem__(self, index):
        """Index with ints, slices and lists (array.py:595-676).

        Same normalisation, bounds errors, result shape/split and element
        order as the reference (indexing.py): basic selections are one
        strided copy, list selections one gather kernel; across GPUs rows
        move with one all-to-all.  Int axes are squeezed out; an all-int
        index returns a scalar.
        """
        from bolt_amd.mi355x import indexing
        index, int_locs, kind = indexing.normalize(index, self._shape, self._split)
        es = self._dtype.itemsize
        if kind == 'basic':
            starts = [s.start for s in index]
            steps = [s.step for s in index]
            shape = tuple(int(np.ceil((s.stop - s.start) / float(s.step))) for s in index)
            d = self.__dict__
            if "_pbuf" in d:  # padded rows: selected in place, no compaction
                data = select_sharded(self._ctx, self._backend, d["_pbuf"], self._shape, starts, steps, shape, es,
                                      src_strides=_padded_strides(self._shape, d["_pitch"]))
            else:
                data = select_sharded(self._ctx, self._backend, self._data, self._shape, starts, steps, shape, es)
            result = self._like(data, shape, self._split)
        elif kind == 'advanced':
            pts, shape = indexing.advanced_points(index, self._shape, self._split)
            if len(shape) == 0:
                raise ValueError("0-d index arrays are not supported")
            out_upr = int(np.prod(shape[1:], dtype=np.int64))
            d = self.__dict__
            upr = int(np.prod(self._shape[1:], dtype=np.int64))
            if "_pbuf" in d:
                # padded rows: the elements' offsets in the padded layout
                Rl, P = self._shape[-1], d["_pitch"]
                src, pts, upr = d["_pbuf"], pts // Rl * P + pts % Rl, upr // Rl * P
            else:
                src = self._data
            data = indexing.gather_units_sharded(self._ctx, self._backend, src, self._shape[0], es, upr, pts,
                                                 shape[0], out_upr)
            result = self._like(data, shape, len(shape))
        else:
            loc, idx = indexing.mixed_take(index, self._shape, self._split)
            newshape = list(self._shape)
            newshape[loc] = len(idx)
            d = self.__dict__
            if "_pbuf" in d and self._ctx.world_size == 1:
                # padded rows (one GPU): taking along the last axis gathers
                # within the rows (a dense result); along another axis whole
                # padded rows move and the result keeps the pitch
                P, nd = d["_pitch"], self.ndim
                n_outer = int(np.prod(self._shape[:min(loc, nd - 1)], dtype=np.int64))
                if loc == nd - 1:
                    data = _empty(n_outer * len(idx) * es, d["_pbuf"].device)
                    if n_outer and len(idx):
                        self._backend.gather_rows(d["_pbuf"], 0, data, 0, n_outer, P, es, idx)
                    taken = self._like(data, tuple(newshape), self._split)
                else:
                    row = int(np.prod(self._shape[loc + 1:-1], dtype=np.int64)) * P * es
                    data = _empty(n_outer * len(idx) * row, d["_pbuf"].device)
                    if data.numel():
                        self._backend.gather_rows(d["_pbuf"], 0, data, 0, n_outer, self._shape[loc], row, idx)
                        taken = self._derive_padded(data, P, tuple(newshape), self._split)
                    else:
                        taken = self._like(data, tuple(newshape), self._split)
            else:
                data = indexing.take_sharded(self._ctx, self._backend, self._data, self._shape, es, loc, idx)
                taken = self._like(data, tuple(newshape), self._split)
            rest = list(index)
            rest[loc] = slice(0, None, None)
            full = all(isinstance(r, slice) and r.step in (None, 1) and (r.start or 0) == 0 and
                       (r.stop is None or r.stop >= d) for r, d in zip(rest, taken.shape))
            # the other axes untouched: the gathered array is the result (no second copy)
            result = taken if full and not int_locs else taken[tuple(rest)]
        if len(int_locs) == self.ndim:
            return result.toarray().reshape(())[()]
        return result.squeeze(tuple(int_locs)) if int_locs else result

    def concatenate(self, arry, axis=0):
        """Join with another array along ``axis`` (array.py:429-478).

        ndarrays (and local bolt arrays, which are ndarrays) are first built
        as mi355x arrays keyed on this array's key axes, as the reference does;
        the same shape checks and exceptions.  On the dense layout the result
        is two strided copies (rows of the two inputs interleaved at the
        concatenation axis); along the sharded leading axis across GPUs, one
        all-to-all re-slabs the rows.
        """
        from bolt_amd.mi355x.construct import ConstructMI355X
        if isinstance(arry, np.ndarray):
            arry = ConstructMI355X.array(arry, self._ctx, axis=range(0, self._split))
        elif not isinstance(arry, BoltArrayMI355X):
            raise ValueError("other must be local array or mi355x array, got %s" % type(arry))
        if not all([x == y if not i == axis else True
                    for i, (x, y) in enumerate(zip(self.shape, arry.shape))]):
            raise ValueError("all the input array dimensions except for "
                             "the concatenation axis must match exactly")
        if not self._split == arry.split:
            raise NotImplementedError("two arrays must have the same split ")
        if self.ndim != arry.ndim or not 0 <= axis < self.ndim:
            raise ValueError("arrays of %d and %d dimensions cannot be joined on axis %d"
                             % (self.ndim, arry.ndim, axis))
        if arry.dtype != self._dtype:
            raise NotImplementedError("concatenating %s with %s: cast one first (astype)"
                                      % (self._dtype, arry.dtype))
        shape = tuple([x + y if i == axis else x for i, (x, y) in enumerate(zip(self.shape, arry.shape))])
        es = self._dtype.itemsize
        if axis == 0:
            rowbytes = int(np.prod(self._shape[1:], dtype=np.int64)) * es
            data = concat_rows_sharded(self._ctx, self._data, self._shape[0], arry._data, arry.shape[0], rowbytes)
            return self._like(data, shape, self._split)
        lshape = self._local_shape
        outer = int(np.prod(lshape[:axis], dtype=np.int64))
        inner = int(np.prod(lshape[axis + 1:], dtype=np.int64))
        na, nb = self._shape[axis] * inner, arry.shape[axis] * inner
        data = _empty(outer * (na + nb) * es, self._data.device)
        if outer:
            be = self._backend
            if na:
                be.copy_strided(self._data, 0, data, 0, [outer, na], [na, 1], [na + nb, 1], es)
            if nb:
                be.copy_strided(arry._data, 0, data, na * es, [outer, nb], [nb, 1], [na + nb, 1], es)
        return self._like(data, shape, self._split)

    def squeeze(self, axis=None):
        """Drop singleton axes (array.py:879-918); the data does not move on one
        GPU, and re-slabs across GPUs when the leading axis goes away."""
        if not any(d == 1 for d in self._shape):
            return self
        if axis is None:
            drop = [i for i, d in enumerate(self._shape) if d == 1]
        elif isinstance(axis, int):
            drop = [axis]
        elif isinstance(axis, tuple):
            drop = [int(a) for a in axis]
        else:
            raise ValueError("an integer or tuple is required for the axis")
        if any(self._shape[i] > 1 for i in drop):
            raise ValueError("cannot select an axis to squeeze out which has size greater than one")
        if not drop:
            return self
        shape = tuple(d for i, d in enumerate(self._shape) if i not in drop)
        split = len([d for d in range(self._split) if d not in drop])
        d = self.__dict__
        if "_pbuf" in d and len(shape) >= 2 and (self.ndim - 1) not in drop and \
                (0 not in drop or self._ctx.world_size == 1):
            # unit axes only: a padded array's rows stay as they are
            return self._derive_padded(d["_pbuf"], d["_pitch"], shape, split)
        data = self._data
        if 0 in drop and self._ctx.world_size > 1:
            # the leading axis goes: re-slab on the new one (a 0-d result lives on rank 0)
            es = self._dtype.itemsize
            new_rows = shape[0] if shape else 1
            new_rowbytes = int(np.prod(shape[1:], dtype=np.int64)) * es if shape else es
            data = redistribute_rows(self._ctx, data, self._shape[0],
                                     int(np.prod(self._shape[1:], dtype=np.int64)) * es, new_rows, new_rowbytes)
        return self._like(data, shape, split)

    # ---------------------------------------------------------- statistics
    def _reduced(self, axis, stat):
        """Device reduction of ``axis`` -> host ndarray with the kept axes (ascending).

        Returns (result ndarray, out dtype).  Layout per plan.reduce_layout;
        if the reduced axes are not one block they are first permuted to the
        front (what _align's swap does physically, array.py:85-115).
        """
        ctx = self._ctx
        lshape = self._local_shape
        pkey = (lshape, tuple(axis), stat, self._dtype, self._shape, ctx.world_size)
        plan = _REDUCE_PLANS.get(pkey)
        if plan is None:
            axset = sorted(set(int(a) for a in axis))
            kept = [i for i in range(self.ndim) if i not in axset]
            out_shape = tuple(self._shape[i] for i in kept)
            if stat in _KEEP_DTYPE:
                out_dtype = self._dtype
            elif stat in (_lib.STAT_LAND, _lib.STAT_LOR):
                out_dtype = np.dtype(bool)
            else:
                out_dtype = stat_dtype(self._dtype, out_shape)
            perm, O, R, I = reduce_layout(lshape, axset)
            loc_out = tuple(lshape[i] for i in kept)
            plan = (axset, kept, out_shape, out_dtype, dtype_code(self._dtype), dtype_code(out_dtype),
                    perm, O, R, I, int(np.prod(lshape, dtype=np.int64)), loc_out,
                    int(np.prod(loc_out, dtype=np.int64)))
            if len(_REDUCE_PLANS) > 4096:
                _REDUCE_PLANS.clear()
            _REDUCE_PLANS[pkey] = plan
        axset, kept, out_shape, out_dtype, code, ocode, perm, O, R, I, nloc, loc_out, nout = plan
        pbuf = self.__dict__.get("_pbuf")
        if pbuf is not None and perm is None and I == 1 and R == lshape[-1] and ctx.world_size > 1 \
                and 0 not in axset:
            # last-axis statistic of a row-padded slab: every output is this
            # rank's, read in place, then gathered like the dense path's
            be = backend_for(pbuf.device)
            out = _empty(nout * out_dtype.itemsize, pbuf.device)
            if nout and nloc:
                be.reduce_rows(stat, pbuf, code, O, R, self._pitch, out, ocode)
            sizes = [int(np.prod((hi - lo,) + out_shape[1:], dtype=np.int64)) * out_dtype.itemsize
                     for lo, hi in ctx.bounds(self._shape[0])]
            return to_host(all_gather_bytes(ctx, out, sizes), out_dtype, out_shape), out_dtype
        if pbuf is not None and perm is None and I == 1 and R == lshape[-1] and nloc and ctx.world_size == 1:
            # last-axis statistic of a row-padded array: read the rows in place
            be = backend_for(pbuf.device)
            host = host_result(be, nout * out_dtype.itemsize, pbuf.device)
            if host is not None:
                be.reduce_rows(stat, pbuf, code, O, R, self._pitch, host, ocode)
                return finish_host_result(host, pbuf.device, out_dtype, out_shape), out_dtype
            out = _empty(nout * out_dtype.itemsize, pbuf.device)
            be.reduce_rows(stat, pbuf, code, O, R, self._pitch, out, ocode)
            return to_host(out, out_dtype, out_shape), out_dtype
        if pbuf is not None and perm is None and I > 1 and I % lshape[-1] == 0 and nloc and ctx.world_size == 1:
            # leading / middle axes of a row-padded array: the columns run over
            # the padded rows as if the last axis were P long; every column is
            # its own reduction, so the pad columns' (unwritten) values reach
            # only their own outputs, which are dropped
            be = backend_for(pbuf.device)
            Rl, P = lshape[-1], self._pitch
            Ip = I // Rl * P
            nb = O * Ip * out_dtype.itemsize
            host = host_result(be, nb, pbuf.device)
            if host is not None:
                be.reduce(stat, pbuf, code, O, R, Ip, host, ocode)
                full = finish_host_result(host, pbuf.device, out_dtype, (O, I // Rl, P))
            else:
                out = _empty(nb, pbuf.device)
                be.reduce(stat, pbuf, code, O, R, Ip, out, ocode)
                full = to_host(out, out_dtype, (O, I // Rl, P))
            return np.ascontiguousarray(full[:, :, :Rl]).reshape(out_shape), out_dtype
        if pbuf is not None and perm is None and O == 1 and I == 1 and R == nloc and nloc \
                and ctx.world_size == 1 and len(lshape) >= 2 and stat in _MOMENTS \
                and self._dtype.kind == "f" and self._dtype.itemsize >= 4:
            return self._padded_all_moments(pbuf, stat, code, out_dtype, out_shape), out_dtype
        be = self._backend
        dev = self._device
        es = self._dtype.itemsize
        if perm is not None:
            # the reduced axes first (_align's swap): a padded array is read in place
            tmp = _empty(nloc * es, dev)
            if pbuf is not None:
                pstr = _padded_strides(lshape, self._pitch)
                pshape = [lshape[p] for p in perm]
                be.copy_strided(pbuf, 0, tmp, 0, pshape, [pstr[p] for p in perm],
                                _padded_strides(pshape, pshape[-1]), es)
            elif nloc:
                be.permute(self._data, lshape, perm, es, tmp)
            src = tmp
        else:
            src = self._data

        if ctx.world_size == 1 or 0 not in axset:
            # every output lives on this rank (or this rank's slab of them)
            host = host_result(be, nout * out_dtype.itemsize, dev) if ctx.world_size == 1 and nloc else None
            if host is not None:
                # the kernel stores the result into page-locked host memory
                be.reduce(stat, src, code, O, R, I, host, ocode)
                return finish_host_result(host, dev, out_dtype, out_shape), out_dtype
            out = _empty(nout * out_dtype.itemsize, dev)
            if nout and nloc:
                be.reduce(stat, src, code, O, R, I, out, ocode)
            if ctx.world_size > 1:
                sizes = []
                for lo, hi in ctx.bounds(self._shape[0]):
                    sizes.append(int(np.prod((hi - lo,) + out_shape[1:], dtype=np.int64)) * out_dtype.itemsize)
                out = all_gather_bytes(ctx, out, sizes)
            return to_host(out, out_dtype, out_shape), out_dtype

        # the sharded axis is reduced: per-rank states, gathered and combined
        # in rank order (statcounter.py:67-99, deterministic here)
        nout = int(np.prod(out_shape, dtype=np.int64))
        if nout == 0:  # e.g. mean(axis=0) of (4, 0, 3): nothing to merge
            return np.empty(out_shape, out_dtype), out_dtype
        if ctx.world_size > _lib.MAX_COMBINE_PARTS:
            raise NotImplementedError("reductions over the sharded axis merge at most %d ranks (got %d)"
                                      % (_lib.MAX_COMBINE_PARTS, ctx.world_size))
        sbytes = be.state_bytes(stat, code, nout)
        state = _empty(sbytes, dev)
        count = int(np.prod([lshape[i] for i in axset], dtype=np.int64))
        if count:
            be.reduce_state(stat, src, code, O, R, I, state)
        else:
            state.zero_()
        counts = []
        for lo, hi in ctx.bounds(self._shape[0]):
            c = (hi - lo) * int(np.prod([self._shape[i] for i in axset if i != 0], dtype=np.int64))
            counts.append(c)
        states = all_gather_bytes(ctx, state, [sbytes] * ctx.world_size)
        out = _empty(nout * out_dtype.itemsize, dev)
        be.reduce_combine(stat, code, states, counts, nout, out, ocode)
        return to_host(out, out_dtype, out_shape), out_dtype

    def _padded_all_moments(self, pbuf, stat, code, out_dtype, out_shape):
        """mean / var / std over every axis of a row-padded float array, read in
        place: the padded rows are one (rows, pitch) matrix whose columns get a
        float64 mean (and M2 for var / std) state each over all rows
        (bm_reduce_state, the pad columns' states dropped); the row-length states, all of the same count,
        merge on the host -- the StatCounter merge of statcounter.py:67-99 for
        equal counts: mean = mean of the column means, M2 = sum of the column
        M2 + rows * sum of squared deviations of the column means.  No dense
        copy of the array is made; the summation order differs from the dense
        layout's (results within 1e-12 relative in float64, rounded once)."""
        be = backend_for(pbuf.device)
        Rl, P = self._local_shape[-1], self._pitch
        nrows = int(np.prod(self._local_shape[:-1], dtype=np.int64))
        state = _empty(be.state_bytes(stat, code, P), pbuf.device)
        be.reduce_state(stat, pbuf, code, 1, nrows, P, state)
        planes = to_host(state, np.float64, (-1, P))   # mean [, M2] (bm_reduce_state)
        means = planes[0, :Rl]
        mean = means.mean()
        if stat == _lib.STAT_MEAN:
            v = mean
        else:
            v = (planes[1, :Rl].sum() + nrows * np.square(means - mean).sum()) / (nrows * Rl)
            if stat == _lib.STAT_STD:
                v = np.sqrt(v)
        return np.asarray(v, dtype=np.float64).astype(out_dtype).reshape(out_shape)

    def _stat(self, axis=None, func=None, name=None, keepdims=False):
        """Statistic over ``axis`` (array.py:284-334); results are host arrays / scalars."""
        if name and not func:
            try:  # axes already validated for this shape and split, keyed by the argument as given
                ak = (self._shape, self._split, axis)
                hit = _STAT_AXES.get(ak)
            except TypeError:  # unhashable axis (a list)
                ak = hit = None
            if hit is None:
                ax = tupleize(list(range(len(self.shape))) if axis is None else axis)
                inshape(self.shape, ax)
                hit = (ax, self._nrecords(ax), self._aligned_vshape(ax))
                if ak is not None:
                    if len(_STAT_AXES) > 4096:
                        _STAT_AXES.clear()
                    _STAT_AXES[ak] = hit
            axis, nrec, vs = hit
            if nrec == 0:
                # no records after _align: the merged StatCounter is the empty one
                # (statcounter.py:28-41, :109-130): mean 0.0, variance / stdev nan
                arr = 0.0 if name == 'mean' else float('nan')
            else:
                arr, _ = self._reduced(axis, _STAT_CODES[name])
                if vs is not None:
                    arr = arr.reshape(vs)
                if arr.ndim == 0:
                    arr = arr[()]
            if keepdims:
                for i in axis:
                    arr = np.expand_dims(arr, axis=i)
            return BoltArrayLocal(arr).toscalar()

        if axis is None:
            axis = list(range(len(self.shape)))
        axis = tupleize(axis)
        if func and not name:
            return self.reduce(func, axis, keepdims)

        raise ValueError('Must specify either a function or a statistic name.')

    def reduce(self, func, axis=(0,), keepdims=False):
        """Reduce with ``func`` over ``axis`` (array.py:243-282).

        The reference treeReduces ``func`` over the aligned records.  numpy
        ufuncs (add, multiply, maximum, minimum, fmax, fmin, logical_and /
        or, bitwise_and / or / xor and their ``operator`` spellings) run as
        one bm_reduce mode on the GPU, with numpy's result dtype for
        ``func(record, record)``; any other binary function receives device
        tensors and is applied as a pairwise tree in record order,
        ((r0 f r1) f (r2 f r3)) ..., vmapped over the pairs of each level.
        A single record is returned as is, as treeReduce returns it.
        """
        axis = tupleize(axis)
        inshape(self.shape, axis)
        nrec = self._nrecords(axis)
        if nrec == 0:
            raise ValueError("Can not reduce() empty RDD")  # treeReduce of no records (array.py:269)
        stat = _UFUNC_STATS.get(func) if _hashable(func) else None
        vs = self._aligned_vshape(axis)
        if nrec == 1:
            # treeReduce of one record returns it untouched (no func call)
            kept = [d for i, d in enumerate(self._shape) if i not in set(int(a) for a in axis)]
            arr = self.toarray().reshape(kept if vs is None else vs)
        elif stat is not None and self._reduce_dtype_ok(func, stat):
            arr, _ = self._reduced(axis, stat)
        else:
            from bolt_amd.mi355x.functional import user_fn
            arr = self._tree_reduce(user_fn(func), axis, vs)
        if vs is not None:
            arr = arr.reshape(vs)
        if arr.ndim == 0:
            arr = arr[()]
        if keepdims:
            for i in axis:
                arr = np.expand_dims(arr, axis=i)
        if not isinstance(arr, np.ndarray):
            return arr
        elif arr.shape == (1,):
            return arr[0]
        return BoltArrayLocal(arr)

    def _reduce_dtype_ok(self, func, stat):
        """numpy's own rule for func(record, record) (raises numpy's TypeError for
        bitwise ufuncs on floats); True if the kernel mode produces that dtype."""
        probe = np.asarray(func(np.zeros(1, self._dtype), np.zeros(1, self._dtype)))
        want = np.dtype(bool) if stat in (_lib.STAT_LAND, _lib.STAT_LOR) else self._dtype
        return probe.dtype == want

    def _tree_reduce(self, func, axis, vshape=None):
        """Pairwise tree of a user function over the aligned records, on the
        device; ``vshape``: the records' shape when the reference's _align
        squeezes a unit axis (see _aligned_vshape)."""
        import torch
        from bolt_amd.mi355x.functional import view, apply_pairs, numpy_dtype
        ctx = self._ctx
        axset = sorted(set(int(a) for a in axis))
        kept = [i for i in range(self.ndim) if i not in axset]
        gshape = self._shape
        lshape = self._local_shape
        src = self._data
        if ctx.world_size > 1 and 0 not in axset:
            # a rank's slab of the sharded axis is a slab of every record: a
            # function that is not elementwise must see whole records, as the
            # reference's treeReduce after _align does (array.py:268-269).  Bring
            # the reduced axes to the front across GPUs (one exchange), so each
            # rank holds whole records, and reduce the sharded axis below.
            gperm = axset + kept
            src = permute_sharded(ctx, self._backend, src, gshape, gperm, self._dtype.itemsize)
            gshape = tuple(gshape[p] for p in gperm)
            lo, hi = ctx.local_bounds(gshape[0])
            lshape = (hi - lo,) + gshape[1:]
            axset = list(range(len(axset)))
            kept = list(range(len(axset), len(gshape)))
        perm, O, R, I = reduce_layout(lshape, axset)
        if perm is not None:
            tmp = _empty(src.numel(), src.device)
            if src.numel():
                self._backend.permute(src, lshape, perm, self._dtype.itemsize, tmp)
            src = tmp
        rec_shape = tuple(lshape[i] for i in kept) if vshape is None else tuple(vshape)
        recs = view(src, (O, R, I), self._dtype).permute(1, 0, 2).reshape((R,) + rec_shape)
        if R:
            part = _tree(func, recs)
        else:
            # a rank with no records still needs the result's dtype and shape
            z = torch.zeros((1,) + rec_shape, dtype=recs.dtype, device=recs.device)
            part = apply_pairs(func, z, z)[0]
        out_dtype = numpy_dtype(part.dtype)
        if ctx.world_size == 1:
            return part.cpu().numpy().astype(out_dtype, copy=False)
        from bolt_amd.mi355x.functional import as_bytes
        # the sharded axis is reduced: rank partials, then the same tree over
        # the ranks that hold records, in rank order
        pbytes = as_bytes(part)
        allp = all_gather_bytes(ctx, pbytes, [pbytes.numel()] * ctx.world_size)
        per = view(allp, (ctx.world_size,) + tuple(part.shape), out_dtype)
        has = [r for r, (lo, hi) in enumerate(ctx.bounds(gshape[0])) if hi > lo]
        res = _tree(func, per[has])
        return res.cpu().numpy().astype(numpy_dtype(res.dtype), copy=False)

    def _aligned_vshape(self, axis):
        """The record shape after the reference's _align(axis) (array.py:85-115)
        when its swap squeezes a unit axis (plan.swap_shape), else None: the
        kept axes' extents in ascending order."""
        try:
            return _aligned_vshape_of(self._shape, self._split, tuple(int(a) for a in axis))
        except TypeError:
            return _aligned_vshape_of.__wrapped__(self._shape, self._split, tuple(axis))

    def _nrecords(self, axis):
        """Records the reduction sees after _align: the product of the reduced extents."""
        n = 1
        for a in axis:
            n *= int(self._shape[int(a)])
        return n

    def mean(self, axis=None, keepdims=False):
        """Mean over ``axis`` (array.py:336-349)."""
        return self._stat(axis, name='mean', keepdims=keepdims)

    def var(self, axis=None, keepdims=False):
        """Population variance over ``axis`` (array.py:351-364)."""
        return self._stat(axis, name='variance', keepdims=keepdims)

    def std(self, axis=None, keepdims=False):
        """Population standard deviation over ``axis`` (array.py:366-379)."""
        return self._stat(axis, name='stdev', keepdims=keepdims)

    def sum(self, axis=None, keepdims=False):
        """Sum over ``axis`` in the input dtype (array.py:381-395; integer sums wrap)."""
        import operator
        return self._stat(axis, func=operator.add, keepdims=keepdims)

    def max(self, axis=None, keepdims=False):
        """Maximum over ``axis`` (array.py:397-411): numpy.maximum, NaNs propagate."""
        return self._stat(axis, func=np.maximum, keepdims=keepdims)

    def min(self, axis=None, keepdims=False):
        """Minimum over ``axis`` (array.py:413-427): numpy.minimum, NaNs propagate."""
        return self._stat(axis, func=np.minimum, keepdims=keepdims)

    # -------------------------------------------------------------- egress
    def toarray(self):
        """The whole array on the host (array.py:1006-1014).  Across GPUs the
        slabs are gathered window by window (dist.gather_to_host): device
        memory per rank stays at its slab plus one window."""
        ctx = self._ctx
        d = self.__dict__
        if "_pbuf" in d and ctx.world_size == 1:
            return self._padded_to_host()
        if ctx.world_size == 1:
            return to_host(self._data, self._dtype, self._shape)
        rowbytes = int(np.prod(self._shape[1:], dtype=np.int64)) * self._dtype.itemsize
        rows = self._shape[0] if self._shape else 1  # a 0-d array lives on rank 0
        sizes = [(hi - lo) * rowbytes for lo, hi in ctx.bounds(rows)]
        if "_pbuf" in d:
            # padded rows: each egress window compacted on the way
            es = self._dtype.itemsize
            spec = (self._shape[-1] * es, d["_pitch"] * es, self._backend)
            return gather_to_host(ctx, d["_pbuf"], sizes, rows=spec).view(self._dtype).reshape(self._shape)
        return gather_to_host(ctx, self._data, sizes).view(self._dtype).reshape(self._shape)

    def _padded_to_host(self):
        """toarray of a row-padded array (one GPU): the rows are compacted
        window by window into two device windows of at most transfer.CHUNK
        bytes, each DMA'd to page-locked memory while the next is compacted
        -- no dense copy of the whole array on the device (array.py:1006-1014)."""
        from bolt_amd.mi355x import transfer
        d = self.__dict__
        pbuf, P = d["_pbuf"], d["_pitch"]
        es = self._dtype.itemsize
        R = self._shape[-1]
        rows = int(np.prod(self._local_shape[:-1], dtype=np.int64))
        rb = R * es
        out = np.empty(rows * rb, dtype=np.uint8)
        if rows == 0 or rb == 0:
            return out.view(self._dtype).reshape(self._shape)
        wrows = max(1, min(rows, transfer.CHUNK // rb)) if pbuf.device.type == "cuda" else rows
        be = backend_for(pbuf.device)
        wins = [_empty(wrows * rb, pbuf.device) for _ in range(2 if rows > wrows else 1)]

        def produce(lo, hi, k):
            r0, r1 = lo // rb, hi // rb
            be.copy_strided(pbuf, r0 * P * es, wins[k], 0, [r1 - r0, R], [P, 1], [R, 1], es)
            return wins[k][:(r1 - r0) * rb]
        transfer.copy_to_host(pbuf, out, produce=produce, chunk=wrows * rb)
        return out.view(self._dtype).reshape(self._shape)

    def tolocal(self):
        """As a local bolt array (array.py:999-1004)."""
        return BoltArrayLocal(self.toarray())

    def __array__(self, dtype=None, copy=None):
        a = self.toarray()
        return a if dtype is None else a.astype(dtype)

    def records(self):
        """(key tuple, value ndarray) pairs in key order -- the content of
        ``tordd().sortByKey().collect()`` of the Spark path."""
        x = self.toarray()
        kshape = self._shape[:self._split]
        flat = x.reshape((int(np.prod(kshape, dtype=np.int64)),) + self._shape[self._split:])
        for i, key in enumerate(np.ndindex(*kshape)):
            yield tuple(int(k) for k in key), flat[i]

    def display(self):
        """Print the first 10 records as (key, value) pairs, as the Spark
        mode's ``rdd.take(10)`` does (array.py:1022-1027).  Only the
        leading-axis rows that hold them leave the GPU; every rank takes part
        in the gather, rank 0 prints (the driver's console in Spark)."""
        kshape = self._shape[:self._split]
        nrec = int(np.prod(kshape, dtype=np.int64))
        n = min(10, nrec)
        if n == 0:
            return
        per_row = int(np.prod(kshape[1:], dtype=np.int64))
        rows = -(-n // per_row)
        part = self if rows >= self._shape[0] else self[0:rows]
        for i, rec in enumerate(part.records()):
            if i >= n:
                break
            if self._ctx.rank == 0:
                print(rec)

    def tordd(self):
        from bolt_amd.mi355x.records import RecordView
        return RecordView(list(self.records()), self._npartitions or self._ctx.world_size,
                          cached=getattr(self, "_cached", False))

    @property
    def _rdd(self):
        """A host view of the records (RecordView), for code written against
        the Spark mode's ``_rdd`` (collect, map, sortByKey, ...)."""
        return self.tordd()

    def __repr__(self):
        s = "BoltArray\n"
        s += "mode: %s\n" % self._mode
        s += "shape: %s\n" % str(self.shape)
        return s
