"""ChunkedArrayMI355X: bolt's ChunkedArray (bolt/spark/chunk.py) on MI355X.

A chunked array's records are ``(key + chunk_id, chunk_value)`` pairs
(chunk.py:87-144).  Here every record's chunks live packed back to back in
HBM, in chunk-id order, each chunk a dense box of its (padded) extent -- the
layout described by plan.ChunkGeometry.  Building it (pack) and undoing it
(unpack, padding removed) are strided-copy kernels, one launch per run of
equally shaped chunks, or for records of at most 64 KiB one record-map
gather (pack) / record scatter (unpack); when the packed layout is the dense
one both are relabellings.  Records never leave their GPU.

keys_to_values / values_to_keys change which axes are keys and re-chunk the
moved axes; their result is by construction the chunking of the permuted
array with the new plan/padding (chunk.py:202-347).  They go packed ->
packed in one pass where the leading key stays (strided copies, a record
scatter for trailing keys, a masked record gather for values_to_keys), and
otherwise unpack -> permute (RCCL all-to-all if the sharded axis moves) ->
pack.
"""
import numpy as np

from bolt_amd.mi355x.context import local_shape
from bolt_amd.mi355x.dist import permute_sharded, _empty
from bolt_amd.mi355x.plan import (ChunkGeometry, getplan, check_plan, getnumber, getslices, getmask,
                                  removepad_slices, k2v_copies, v2k_copies, copies_to_map, copies_to_scatter)


RECORD_MAP_MAX_BYTES = 65536  # a source record staged whole in LDS (bm_record_gather)


# Which of the equivalent chunk paths run.  Every path gives the same bytes;
# tests/test_chunk_paths.py flips these to compare them with each other:
#   fused_rechunk  keys_to_values / values_to_keys packed -> packed in one pass
#                  (False: unpack -> permute -> pack)
#   scatter        "on": unchunk / keys_to_values / values_to_keys of small
#                  records as one record scatter where its writes are whole
#                  runs; "off": strided copies / record gather; "force": the
#                  scatter also where its writes would be piecewise
#   runs           keys_to_values whose records are a few long runs as
#                  bm_record_runs (False: the map scatter)
#   record_map     small records packed by one record-map gather (False: one
#                  strided copy per chunk run)
PATHS = {"fused_rechunk": True, "scatter": "on", "runs": True, "record_map": True}


def _fused_rechunk():
    return bool(PATHS["fused_rechunk"])


def _use_scatter():
    """unchunk / keys_to_values / values_to_keys of small records as one
    record scatter (bm_record_scatter)."""
    return PATHS["scatter"] != "off"


_SCATTER_PLANS = {}


def _scatter_plan(key, build, src_rec, gstride, es):
    """(map_a, map_b, vec) for a record scatter, or None when the move is not
    a record scatter or would write lines piecewise (plan.scatter_runs_ok);
    built once per key (geometry, move, element size)."""
    from bolt_amd.mi355x.plan import scatter_vec, scatter_runs_ok
    key = key + (PATHS["scatter"],)
    if key in _SCATTER_PLANS:
        return _SCATTER_PLANS[key]
    maps = build()
    plan = None
    force = PATHS["scatter"] == "force"
    if maps is not None and (force or scatter_runs_ok(maps[0], maps[1], es)):
        map_a, map_b = maps
        plan = (map_a, map_b, scatter_vec(map_a, map_b, src_rec, gstride, es))
    if len(_SCATTER_PLANS) > 256:
        _SCATTER_PLANS.clear()
    _SCATTER_PLANS[key] = plan
    return plan


def _use_runs():
    """keys_to_values whose records are a few long runs as bm_record_runs."""
    return bool(PATHS["runs"])


_RUNS_PLANS = {}


def _runs_plan(key, plan, src_rec, gstride, es):
    """(runs, vec_bytes) of a scatter plan (plan.scatter_to_runs), cached per key."""
    from bolt_amd.mi355x.plan import scatter_to_runs
    if key not in _RUNS_PLANS:
        if len(_RUNS_PLANS) > 256:
            _RUNS_PLANS.clear()
        _RUNS_PLANS[key] = scatter_to_runs(plan[0], plan[1], src_rec, gstride, es)
    return _RUNS_PLANS[key]


def _use_record_map(src_rec, es):
    """Small records: one record-map gather instead of a strided copy per chunk run."""
    if not PATHS["record_map"]:
        return False
    return es in (1, 2, 4, 8) and 0 < src_rec * es <= RECORD_MAP_MAX_BYTES


class ChunkedArrayMI355X(object):

    _metadata = ['_shape', '_split', '_dtype', '_plan', '_padding', '_ordered']

    def __init__(self, packed, shape=None, split=None, dtype=None, plan=None, padding=None,
                 ordered=True, context=None):
        self._packed = packed
        self._shape = tuple(int(s) for s in shape)
        self._split = int(split)
        self._dtype = np.dtype(dtype)
        self._plan = np.asarray(plan, dtype=int)
        self._padding = np.asarray(padding, dtype=int)
        self._ordered = ordered
        self._ctx = context
        self._geom = ChunkGeometry(self.vshape, self._plan, self._padding)
        # values_to_keys down to no value axes appends a (1,) value axis whose
        # records carry no chunk id (chunk.py:335-345); chunk() of an all-key
        # array appends one with chunk id 0 (chunk.py:113-118)
        self._bare_singleton = False
        # keys_to_values of an array whose values are (1,) squeezes each new
        # record (chunk.py:284-287: squeeze drops EVERY unit axis, so a moved
        # key of extent 1 leaves 0-d records); records() shows them that way
        self._squeezed_records = False

    # ---------------------------------------------------------- properties
    @property
    def dtype(self):
        return self._dtype

    @property
    def shape(self):
        return self._shape

    @property
    def split(self):
        return self._split

    @property
    def plan(self):
        return self._plan

    @property
    def padding(self):
        return self._padding

    @property
    def uniform(self):
        """Every value axis divides evenly by its chunk size (chunk.py:54-56)."""
        return all([np.mod(x, y) == 0 for x, y in zip(self.vshape, self.plan)])

    @property
    def padded(self):
        return not all([p == 0 for p in self.padding])

    @property
    def kshape(self):
        return np.asarray(self._shape[:self._split])

    @property
    def vshape(self):
        return np.asarray(self._shape[self._split:])

    def kmask(self, axes):
        return self.getmask(axes, len(self.kshape))

    def vmask(self, axes):
        return self.getmask(axes, len(self.vshape))

    @property
    def _constructor(self):
        return ChunkedArrayMI355X

    # host helpers with the reference's names (chunk.py:434-636)
    def getplan(self, size="150", axes=None, padding=None):
        return getplan(self.vshape, self._dtype, size, axes, padding)

    @staticmethod
    def removepad(idx, value, number, padding, axes=None):
        return value[removepad_slices(idx, number, padding, axes)]

    @staticmethod
    def getnumber(plan, shape):
        return getnumber(plan, shape)

    @staticmethod
    def getslices(plan, padding, shape):
        return getslices(plan, padding, shape)

    @staticmethod
    def getmask(inds, n):
        return getmask(inds, n)

    # --------------------------------------------------------- pack/unpack
    @staticmethod
    def _pack(ctx, backend, dense, shape, split, dtype, plan, padding, src_stride=None):
        """Packed chunk buffer for this rank's records of a dense sharded array
        (``src_stride``: elements between records when they are not back to
        back -- the single-row records of a row-padded array)."""
        es = np.dtype(dtype).itemsize
        lshape = local_shape(ctx, shape)
        nrec = int(np.prod(lshape[:split], dtype=np.int64))
        vshape = shape[split:]
        geom = ChunkGeometry(vshape, plan, padding)
        rec = int(np.prod(vshape, dtype=np.int64))
        stride = rec if src_stride is None else int(src_stride)
        if geom.is_identity():
            # the packed layout is the dense one: the chunked array shares the
            # records' bytes (arrays are never written in place)
            if stride == rec:
                return dense[:nrec * rec * es]
            packed = _empty(nrec * rec * es, dense.device)
            if nrec:
                backend.copy_strided(dense, 0, packed, 0, [nrec, rec], [stride, 1], [rec, 1], es)
            return packed
        packed = _empty(nrec * geom.size * es, dense.device)
        if nrec and _use_record_map(stride, es):
            backend.record_gather(dense, 0, packed, 0, nrec, stride, geom.size,
                                  geom.record_map(unpack=False), ("pack",) + geom.key(), es)
        elif nrec:
            for (cshape, dstr, pstr, doff, poff) in geom.copies(unpack=False):
                backend.copy_strided(dense, doff * es, packed, poff * es, [nrec] + cshape,
                                     [stride] + dstr, [geom.size] + pstr, es)
        return packed

    def _unpack(self):
        """Dense bytes of this rank's records (padding removed, chunk.py:146-200)."""
        es = self._dtype.itemsize
        lshape = local_shape(self._ctx, self._shape)
        nrec = int(np.prod(lshape[:self._split], dtype=np.int64))
        rec = int(np.prod(self.vshape, dtype=np.int64))
        if self._geom.is_identity():
            return self._packed[:nrec * rec * es]  # same bytes, dense order
        dense = _empty(nrec * rec * es, self._packed.device)
        g = self._geom
        if nrec and _use_scatter() and _use_record_map(g.size, es):
            # one stream over the packed records, cores scattered to their
            # dense places, halos dropped
            plan = _scatter_plan(("unpack", es) + g.key(), lambda: copies_to_scatter(
                [(sh, ps, ds, po, do) for sh, ds, ps, do, po in g.copies(unpack=True)], g.size),
                g.size, rec, es)
            if plan is not None:
                self._backend.record_scatter(self._packed, 0, dense, 0, nrec, g.size, 1, rec, plan,
                                             ("scatter", "unpack", es) + g.key(), es)
                return dense
        if nrec:
            be = self._backend
            for (cshape, dstr, pstr, doff, poff) in self._geom.copies(unpack=True):
                be.copy_strided(self._packed, poff * es, dense, doff * es, [nrec] + cshape,
                                [self._geom.size] + pstr, [rec] + dstr, es)
        return dense

    @property
    def _backend(self):
        from bolt_amd.mi355x._ops import backend_for
        return backend_for(self._packed.device)

    @classmethod
    def _from_array(cls, barray, size="150", axis=None, padding=None):
        """ChunkedArray._chunk (chunk.py:87-144) on a BoltArrayMI355X."""
        shape, split, dtype = barray.shape, barray.split, barray.dtype
        if split == len(shape) and padding is None:
            # all keys: every record gets a trailing value axis of length 1
            shape = shape + (1,)
            plan, pad = np.array([1]), np.array([0])
        else:
            vshape = shape[split:]
            plan, pad = getplan(vshape, dtype, size, axis, padding)
            check_plan(plan, pad, vshape)
        d = barray.__dict__
        if "_pbuf" in d and split == len(shape) - 1:
            # a row-padded array whose records are single rows: packed straight
            # from the padded rows (records P elements apart)
            packed = cls._pack(barray._ctx, barray._backend, d["_pbuf"], shape, split, dtype, plan, pad,
                               src_stride=d["_pitch"])
        else:
            packed = cls._pack(barray._ctx, barray._backend, barray._data, shape, split, dtype, plan, pad)
        return cls(packed, shape=shape, split=split, dtype=dtype, plan=plan, padding=pad,
                   ordered=barray._ordered, context=barray._ctx)

    def _rechunk(self, dense, perm, shape_before, newshape, newsplit, newplan, newpadding):
        """Permute this rank's dense records (exchange if the sharded axis moves) and pack."""
        es = self._dtype.itemsize
        if list(perm) != list(range(len(perm))):
            dense = permute_sharded(self._ctx, self._backend, dense, shape_before, perm, es)
        packed = self._pack(self._ctx, self._backend, dense, newshape, newsplit, self._dtype,
                            newplan, newpadding)
        return self._constructor(packed, shape=newshape, split=newsplit, dtype=self._dtype,
                                 plan=newplan, padding=newpadding, ordered=True, context=self._ctx)

    def _repack(self, copies, rmap, newshape, newsplit, newplan, newpadding, new):
        """New packing straight from this packing: strided copies or one record-map gather."""
        es = self._dtype.itemsize
        lnew = local_shape(self._ctx, newshape)
        nrec = int(np.prod(lnew[:newsplit], dtype=np.int64))
        packed = _empty(nrec * new.size * es, self._packed.device)
        be = self._backend
        if nrec and rmap is not None:
            nold = int(np.prod(local_shape(self._ctx, self._shape)[:self._split], dtype=np.int64))
            m, key = rmap
            be.record_gather(self._packed, 0, packed, 0, nold, self._geom.size, m.size, m, key, es)
        elif nrec:
            for shape, ss, ds, so, do in copies:
                be.copy_strided(self._packed, so * es, packed, do * es, shape, ss, ds, es)
        return self._constructor(packed, shape=newshape, split=newsplit, dtype=self._dtype,
                                 plan=newplan, padding=newpadding, ordered=True, context=self._ctx)

    # ------------------------------------------------------------- the API
    def unchunk(self):
        """Back to a BoltArrayMI355X (chunk.py:146-200); a trailing (1,) value axis is squeezed."""
        from bolt_amd.mi355x.array import BoltArrayMI355X
        dense = self._unpack()
        if np.array_equal(self.vshape, [1]):
            newshape = self.shape[:-1]
        else:
            newshape = self.shape
        return BoltArrayMI355X(dense, shape=newshape, split=self._split, dtype=self._dtype,
                               context=self._ctx)

    def keys_to_values(self, axes, size=None):
        """Move key axes to the front of the values, chunked by ``size`` (chunk.py:202-289)."""
        if len(axes) == 0:
            return self
        kmask = self.kmask(axes)
        if size is None:
            size = self.kshape[kmask]
        newplan = np.r_[size, self.plan].astype(int)
        newsplit = self._split - len(axes)
        newshape = tuple(np.r_[self.kshape[~kmask], self.kshape[kmask], self.vshape].astype(int).tolist())
        newpadding = np.r_[np.zeros(len(axes), dtype=int), self.padding].astype(int)
        ks = np.arange(self._split)
        perm = list(ks[~kmask]) + list(ks[kmask]) + list(range(self._split, len(self._shape)))
        squeeze = np.array_equal(self.vshape, [1])
        if _fused_rechunk() and not squeeze and (self._ctx.world_size == 1 or not kmask[0]):
            # packed -> packed in one pass: no exchange, no dense intermediate
            new = ChunkGeometry(newshape[newsplit:], newplan, newpadding)
            lk = [int(k) for k in local_shape(self._ctx, self._shape)[:self._split]]
            nmov = int(kmask.sum())
            es = self._dtype.itemsize
            kfull = np.array_equal(np.asarray(size).reshape(-1), self.kshape[kmask])
            if (_use_scatter() and kfull and kmask[self._split - nmov:].all() and
                    _use_record_map(self._geom.size, es) and (self._ctx.world_size == 1 or nmov < self._split)):
                # the moved keys are the trailing ones, unchunked: every run of
                # K = their extent old records becomes one new record, old
                # chunk boxes stacked -- one record scatter
                K = int(np.prod(self.kshape[kmask], dtype=np.int64))
                ones = [1] * (self._split - nmov) + [int(k) for k in self.kshape[kmask]]
                g = self._geom
                plan = _scatter_plan(("k2v", es, K) + g.key() + new.key(), lambda: copies_to_scatter(
                    k2v_copies(g, new, ones, kmask), K * g.size, group=K, src_rec=g.size), g.size, new.size, es)
                if plan is not None:
                    nold = int(np.prod(lk, dtype=np.int64))
                    packed = _empty(nold // K * new.size * es, self._packed.device)
                    key = ("k2v", es, K) + g.key() + new.key()
                    runs = _runs_plan(key, plan, g.size, new.size, es) if _use_runs() else None
                    if runs is not None:
                        # every old record is a few chunk boxes: one wave per box
                        self._backend.record_runs(self._packed, 0, packed, 0, nold, g.size, K, new.size, runs,
                                                  ("runs",) + key, es)
                    else:
                        self._backend.record_scatter(self._packed, 0, packed, 0, nold, g.size, K, new.size, plan,
                                                     ("scatter",) + key, es)
                    return self._constructor(packed, shape=newshape, split=newsplit, dtype=self._dtype,
                                             plan=newplan, padding=newpadding, ordered=True, context=self._ctx)
            copies = k2v_copies(self._geom, new, lk, kmask)
            return self._repack(copies, None, newshape, newsplit, newplan, newpadding, new)
        dense = self._unpack()
        if squeeze:
            # the singleton value axis of an all-keys chunking is squeezed
            # (chunk.py:284-287; padding and stale chunk id trimmed as numpy<1.13 did)
            newshape = newshape[:-1]
            newplan = newplan[:-1]
            newpadding = newpadding[:len(newplan)]
            res = self._rechunk(dense, perm[:-1], self._shape[:-1], newshape, newsplit,
                                newplan, newpadding)
            res._squeezed_records = True
            return res
        return self._rechunk(dense, perm, self._shape, newshape, newsplit, newplan, newpadding)

    def values_to_keys(self, axes):
        """Move value axes to the end of the keys (chunk.py:291-347)."""
        vmask = self.vmask(axes)
        newplan = self.plan[~vmask]
        newsplit = self._split + len(axes)
        newshape = tuple(np.r_[self.kshape, self.vshape[vmask], self.vshape[~vmask]].astype(int).tolist())
        newpadding = self.padding[~vmask]
        vs = np.arange(len(self.vshape))
        perm = (list(range(self._split)) + [self._split + v for v in vs[vmask]] +
                [self._split + v for v in vs[~vmask]])
        if _fused_rechunk() and len(newshape) > newsplit:
            # the leading key never moves: always local, packed -> packed in one pass
            new = ChunkGeometry(newshape[newsplit:], newplan, newpadding)
            lk = [int(k) for k in local_shape(self._ctx, self._shape)[:self._split]]
            m = int(np.prod(self.vshape[vmask], dtype=np.int64))
            es = self._dtype.itemsize
            if _use_scatter() and _use_record_map(self._geom.size, es) and m * new.size < 2 ** 31:
                # every old record yields m consecutive new records: one record
                # scatter, the old packed record read front to back
                g = self._geom
                plan = _scatter_plan(("v2k", es, vmask.tobytes()) + g.key() + new.key(), lambda: copies_to_scatter(
                    v2k_copies(g, new, [], vmask), g.size), g.size, m * new.size, es)
                if plan is not None:
                    nold = int(np.prod(lk, dtype=np.int64))
                    packed = _empty(nold * m * new.size * es, self._packed.device)
                    self._backend.record_scatter(self._packed, 0, packed, 0, nold, g.size, 1, m * new.size, plan,
                                                 ("scatter", "v2k", es, vmask.tobytes()) + g.key() + new.key(), es)
                    return self._constructor(packed, shape=newshape, split=newsplit, dtype=self._dtype,
                                             plan=newplan, padding=newpadding, ordered=True, context=self._ctx)
            if _use_record_map(self._geom.size, self._dtype.itemsize) and m * new.size < 2 ** 31:
                # every old record yields m consecutive new records: one record-map
                # gather with the old packed record staged in LDS
                per_rec = v2k_copies(self._geom, new, [], vmask)
                rmap = (copies_to_map(per_rec, m * new.size), ("v2k", vmask.tobytes()) +
                        self._geom.key() + new.key())
                return self._repack(None, rmap, newshape, newsplit, newplan, newpadding, new)
            copies = v2k_copies(self._geom, new, lk, vmask)
            return self._repack(copies, None, newshape, newsplit, newplan, newpadding, new)
        dense = self._unpack()
        shape_before = self._shape
        bare = False
        if len(newshape) == newsplit:
            newshape = newshape + (1,)
            newplan = np.array([1])
            newpadding = np.array([0])
            perm = perm + [len(perm)]
            shape_before = shape_before + (1,)
            bare = True
        res = self._rechunk(dense, perm, shape_before, newshape, newsplit, newplan, newpadding)
        res._bare_singleton = bare
        return res

    # ------------------------------------------------------------ functions
    def _chunk_batches(self):
        """(combo, batch) per run of equally shaped chunks: batch is a dense
        (records x chunks-in-run, *padded chunk shape) tensor gathered from the
        packed layout with one strided copy."""
        from bolt_amd.mi355x import functional as F
        es = self._dtype.itemsize
        g = self._geom
        n = len(g.vshape)
        lshape = local_shape(self._ctx, self._shape)
        nrec = int(np.prod(lshape[:self._split], dtype=np.int64))
        be = self._backend
        for combo in g.copies(unpack=False):
            shape, _, pstr, _, poff = combo
            cnt, ex = shape[:n], shape[n:]
            full = [nrec] + list(cnt) + list(ex)
            nb = int(np.prod(full, dtype=np.int64)) * es
            buf = _empty(nb, self._packed.device)
            if nb:
                dstr = [1] * len(full)
                for k in range(len(full) - 2, -1, -1):
                    dstr[k] = dstr[k + 1] * full[k + 1]
                be.copy_strided(self._packed, poff * es, buf, 0, full, [g.size] + list(pstr), dstr, es)
            yield combo, nrec, F.view(buf, [nrec * int(np.prod(cnt, dtype=np.int64))] + list(ex), self._dtype)

    def _first_chunk(self):
        from bolt_amd.mi355x import functional as F
        cs = self._geom.chunk_shape(self._geom.chunk_ids()[0])
        n = int(np.prod(cs, dtype=np.int64)) * self._dtype.itemsize
        return F.view(self._packed[:n], cs, self._dtype)

    def map(self, func, value_shape=None, dtype=None):
        """Apply an array -> array function to every chunk (chunk.py:349-410).

        ``func`` receives each chunk (with its padding) as a torch tensor on the
        GPU; it is vmapped over all chunks of equal shape at once.  The same
        shape inference, checks and exceptions as the reference: the function
        may change only the unchunked axes; the result's plan is value_shape.
        """
        from bolt_amd.mi355x import functional as F
        dev = self._packed.device
        func = F.user_fn(func)
        if value_shape is None or dtype is None:
            try:
                mapped = F.to_device(func(F.random_like(self.plan, self._dtype, dev)), dev)
            except Exception:
                mapped = F.to_device(func(self._first_chunk()), dev)
            if value_shape is None:
                value_shape = tuple(mapped.shape)
            if dtype is None:
                dtype = F.numpy_dtype(mapped.dtype)
        dtype = np.dtype(dtype)
        value_shape = tuple(int(v) for v in value_shape)
        chunked = np.where(self.plan != self.vshape)[0]
        unchunked = np.where(self.plan == self.vshape)[0]
        if len(value_shape) != len(self.plan):
            raise NotImplementedError('map on ChunkedArray cannot drop dimensions')
        if any([value_shape[i] != self.plan[i] for i in chunked]):
            raise ValueError('map cannot change the sizes of chunked dimensions')
        vshape = [value_shape[i] if i in unchunked else int(self.vshape[i]) for i in range(len(self.vshape))]
        newshape = tuple(int(k) for k in self.kshape) + tuple(vshape)
        g2 = ChunkGeometry(vshape, value_shape, self._padding)
        es2 = dtype.itemsize
        lshape = local_shape(self._ctx, newshape)
        nrec = int(np.prod(lshape[:self._split], dtype=np.int64))
        packed = _empty(nrec * g2.size * es2, dev)
        n = len(vshape)
        be = self._backend
        tdt = F.torch_dtype(dtype)
        for (combo, nrec_, batch), combo2 in zip(self._chunk_batches(), g2.copies(unpack=False)):
            shape2, _, pstr2, _, poff2 = combo2
            out = F.apply_batched(func, batch)
            if out is None:
                continue
            new = tuple(out.shape[1:])
            ex = tuple(batch.shape[1:])
            if len(unchunked) and any(new[i] != value_shape[i] for i in unchunked):
                raise Exception("Map operation did not produce values of uniform shape.")
            if len(chunked) and any(ex[i] != new[i] for i in chunked):
                raise Exception("Map operation changed the size of a chunked dimension")
            if new != tuple(shape2[n:]):
                raise Exception("Map operation did not produce values of uniform shape.")
            src = F.as_bytes(out.to(tdt))
            full = [nrec_] + list(shape2)
            sstr = [1] * len(full)
            for k in range(len(full) - 2, -1, -1):
                sstr[k] = sstr[k + 1] * full[k + 1]
            be.copy_strided(src, 0, packed, poff2 * es2, full, sstr, [g2.size] + list(pstr2), es2)
        res = self._constructor(packed, shape=newshape, split=self._split, dtype=dtype, plan=value_shape,
                                padding=self._padding, ordered=self._ordered, context=self._ctx)
        res._bare_singleton = self._bare_singleton
        return res

    def map_generic(self, func):
        """Apply an array -> object function to every chunk (chunk.py:412-432).

        The reference returns an object-dtype BoltArraySpark of shape
        kshape + number of chunks (split = its ndim); objects cannot live in
        HBM, so the result here is that object array on the host, as a local
        bolt array.  ``func`` receives each chunk as a torch tensor.
        """
        from bolt_amd.local import BoltArrayLocal
        from bolt_amd.mi355x import functional as F
        func = F.user_fn(func)
        g = self._geom
        es = self._dtype.itemsize
        lshape = local_shape(self._ctx, self._shape)
        nrec = int(np.prod(lshape[:self._split], dtype=np.int64))
        ids = g.chunk_ids()
        objs = []
        for r in range(nrec):
            for j in ids:
                cs = g.chunk_shape(j)
                off = (r * g.size + g.chunk_offset(j)) * es
                nb = int(np.prod(cs, dtype=np.int64)) * es
                objs.append(func(F.view(self._packed[off:off + nb], cs, self._dtype)))
        if self._ctx.world_size > 1:
            import torch.distributed as dist
            allobjs = [None] * self._ctx.world_size
            dist.all_gather_object(allobjs, objs, group=self._ctx.group)
            objs = [o for part in allobjs for o in part]
        newshape = tuple(int(s) for s in np.r_[self.kshape, g.nchunks])
        out = np.empty(len(objs), dtype=object)
        for i, o in enumerate(objs):
            out[i] = o
        return BoltArrayLocal(out.reshape(newshape))

    # ------------------------------------------------------------- records
    def records(self):
        """((key..., chunk id...), chunk ndarray) in key order (``tordd().sortByKey()``)."""
        from bolt_amd.mi355x.dist import gather_to_host
        ctx = self._ctx
        es = self._dtype.itemsize
        g = self._geom
        if ctx.world_size == 1:
            sizes = [self._packed.numel()]
        else:
            per = g.size * int(np.prod(self._shape[1:self._split], dtype=np.int64)) * es
            sizes = [(hi - lo) * per for lo, hi in ctx.bounds(self._shape[0])]
        host = gather_to_host(ctx, self._packed, sizes).view(self._dtype)
        kshape = self._shape[:self._split]
        ids = g.chunk_ids()
        for i, key in enumerate(np.ndindex(*kshape)):
            base = i * g.size
            for j in ids:
                off = g.chunk_offset(j)
                cs = g.chunk_shape(j)
                n = int(np.prod(cs, dtype=np.int64))
                chk = () if self._bare_singleton else tuple(int(c) for c in j)
                v = host[base + off: base + off + n].reshape(cs).copy()
                yield (tuple(int(k) for k in key) + chk, v.squeeze() if self._squeezed_records else v)

    def tordd(self):
        from bolt_amd.mi355x.records import RecordView
        return RecordView(list(self.records()), self._ctx.world_size)

    @property
    def _rdd(self):
        return self.tordd()

    def cache(self):
        """No-op: resident in HBM (chunk.py:648-652)."""

    def unpersist(self):
        """No-op (chunk.py:654-658)."""

    def __str__(self):
        s = "Chunked BoltArray\n"
        s += "shape: %s\n" % str(self.shape)
        return s

    def __repr__(self):
        string = str(self)
        if np.array_equal(self.vshape, [1]):
            newlines = [i for (i, char) in enumerate(string) if char == '\n']
            string = string[:newlines[-2] + 1]
            string += "shape: %s\n" % str(self.shape[:-1])
        string += "chunk size: %s\n" % str(tuple(self.plan))
        if self.padded:
            string += "padding: %s\n" % str(tuple(self.padding))
        else:
            string += "padding: none\n"
        return string
