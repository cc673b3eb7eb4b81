"""StackedArrayMI355X: bolt's StackedArray (bolt/spark/stack.py) on MI355X.

The reference gathers the records of each partition into "stacks" of up to
``size`` records (keys list + values stacked on a new leading axis) so that a
vectorised function runs once per stack (stack.py:49-66).  On the dense
layout a partition's records are consecutive rows in HBM, so a stack is a
zero-copy row range of the record buffer: map calls the function once per
stack on a torch view and writes its result rows.

Partitions: on one GPU the records are cut into ``npartitions`` contiguous
ranges exactly as the reference's parallelize cuts them (spark/construct.py
:69 -> ``data[i*L//n:(i+1)*L//n]``); across GPUs each rank's slab is one
partition.  (After a shuffle the reference's partitions hold hashed keys; a
dense array keeps key order, so stacks here are always consecutive keys.)
"""
import numpy as np

from bolt_amd.mi355x.dist import _empty, reslab_counts


def _stacks(parts, size):
    """Row ranges of the stacks of each partition (stack.py:49-66)."""
    out = []
    for a, b in parts:
        if b <= a:
            continue
        if size and 0 <= size:
            for lo in range(a, b, size):
                out.append((lo, min(b, lo + size)))
        else:
            out.append((a, b))
    return out


class StackedArrayMI355X(object):

    _metadata = ['_shape', '_split', '_rekeyed']

    def __init__(self, data, stacks, shape, split, dtype, context, rekeyed=False):
        self._data = data            # this rank's rows (uint8), row shape = shape[split:]
        self._stacks = stacks        # [(row lo, row hi)] of this rank's stacks
        self._shape = tuple(int(s) for s in shape)
        self._split = int(split)
        self._dtype = np.dtype(dtype)
        self._ctx = context
        self._rekeyed = rekeyed      # True: one record per stack, value = the row itself

    @classmethod
    def _from_array(cls, barray, size):
        ctx = barray._ctx
        lshape = barray._local_shape
        nrec = int(np.prod(lshape[:barray.split], dtype=np.int64))
        if ctx.world_size == 1:
            n = barray._npartitions or ctx.defaultParallelism
            parts = [(i * nrec // n, (i + 1) * nrec // n) for i in range(n)]
        else:
            parts = [(0, nrec)]
        return cls(barray._data, _stacks(parts, size), barray.shape, barray.split, barray.dtype, ctx)

    # ---------------------------------------------------------- properties
    @property
    def shape(self):
        return self._shape

    @property
    def split(self):
        return self._split

    @property
    def rekey(self):
        return self._rekeyed

    @property
    def dtype(self):
        return self._dtype

    @property
    def _constructor(self):
        return StackedArrayMI355X

    def _rowshape(self):
        return self._shape[self._split:]

    def _value(self, i):
        """Stack i as a torch view: (rows, *rowshape), or the row itself once rekeyed."""
        from bolt_amd.mi355x import functional as F
        lo, hi = self._stacks[i]
        rs = self._rowshape()
        rb = int(np.prod(rs, dtype=np.int64)) * self._dtype.itemsize
        v = F.view(self._data[lo * rb:hi * rb], (hi - lo,) + tuple(rs), self._dtype)
        return v[0] if self._rekeyed else v

    # ------------------------------------------------------------------ map
    def _probe(self, func):
        """The reference's shape test (stack.py:97-110) on the first stack,
        agreed across ranks: (a.shape, atest.shape, btest.shape, dtype) or an error."""
        import torch
        from bolt_amd.mi355x import functional as F
        res = None
        if self._stacks:
            x = self._value(0)
            if tuple(x.shape) == tuple(self._rowshape()):
                a, b = x[None], torch.stack((x, x))
            else:
                a, b = x, torch.cat((x, x))
            try:
                atest, btest = func(a), func(b)
            except Exception as e:
                res = ("RuntimeError", "Error evaluating function on test array, got error:\n %s" % e)
            else:
                ok = all(isinstance(t, (torch.Tensor, np.ndarray)) for t in (atest, btest))
                if not ok:
                    res = ("ValueError", "Function must return ndarray")
                else:
                    atest = F.to_device(atest, x.device)
                    res = (tuple(a.shape), tuple(atest.shape), tuple(btest.shape), tuple(b.shape),
                           str(F.numpy_dtype(atest.dtype)))
        if self._ctx.world_size > 1:
            import torch.distributed as dist
            allres = [None] * self._ctx.world_size
            dist.all_gather_object(allres, res, group=self._ctx.group)
            res = next((r for r in allres if r is not None), None)
        if res is None:
            raise ValueError("map of an empty stacked array")
        if res[0] in ("RuntimeError", "ValueError"):
            raise {"RuntimeError": RuntimeError, "ValueError": ValueError}[res[0]](res[1])
        return res

    def map(self, func):
        """Apply ``func`` to every stack (stack.py:80-139); same shape inference
        and exceptions as the reference.  ``func`` gets torch tensors on the GPU."""
        import torch
        from bolt_amd.mi355x import functional as F
        func = F.user_fn(func)
        ashape, atest, btest, bshape, dt = self._probe(func)
        dtype = np.dtype(dt)
        tdt = F.torch_dtype(dtype)
        dev = self._data.device
        if atest == btest:
            # every stack becomes one record keyed by its index (zipWithIndex)
            outshape = atest
            outs = []
            for i in range(len(self._stacks)):
                o = F.to_device(func(self._value(i)), dev)
                if tuple(o.shape) != outshape:
                    raise ValueError("stack %d maps to shape %s, expected %s" % (i, tuple(o.shape), outshape))
                outs.append(F.as_bytes(o.to(tdt)))
            if self._rekeyed:
                count = self._shape[0]
            else:
                count = len(self._stacks)
                if self._ctx.world_size > 1:
                    import torch.distributed as dist
                    allc = [None] * self._ctx.world_size
                    dist.all_gather_object(allc, count, group=self._ctx.group)
                    count = sum(allc)
            data = torch.cat(outs) if outs else _empty(0, dev)
            stacks = [(i, i + 1) for i in range(len(outs))]
            return self._constructor(data, stacks, (count,) + outshape, 1, dtype, self._ctx, rekeyed=True)
        if len(atest) and len(btest) and atest[0] == ashape[0] and btest[0] == bshape[0]:
            # records stay records; the value shape follows the function
            rowshape = atest[1:]
            outs = []
            for i in range(len(self._stacks)):
                lo, hi = self._stacks[i]
                o = F.to_device(func(self._value(i)), dev)
                want = rowshape if self._rekeyed else (hi - lo,) + rowshape
                if tuple(o.shape) != tuple(want):
                    raise ValueError("stack %d maps to shape %s, expected %s" % (i, tuple(o.shape), want))
                outs.append(F.as_bytes(o.to(tdt)))
            data = torch.cat(outs) if outs else _empty(0, dev)
            shape = self._shape[:self._split] + rowshape
            return self._constructor(data, list(self._stacks), shape, self._split, dtype, self._ctx,
                                     rekeyed=self._rekeyed)
        raise ValueError("Cannot infer effect of function on shape")

    def unstack(self):
        """Back to a BoltArrayMI355X (stack.py:68-78)."""
        from bolt_amd.mi355x.array import BoltArrayMI355X
        data = self._data
        if self._rekeyed and self._ctx.world_size > 1:
            import torch.distributed as dist
            counts = [None] * self._ctx.world_size
            dist.all_gather_object(counts, len(self._stacks), group=self._ctx.group)
            rb = int(np.prod(self._rowshape(), dtype=np.int64)) * self._dtype.itemsize
            data = reslab_counts(self._ctx, data, counts, rb)
        return BoltArrayMI355X(data, shape=self._shape, split=self._split, dtype=self._dtype,
                               context=self._ctx)

    # ------------------------------------------------------------- records
    def tordd(self):
        """Host view of the stacks: (list of keys, stacked values) per stack, or
        ((index,), value) once rekeyed -- the reference's intermediate RDD."""
        from bolt_amd.mi355x.records import RecordView
        from bolt_amd.mi355x.transfer import to_host
        recs = []
        rec0 = stack0 = 0  # this rank's first record / stack in global order
        if self._ctx.world_size > 1:
            import torch.distributed as dist
            sizes = [None] * self._ctx.world_size
            dist.all_gather_object(sizes, (len(self._stacks), self._stacks[-1][1] if self._stacks else 0),
                                   group=self._ctx.group)
            stack0 = sum(s[0] for s in sizes[:self._ctx.rank])
            rec0 = sum(s[1] for s in sizes[:self._ctx.rank])
        kshape = self._shape[:self._split]
        for i in range(len(self._stacks)):
            v = self._value(i)
            host = to_host(v.contiguous().reshape(-1).view(__import__("torch").uint8), self._dtype, tuple(v.shape))
            if self._rekeyed:
                recs.append(((stack0 + i,), host))
            else:
                lo, hi = self._stacks[i]
                keys = [tuple(int(k) for k in np.unravel_index(rec0 + r, kshape)) for r in range(lo, hi)]
                recs.append((keys, host))
        return RecordView(recs, self._ctx.world_size)

    @property
    def _rdd(self):
        return self.tordd()

    def __str__(self):
        return "Stacked BoltArray\nshape: %s\n" % str(self.shape)

    def __repr__(self):
        return str(self)
