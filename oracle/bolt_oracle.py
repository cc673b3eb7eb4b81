"""CPU oracle: a record-level numpy restatement of bolt's Spark-mode hot path.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker -- never by bolt_amd (the product
path has no CPU fallback).

It restates, record by record and partition by partition, what the reference
does with an RDD of (key tuple, value ndarray) records (beautifulNow1992/bolt
v0.7.1; file:line per function).  A "partitioned record set" is a list of
partitions, each a list of (key, value) pairs, as Spark local[N] holds them.
Pinned against fixtures produced by the reference itself
(tests/golden/make_golden.py -> tests/golden/golden.{json,npz});
tests/test_oracle_golden.py checks every fixture.

Numerics follow the reference: StatCounter's Welford merge runs in the record
dtype under numpy's casting rules (statcounter.py:51-59), partitions are
combined left to right with the Chan formula and its 10x size heuristic
(statcounter.py:67-99), sum is elementwise `+` in the input dtype
(array.py:269).
"""
import copy
from functools import reduce as _reduce
from itertools import product

import numpy as np


# ---------------------------------------------------------------- records
class RecSet(object):
    """Partitioned (key, value) records with bolt metadata (array.py:13-28)."""

    def __init__(self, parts, shape, split, dtype):
        self.parts = parts
        self.shape = tuple(int(s) for s in shape)
        self.split = int(split)
        self.dtype = np.dtype(dtype)

    def records(self):
        return [kv for p in self.parts for kv in p]


def _contiguous_parts(records, n):
    L = len(records)
    return [records[i * L // n:(i + 1) * L // n] for i in range(n)]


def parallelize(x, axis=(0,), npartitions=2, dtype=None):
    """ConstructSpark.array (spark/construct.py:43-70), quirk included:
    records are taken from x.transpose(keys+values) but the shape stays x.shape."""
    x = np.asarray(x) if dtype is None else np.asarray(x, dtype)
    shape = x.shape
    axes = (axis,) if isinstance(axis, int) else tuple(axis)
    if min(axes) < 0 or max(axes) > len(shape) - 1:
        raise ValueError("invalid key axes")
    perm = list(axes) + [i for i in range(len(shape)) if i not in axes]
    split = len(axes)
    xt = x.transpose(perm)
    kshape, vshape = shape[:split], shape[split:]
    vals = xt.reshape((int(np.prod(kshape)),) + vshape)
    keys = list(np.ndindex(*kshape))
    recs = [(tuple(int(k) for k in key), vals[i]) for i, key in enumerate(keys)]
    return RecSet(_contiguous_parts(recs, npartitions), shape, split, x.dtype)


def toarray(rs):
    """sortByKey + collect + reshape (array.py:1006-1014)."""
    recs = sorted(rs.records(), key=lambda kv: kv[0])
    return np.asarray([v for _, v in recs]).reshape(rs.shape)


# ---------------------------------------------------------------- chunk plan
def getplan(vshape, dtype, size="150", axes=None, padding=None):
    """ChunkedArray.getplan (chunk.py:434-512)."""
    vshape = np.asarray(vshape)
    plan = vshape.copy()
    if axes is None:
        axes = np.arange(len(vshape)) if isinstance(size, str) else np.arange(len(size))
    else:
        axes = np.asarray(axes, 'int')
    pad = np.zeros(len(vshape), dtype=int)
    if padding is not None:
        pad[axes] = padding
    if isinstance(size, tuple):
        plan[axes] = size
    elif isinstance(size, str):
        nbytes = 1000.0 * float(size)
        item = np.dtype(dtype).itemsize
        mask = np.zeros(len(vshape), dtype=bool)
        mask[axes] = True
        dims = vshape[mask]
        if nbytes <= item:
            s = np.ones(len(axes))
        else:
            rem = 1.0 * np.prod(vshape) * item
            s = []
            for i, d in enumerate(dims):
                per = rem / d
                if per >= nbytes:
                    s.append(1)
                    rem = per
                    continue
                s.append(min(d, np.floor(nbytes / per)))
                s[i + 1:] = plan[i + 1:]
                break
        plan[axes] = s
    else:
        raise ValueError("Chunk size not understood")
    return plan, pad


def chunk_slices(plan, padding, vshape):
    """getslices (chunk.py:574-618): full chunks get the right pad (clipped by
    slicing), a remainder chunk is [floor(d/s)*s - p, d)."""
    out = []
    for s, p, d in zip(plan, padding, vshape):
        s, p, d = int(s), int(p), int(d)
        n, rem = d // s, d % s
        sl = [slice(0 if j == 0 else j * s - p, j * s + s + p) for j in range(n)]
        if rem:
            sl.append(slice(n * s - p, d))
        out.append(sl)
    return out


class ChunkSet(object):
    """Chunk records ((key..., chunk id...), chunk) with plan/padding (chunk.py:11-33)."""

    def __init__(self, parts, shape, split, dtype, plan, padding):
        self.parts = parts
        self.shape = tuple(int(s) for s in shape)
        self.split = int(split)
        self.dtype = np.dtype(dtype)
        self.plan = np.asarray(plan, dtype=int)
        self.padding = np.asarray(padding, dtype=int)

    @property
    def kshape(self):
        return np.asarray(self.shape[:self.split])

    @property
    def vshape(self):
        return np.asarray(self.shape[self.split:])

    def records(self):
        return [kv for p in self.parts for kv in p]


def chunk(rs, size="150", axis=None, padding=None):
    """BoltArraySpark.chunk -> ChunkedArray._chunk (array.py:678-714, chunk.py:87-144)."""
    if not isinstance(size, str):
        size = tuple(size) if isinstance(size, (tuple, list)) else (size,)
    if axis is not None and not isinstance(axis, tuple):
        axis = tuple(axis) if isinstance(axis, list) else (axis,)
    if padding is not None and not isinstance(padding, tuple):
        padding = tuple(padding) if isinstance(padding, list) else (padding,)
    if rs.split == len(rs.shape) and padding is None:
        parts = [[(k + (0,), np.array(v, ndmin=1)) for k, v in p] for p in rs.parts]
        return ChunkSet(parts, rs.shape + (1,), rs.split, rs.dtype, (1,), [0])
    vshape = rs.shape[rs.split:]
    plan, pad = getplan(vshape, rs.dtype, size, axis, padding)
    if any(x + y > z for x, y, z in zip(plan, pad, vshape)):
        raise ValueError("Chunk sizes plus padding sizes cannot exceed value dimensions")
    if any(x > y for x, y in zip(pad, plan)):
        raise ValueError("Padding sizes cannot exceed chunk sizes")
    sl = chunk_slices(plan, pad, vshape)
    scheme = list(product(*[list(enumerate(s)) for s in sl]))
    parts = []
    for p in rs.parts:
        q = []
        for k, v in p:
            for combo in scheme:
                chk = tuple(c[0] for c in combo)
                q.append((k + chk, v[tuple(c[1] for c in combo)]))
        parts.append(q)
    return ChunkSet(parts, rs.shape, rs.split, rs.dtype, plan, pad)


def _nchunks(plan, vshape):
    return [int(np.ceil(1.0 * d / s)) for s, d in zip(plan, vshape)]


def _strip(idx, value, number, padding, axes):
    """removepad (chunk.py:514-550), indexing with a tuple."""
    sl = []
    for a, (i, p, n) in enumerate(zip(idx, padding, number)):
        m = (a in axes) and p != 0
        lo = 0 if (i == 0 or not m) else p
        hi = None if (i == n - 1 or not m) else -p
        sl.append(slice(lo, hi))
    return value[tuple(sl)]


def _stack(nested):
    """allstack (bolt/utils.py:193-208)."""
    def go(v, depth):
        if isinstance(v[0], np.ndarray):
            return np.concatenate(v, axis=depth)
        return np.concatenate([go(x, depth + 1) for x in v], axis=depth)
    return go(nested, 0)


def unchunk(cs):
    """ChunkedArray.unchunk (chunk.py:146-200): strip padding, reassemble per key."""
    split, vshape = cs.split, cs.vshape
    number = _nchunks(cs.plan, vshape)
    n = len(vshape)
    recs = cs.records()
    if np.any(cs.padding != 0):
        recs = [(k, _strip(k[split:], v, number, cs.padding, range(n))) for k, v in recs]
    if np.array_equal(cs.plan, vshape):
        out = [(k[:split], v) for k, v in recs]
    else:
        groups = {}
        for k, v in recs:
            groups.setdefault(k[:split], []).append((k[split:], v))
        out = []
        for key in sorted(groups):
            arr = np.empty(number, dtype=object)
            for chk, v in groups[key]:
                arr[chk] = v
            out.append((key, _stack(arr.tolist())))
    shape = cs.shape
    if np.array_equal(vshape, [1]):
        out = [(k, np.squeeze(v)) for k, v in out]
        shape = shape[:-1]
    return RecSet([out], shape, split, cs.dtype)


def chunk_map(cs, func, value_shape=None, dtype=None):
    """ChunkedArray.map (chunk.py:349-410): func on every chunk; only unchunked
    axes may change; the new plan is value_shape."""
    if value_shape is None or dtype is None:
        try:
            mapped = func(np.random.randn(*cs.plan).astype(cs.dtype))
        except Exception:
            mapped = func(cs.records()[0][1])
        value_shape = mapped.shape if value_shape is None else value_shape
        dtype = mapped.dtype if dtype is None else dtype
    chunked = np.where(cs.plan != cs.vshape)[0]
    unchunked = np.where(cs.plan == cs.vshape)[0]
    if len(value_shape) != len(cs.plan):
        raise NotImplementedError('map on ChunkedArray cannot drop dimensions')
    if any(value_shape[i] != cs.plan[i] for i in chunked):
        raise ValueError('map cannot change the sizes of chunked dimensions')

    def apply(v):
        new = func(v)
        if any(new.shape[i] != value_shape[i] for i in unchunked):
            raise Exception("Map operation did not produce values of uniform shape.")
        if any(v.shape[i] != new.shape[i] for i in chunked):
            raise Exception("Map operation changed the size of a chunked dimension")
        return new

    parts = [[(k, apply(v)) for k, v in p] for p in cs.parts]
    vshape = [value_shape[i] if i in unchunked else cs.vshape[i] for i in range(len(cs.vshape))]
    shape = tuple(int(x) for x in np.r_[cs.kshape, vshape])
    return ChunkSet(parts, shape, cs.split, dtype, value_shape, cs.padding)


def chunk_map_generic(cs, func):
    """ChunkedArray.map_generic (chunk.py:412-432): object per chunk, shape kshape + nchunks."""
    recs = sorted(cs.records(), key=lambda kv: kv[0])
    out = np.empty(len(recs), dtype=object)
    for i, (_, v) in enumerate(recs):
        out[i] = func(v)
    return out.reshape(tuple(int(x) for x in np.r_[cs.kshape, _nchunks(cs.plan, cs.vshape)]))


def keys_to_values(cs, axes, size=None):
    """ChunkedArray.keys_to_values (chunk.py:202-289): relabel, group by
    (stationary keys, new chunk ids, old chunk ids), stack each group."""
    if len(axes) == 0:
        return cs
    split = cs.split
    kmask = np.zeros(split, dtype=bool)
    kmask[list(axes)] = True
    if size is None:
        size = cs.kshape[kmask]
    size = np.asarray(size, dtype=int)
    newplan = np.r_[size, cs.plan]
    newshape = tuple(np.r_[cs.kshape[~kmask], cs.kshape[kmask], cs.vshape].astype(int).tolist())
    newpad = np.r_[np.zeros(len(axes), dtype=int), cs.padding]
    groups = {}
    for k, v in cs.records():
        keys, chks = np.asarray(k[:split]), tuple(k[split:])
        mov, sta = keys[kmask], keys[~kmask]
        newchk = tuple(int(m) for m in mov // size)
        label = tuple(int(m) for m in mov % size)
        gk = tuple(int(s) for s in sta) + newchk + chks
        groups.setdefault(gk, []).append((label, v))
    out = []
    for gk in sorted(groups):
        items = sorted(groups[gk], key=lambda t: t[0])
        labels = np.asarray([t[0] for t in items])
        lshape = tuple(labels.max(axis=0) - labels.min(axis=0) + 1)
        out.append((gk, np.asarray([t[1] for t in items]).reshape(lshape + items[0][1].shape)))
    res = ChunkSet([out], newshape, split - len(axes), cs.dtype, newplan, newpad)
    if np.array_equal(cs.vshape, [1]):
        # squeeze the all-keys singleton (chunk.py:284-287, numpy<1.13 semantics)
        res.parts = [[(k[:-1], np.squeeze(v)) for k, v in out]]
        res.shape = res.shape[:-1]
        res.plan = res.plan[:-1]
        res.padding = res.padding[:len(res.plan)]
    return res


def values_to_keys(cs, axes):
    """ChunkedArray.values_to_keys (chunk.py:291-347): strip padding on the
    moved axes, emit one record per index of the moved dims."""
    split = cs.split
    nv = len(cs.vshape)
    vmask = np.zeros(nv, dtype=bool)
    vmask[list(axes)] = True
    newplan = cs.plan[~vmask]
    newshape = tuple(np.r_[cs.kshape, cs.vshape[vmask], cs.vshape[~vmask]].astype(int).tolist())
    newpad = cs.padding[~vmask]
    number = _nchunks(cs.plan, cs.vshape)
    moving = cs.plan[vmask]
    out = []
    for k, v in cs.records():
        key, chk = k[:split], np.asarray(k[split:])
        if np.any(cs.padding != 0):
            v = _strip(tuple(chk), v, number, cs.padding, list(axes))
        offs = chk[vmask] * moving
        for b in np.ndindex(*np.asarray(v.shape)[vmask]):
            sl = [slice(None)] * nv
            for a, bi in zip(np.flatnonzero(vmask), b):
                sl[a] = bi
            nk = tuple(int(x) for x in key) + tuple(int(o + bi) for o, bi in zip(offs, b))
            out.append((nk + tuple(int(c) for c in chk[~vmask]), v[tuple(sl)]))
    res = ChunkSet([out], newshape, split + len(axes), cs.dtype, newplan, newpad)
    if len(newshape) == split + len(axes):
        res.parts = [[(k, np.array(v, ndmin=1)) for k, v in out]]
        res.shape = res.shape + (1,)
        res.plan = np.array([1])
        res.padding = np.array([0])
    return res


# ---------------------------------------------------------------- swap etc.
def swap(rs, kaxes, vaxes, size="150"):
    """BoltArraySpark.swap (array.py:716-763) through the chunk machinery."""
    kaxes = [int(k) for k in np.atleast_1d(np.asarray(kaxes, dtype=int))]
    vaxes = [int(v) for v in np.atleast_1d(np.asarray(vaxes, dtype=int))]
    if len(kaxes) == rs.split and len(vaxes) == 0:
        raise ValueError('Cannot perform a swap that would end up with all data on a single key')
    if len(kaxes) == 0 and len(vaxes) == 0:
        return rs
    c = chunk(rs, size)
    c = keys_to_values(c, kaxes)
    c = values_to_keys(c, [v + len(kaxes) for v in vaxes])
    return unchunk(c)


def _keys_permute(rs, p):
    recs = [(tuple(k[i] for i in p), v) for k, v in rs.records()]
    shape = tuple(rs.shape[i] for i in p) + rs.shape[rs.split:]
    return RecSet([sorted(recs, key=lambda kv: kv[0])], shape, rs.split, rs.dtype)


def _values_permute(rs, p):
    recs = [(k, v.transpose(p)) for k, v in rs.records()]
    shape = rs.shape[:rs.split] + tuple(rs.shape[rs.split + i] for i in p)
    return RecSet([recs], shape, rs.split, rs.dtype)


def transpose(rs, p):
    """BoltArraySpark.transpose (array.py:765-808): swap the crossing axes,
    then permute keys (shapes.py:66-89) and values (shapes.py:136-159)."""
    p = np.asarray(p)
    split = rs.split
    nk, nv = p[:split], p[split:]
    sk = np.sort(nv[nv < split])
    sv = np.sort(nk[nk >= split])
    stk = np.sort(nk[nk < split])
    stv = np.sort(nv[nv >= split])
    pswap = np.r_[stk, sv, sk, stv]
    px = np.argsort(pswap)[p]
    out = swap(rs, sk, sv - split) if (len(sk) or len(sv)) else rs
    out = _keys_permute(out, [int(i) for i in px[:split]])
    return _values_permute(out, [int(i) - split for i in px[split:]])


def _isreshapeable(new, old):
    """bolt/utils.py:174-191: same number of elements, else ValueError."""
    if int(np.prod(new)) != int(np.prod(old)):
        raise ValueError("Total size of new keys must remain unchanged")


def keys_reshape(rs, new):
    """Keys.reshape (shapes.py:40-64): every key re-raveled into the new key shape."""
    new = tuple(int(v) for v in new)
    old = tuple(rs.shape[:rs.split])
    _isreshapeable(new, old)
    if new == old:
        return rs
    recs = [(tuple(int(i) for i in np.unravel_index(np.ravel_multi_index(k, old), new)), v)
            for k, v in rs.records()]
    return RecSet([recs], new + tuple(rs.shape[rs.split:]), len(new), rs.dtype)


def values_reshape(rs, new):
    """Values.reshape (shapes.py:111-134): every record's value reshaped."""
    new = tuple(int(v) for v in new)
    old = tuple(rs.shape[rs.split:])
    _isreshapeable(new, old)
    if new == old:
        return rs
    recs = [(k, v.reshape(new)) for k, v in rs.records()]
    return RecSet([recs], tuple(rs.shape[:rs.split]) + new, rs.split, rs.dtype)


# ---------------------------------------------------------------- statistics
class StatCounter(object):
    """statcounter.py:28-130 (Welford merge, Chan combine), in the record dtype."""

    def __init__(self, values=(), need_m2=True):
        self.n = 0
        self.mu = 0.0
        self.m2 = 0.0
        self.need_m2 = need_m2
        for v in values:
            self.merge(v)

    def merge(self, value):
        self.n += 1
        delta = value - self.mu
        self.mu += delta / self.n
        if self.need_m2:
            self.m2 += delta * (value - self.mu)
        return self

    def combine(self, other):
        if other is self:
            return self.merge(copy.deepcopy(other))
        if self.n == 0:
            self.n, self.mu, self.m2 = other.n, other.mu, other.m2
        elif other.n != 0:
            delta = other.mu - self.mu
            if other.n * 10 < self.n:
                self.mu = self.mu + (delta * other.n) / (self.n + other.n)
            elif self.n * 10 < other.n:
                self.mu = other.mu - (delta * self.n) / (self.n + other.n)
            else:
                self.mu = (self.mu * self.n + other.mu * other.n) / (self.n + other.n)
            if self.need_m2:
                self.m2 += other.m2 + (delta * delta * self.n * other.n) / (self.n + other.n)
            self.n += other.n
        return self

    def stat(self, name):
        if name == 'mean':
            return self.mu
        var = float('nan') if self.n == 0 else self.m2 / self.n
        return var if name == 'variance' else np.sqrt(var)


def align(rs, axis):
    """BoltArraySpark._align (array.py:85-115): reduced axes become the keys."""
    if not all(0 <= a < len(rs.shape) for a in axis):
        raise ValueError("axes not valid for an ndarray of shape: %s" % str(rs.shape))
    tokeys = [a - rs.split for a in axis if a >= rs.split]
    tovalues = [a for a in range(rs.split) if a not in axis]
    if tokeys or tovalues:
        return swap(rs, tovalues, tokeys)
    return rs


def _normalise_axis(rs, axis):
    if axis is None:
        axis = list(range(len(rs.shape)))
    return tuple(axis) if isinstance(axis, (tuple, list)) else (axis,)


def stat(rs, name, axis=None, keepdims=False):
    """BoltArraySpark._stat with a name (array.py:284-334): one StatCounter per
    partition, combined in partition order; a 0-d result becomes a scalar."""
    axis = _normalise_axis(rs, axis)
    sw = align(rs, axis)
    counters = [StatCounter((v for _, v in p), need_m2=(name != 'mean')) for p in sw.parts]
    arr = _reduce(lambda a, b: a.combine(b), counters).stat(name)
    if keepdims:
        for i in axis:
            arr = np.expand_dims(arr, axis=i)
    arr = np.asarray(arr) if not np.isscalar(arr) else arr
    if isinstance(arr, np.ndarray) and arr.shape == ():
        return arr.reshape(1)[0]
    return arr


def reduce_(rs, func, axis=None, keepdims=False):
    """BoltArraySpark.reduce (array.py:243-282): treeReduce of ``func`` over the
    aligned records (per partition, then across partitions), input dtype."""
    axis = _normalise_axis(rs, axis)
    sw = align(rs, axis)
    partials = [_reduce(func, [v for _, v in p]) for p in sw.parts if p]
    arr = _reduce(func, partials)
    if keepdims:
        for i in axis:
            arr = np.expand_dims(arr, axis=i)
    if not isinstance(arr, np.ndarray):
        return arr
    if arr.shape == (1,):
        return arr[0]
    return arr


def sum_(rs, axis=None, keepdims=False):
    """sum = reduce(operator.add) (array.py:381-395)."""
    return reduce_(rs, lambda a, b: a + b, axis, keepdims)


def max_(rs, axis=None, keepdims=False):
    """max = reduce(numpy.maximum) (array.py:397-411)."""
    return reduce_(rs, np.maximum, axis, keepdims)


def min_(rs, axis=None, keepdims=False):
    """min = reduce(numpy.minimum) (array.py:413-427)."""
    return reduce_(rs, np.minimum, axis, keepdims)


# ---------------------------------------------------------------- indexing
def slicify(slc, dim):
    """bolt/utils.py:105-147: explicit start/stop/step; stop -1 marks a negative
    step running past the front; an int i is slice(i, i+1, 1)."""
    if isinstance(slc, slice):
        start = 0 if slc.start is None else slc.start
        stop = dim if slc.stop is None else slc.stop
        step = 1 if slc.step is None else slc.step
        start = start + dim if start < 0 else start
        stop = stop + dim if stop < 0 else stop
        if step > 0:
            start, stop = max(start, 0), min(stop, dim)
        else:
            stop = -1 if stop < 0 else stop
            start = dim - 1 if start > dim else start
        return slice(start, stop, step)
    if isinstance(slc, int):
        return slice(slc + dim if slc < 0 else slc, (slc + dim if slc < 0 else slc) + 1, 1)
    raise ValueError("Type for slice %s not recongized" % type(slc))


def _getbasic(rs, index):
    """array.py:480-512 (value index as a tuple)."""
    ks, vs = index[:rs.split], index[rs.split:]

    def keep(key):
        for k, s in zip(key, ks):
            inside = (s.start <= k < s.stop) if s.step > 0 else (s.stop < k <= s.start)
            if not inside or (k - s.start) % s.step:
                return False
        return True

    vt = tuple(s if s.stop != -1 else slice(s.start, None, s.step) for s in vs)
    parts = [[(tuple((k - s.start) // s.step for k, s in zip(key, ks)), v[vt] if vs else v)
              for key, v in p if keep(key)] for p in rs.parts]
    shape = tuple(int(np.ceil((s.stop - s.start) / float(s.step))) for s in index)
    return RecSet(parts, shape, rs.split, rs.dtype)


def _getadvanced(rs, index):
    """array.py:514-559: listed keys in record order, each expanded into the
    value positions of its (last consecutive) group, renumbered in order."""
    index = [np.asarray(i) for i in index]
    ishape = index[0].shape
    if not all(i.shape == ishape for i in index):
        raise ValueError("shape mismatch: indexing arrays could not be broadcast together")
    flat = []
    for i, d in zip(index, rs.shape):
        if not all(np.asarray(v).dtype == int for v in i):
            raise ValueError("indices must be integers")
        if np.any(i >= d):
            raise ValueError("indices out of bounds for axis with size %s" % d)
        flat.append(i.flatten())
    keys = [tuple(int(v) for v in t) for t in zip(*flat[:rs.split])]
    vals = [tuple(int(v) for v in t) for t in zip(*flat[rs.split:])]
    groups = {}
    for pos, (k, v) in enumerate(zip(keys, vals) if vals else [(k, None) for k in keys]):
        if pos == 0 or keys[pos - 1] != k:
            groups[k] = []
        groups[k].append(v)
    out = []
    for key, v in rs.records():
        if key in groups:
            out.extend([v[t] for t in groups[key]] if vals else [v])
    recs = [(tuple(int(i) for i in np.unravel_index(n, ishape)), val) for n, val in enumerate(out)]
    return RecSet([recs], ishape, len(ishape), rs.dtype)


def _getmixed(rs, index):
    """array.py:561-593 (value index as a tuple): the listed axis first, then
    the basic selection through getitem again, as the reference composes it."""
    loc = [i for i, x in enumerate(index) if isinstance(x, np.ndarray)][0]
    idx = list(index[loc])
    if isinstance(idx[0], (tuple, list, np.ndarray)):
        raise ValueError("When mixing basic and advanced indexing, advanced index must be one-dimensional")
    if loc < rs.split:
        parts = [[(key[:loc] + (idx.index(key[loc]),) + key[loc + 1:], v) for key, v in p if key[loc] in idx]
                 for p in rs.parts]
    else:
        vt = [slice(None)] * (len(rs.shape) - rs.split)
        vt[loc - rs.split] = idx
        parts = [[(key, v[tuple(vt)]) for key, v in p] for p in rs.parts]
    shape = list(rs.shape)
    shape[loc] = len(idx)
    rest = list(index)
    rest[loc] = slice(0, None, None)
    return getitem(RecSet(parts, shape, rs.split, rs.dtype), tuple(rest))


def squeeze(rs, axis=None):
    """BoltArraySpark.squeeze (array.py:879-918)."""
    if not any(d == 1 for d in rs.shape):
        return rs
    if axis is None:
        drop = [i for i, d in enumerate(rs.shape) if d == 1]
    elif isinstance(axis, int):
        drop = [axis]
    elif isinstance(axis, tuple):
        drop = list(axis)
    else:
        raise ValueError("an integer or tuple is required for the axis")
    if any(rs.shape[i] > 1 for i in drop):
        raise ValueError("cannot select an axis to squeeze out which has size greater than one")
    vdrop = tuple(d - rs.split for d in drop if d >= rs.split)
    parts = [[(tuple(k for i, k in enumerate(key) if i not in drop), v.squeeze(vdrop) if vdrop else v)
              for key, v in p] for p in rs.parts]
    shape = tuple(s for i, s in enumerate(rs.shape) if i not in drop)
    split = len([d for d in range(rs.split) if d not in drop])
    return RecSet(parts, shape, split, rs.dtype)


def getitem(rs, index):
    """BoltArraySpark.__getitem__ (array.py:595-676)."""
    index = list(index) if isinstance(index, tuple) else [index]
    int_locs = [i for i, x in enumerate(index) if isinstance(x, int)]
    nd = len(rs.shape)
    if len(index) > nd:
        raise ValueError("Too many indices for array")
    if not all(isinstance(i, (slice, int, list, tuple, np.ndarray)) for i in index):
        raise ValueError("Each index must either be a slice, int, list, set, or ndarray")
    index += [slice(0, None, None)] * (nd - len(index))
    for n, idx in enumerate(index):
        size = rs.shape[n]
        if isinstance(idx, (slice, int)):
            s = slicify(idx, size)
            lo, hi = (s.start, s.stop) if s.step > 0 else (s.stop, s.start)
            if lo > size - 1 or hi < 1 or lo >= hi:
                raise ValueError("Index %s in dimension %d would produce an empty dimension" % (idx, n))
            index[n] = s
        else:
            a = np.array(idx)
            a[np.where(a < 0)] += size
            if a.min() < 0 or a.max() > size - 1:
                raise ValueError("Index %s out of bounds in dimension %d" % (idx, n))
            index[n] = a
    if all(isinstance(i, slice) for i in index):
        out = _getbasic(rs, index)
    elif all(isinstance(i, np.ndarray) for i in index):
        out = _getadvanced(rs, index)
    elif sum(isinstance(i, np.ndarray) for i in index) == 1:
        out = _getmixed(rs, index)
    else:
        raise NotImplementedError("only a single advanced index may be mixed with basic indices")
    if len(int_locs) == nd:
        return toarray(squeeze(out)).reshape(())[()]
    return squeeze(out, tuple(int_locs))


def concatenate(rs, other, axis=0):
    """BoltArraySpark.concatenate (array.py:429-478): an ndarray is parallelized
    on the same key axes; key axis -> union with shifted keys, value axis ->
    join by key and numpy.concatenate of the two values."""
    if isinstance(other, np.ndarray):
        other = parallelize(other, axis=tuple(range(rs.split)))
    elif not isinstance(other, RecSet):
        raise ValueError("other must be local array or spark array, got %s" % type(other))
    if not all(x == y or i == axis for i, (x, y) in enumerate(zip(rs.shape, other.shape))):
        raise ValueError("all the input array dimensions except for the concatenation axis must match exactly")
    if rs.split != other.split:
        raise NotImplementedError("two arrays must have the same split ")
    if axis < rs.split:
        shift = rs.shape[axis]
        moved = [(k[:axis] + (k[axis] + shift,) + k[axis + 1:], v) for k, v in other.records()]
        parts = rs.parts + [moved]
    else:
        theirs = dict(other.records())
        parts = [[(k, np.concatenate((v, theirs[k]), axis=axis - rs.split)) for k, v in p if k in theirs]
                 for p in rs.parts]
    shape = tuple(x + y if i == axis else x for i, (x, y) in enumerate(zip(rs.shape, other.shape)))
    return RecSet(parts, shape, rs.split, rs.dtype)


# ---------------------------------------------------------------- functional
def align_keys(rs, axis):
    """BoltArraySpark._align (array.py:85-115) for map/filter: swap so that axis are the keys."""
    tokeys = [a - rs.split for a in axis if a >= rs.split]
    tovalues = [a for a in range(rs.split) if a not in axis]
    return swap(rs, tovalues, tokeys) if (tokeys or tovalues) else rs


def map_(rs, func, axis=(0,), value_shape=None, dtype=None, with_keys=False):
    """BoltArraySpark.map (array.py:125-191)."""
    axis = tuple(axis)
    sw = align_keys(rs, axis)
    test = (lambda x: func(((0,), x))) if with_keys else func
    if value_shape is None or dtype is None:
        try:
            mapped = test(np.random.randn(*sw.shape[sw.split:]).astype(rs.dtype))
        except Exception:
            mapped = test(sw.records()[0][1])
        value_shape = mapped.shape if value_shape is None else value_shape
        dtype = mapped.dtype if dtype is None else dtype
    value_shape = tuple(value_shape)
    parts = [[(k, func((k, v)) if with_keys else func(v)) for k, v in p] for p in sw.parts]
    for p in parts:
        for _, v in p:
            if len(v.shape) > 0 and v.shape != value_shape:
                raise Exception("Map operation did not produce values of uniform shape.")
    shape = tuple(sw.shape[a] for a in range(len(axis))) + value_shape
    return RecSet(parts, shape, sw.split, dtype)


def filter_(rs, func, axis=(0,), sort=False):
    """BoltArraySpark.filter (array.py:193-241): kept records renumbered in record order."""
    axis = tuple(axis)
    sw = align_keys(rs, axis)
    kept = [(k, v) for k, v in sw.records() if func(v)]
    if sort:
        kept = sorted(kept, key=lambda kv: kv[0])
    recs = [((i,), v) for i, (_, v) in enumerate(kept)]
    shape = (len(recs),) + tuple(sw.shape[len(axis):]) if recs else (0,)
    return RecSet([recs], shape, 1, sw.dtype)


class StackSet(object):
    """StackedArray (stack.py): per-partition stacks of (keys list, stacked values)."""

    def __init__(self, parts, shape, split, rekeyed=False):
        self.parts, self.shape, self.split, self.rekeyed = parts, tuple(shape), split, rekeyed

    def records(self):
        return [kv for p in self.parts for kv in p]


def stack(rs, size=None):
    """StackedArray.stack (stack.py:49-66)."""
    parts = []
    for p in rs.parts:
        q, keys, vals = [], [], []
        for k, v in p:
            keys.append(k)
            vals.append(v)
            if size and 0 <= size <= len(keys):
                q.append((keys, np.asarray(vals)))
                keys, vals = [], []
        if keys:
            q.append((keys, np.asarray(vals)))
        parts.append(q)
    return StackSet(parts, rs.shape, rs.split)


def stack_map(ss, func):
    """StackedArray.map (stack.py:80-139)."""
    vshape = ss.shape[ss.split:]
    x = ss.records()[0][1]
    a, b = (np.asarray([x]), np.asarray([x, x])) if x.shape == vshape else (x, np.concatenate((x, x)))
    try:
        at, bt = func(a), func(b)
    except Exception as e:
        raise RuntimeError("Error evaluating function on test array, got error:\n %s" % e)
    if not (isinstance(at, np.ndarray) and isinstance(bt, np.ndarray)):
        raise ValueError("Function must return ndarray")
    if at.shape == bt.shape:
        if ss.rekeyed:
            parts = [[(k, func(v)) for k, v in p] for p in ss.parts]
            shape = (ss.shape[0],) + at.shape
        else:
            vals = [func(v) for _, v in ss.records()]
            parts = [[((i,), v) for i, v in enumerate(vals)]]
            shape = (len(vals),) + at.shape
        return StackSet(parts, shape, 1, True)
    if at.shape[0] == a.shape[0] and bt.shape[0] == b.shape[0]:
        parts = [[(k, func(v)) for k, v in p] for p in ss.parts]
        return StackSet(parts, ss.shape[:ss.split] + at.shape[1:], ss.split, ss.rekeyed)
    raise ValueError("Cannot infer effect of function on shape")


def unstack(ss):
    """StackedArray.unstack (stack.py:68-78)."""
    if ss.rekeyed:
        recs = ss.records()
    else:
        recs = [(k, v) for ks, vs in ss.records() for k, v in zip(ks, list(vs))]
    dt = np.asarray(recs[0][1]).dtype if recs else np.float64
    return RecSet([recs], ss.shape, ss.split, dt)


def repartition(rs, n):
    """Records in key order split into n contiguous partitions (parallelize's cut)."""
    recs = sorted(rs.records(), key=lambda kv: kv[0])
    return RecSet(_contiguous_parts(recs, n), rs.shape, rs.split, rs.dtype)
