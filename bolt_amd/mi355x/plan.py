"""Host-side planning for the MI355X backend: chunk plans, chunk geometry,
net permutations of swap/transpose, reduction layouts and result dtypes.

Everything here is integer/shape arithmetic that decides what the HIP kernels
do; no data is touched.  Each function restates the reference semantics it
cites, including the quirks a drop-in must keep.  The chunk-plan functions
(getplan, getslices, removepad_slices) follow chunk.py:434-618 step by step,
because their integer results must be identical to the reference's; the
geometry, permutation and reduction-layout code below them is new.
"""
import functools
from itertools import product

import numpy as np


# --------------------------------------------------------------------------
# chunk plans  (bolt/spark/chunk.py)
# --------------------------------------------------------------------------

def getmask(inds, n):
    """Boolean mask of length n with ``inds`` set (chunk.py:620-636)."""
    inds = np.asarray(inds, 'int')
    mask = np.zeros(n, dtype=bool)
    mask[inds] = True
    return mask


def getplan(vshape, dtype, size="150", axes=None, padding=None):
    """Chunk plan (elements per chunk along each value axis) and padding.

    Restates ChunkedArray.getplan (chunk.py:434-512):
      * str size = kilobytes x 1000 bytes (chunk.py:483); greedy over the value
        axes in order: an axis whose full extent keeps the chunk >= size gets
        chunk 1, the first axis that does not gets floor(size/minsize) (capped
        at its extent) and every later axis stays whole (chunk.py:494-505);
        size <= itemsize gives all ones (chunk.py:490-491);
      * tuple size is written onto ``axes`` (chunk.py:478-479);
      * padding (int or tuple) is broadcast onto ``axes`` (chunk.py:473-475);
      * anything else -> ValueError (chunk.py:509-510).
    ``vshape`` is the value shape, ``dtype`` the array dtype.
    """
    vshape = np.asarray(vshape)
    plan = vshape.copy()

    if axes is None:
        if isinstance(size, str):
            axes = np.arange(len(vshape))
        else:
            axes = np.arange(len(size))
    else:
        axes = np.asarray(axes, 'int')

    pad = np.array(len(vshape) * [0, ])
    if padding is not None:
        pad[axes] = padding

    if isinstance(size, tuple):
        plan[axes] = size
    elif isinstance(size, str):
        size = 1000.0 * float(size)
        elsize = np.dtype(dtype).itemsize
        nelements = np.prod(vshape)
        dims = vshape[getmask(axes, len(vshape))]
        if size <= elsize:
            s = np.ones(len(axes))
        else:
            remsize = 1.0 * nelements * elsize
            s = []
            for (i, d) in enumerate(dims):
                # a zero-length axis gives nan / inf as in the reference (no warning)
                with np.errstate(divide="ignore", invalid="ignore"):
                    minsize = remsize / d
                if minsize >= size:
                    s.append(1)
                    remsize = minsize
                    continue
                else:
                    s.append(min(d, np.floor(size / minsize)))
                    s[i + 1:] = plan[i + 1:]
                    break
        plan[axes] = s
    else:
        raise ValueError("Chunk size not understood, must be tuple or int")

    return plan, pad


def check_plan(plan, padding, vshape):
    """The two validations of ChunkedArray._chunk (chunk.py:123-129)."""
    if any([x + y > z for x, y, z in zip(plan, padding, vshape)]):
        raise ValueError("Chunk sizes %s plus padding sizes %s cannot exceed value dimensions %s along any axis"
                         % (tuple(plan), tuple(padding), tuple(vshape)))
    if any([x > y for x, y in zip(padding, plan)]):
        raise ValueError("Padding sizes %s cannot exceed chunk sizes %s along any axis"
                         % (tuple(padding), tuple(plan)))


def getnumber(plan, shape):
    """Chunks per axis, ceil(d / size) (chunk.py:552-572)."""
    return [int(np.ceil(1.0 * d / size)) for size, d in zip(plan, shape)]


def getslices(plan, padding, shape):
    """Per-axis chunk slices (chunk.py:574-618).

    Chunk j < floor(d/s) spans [j*s - (j>0)*p, j*s + s + p) (the right pad is
    always added -- ``idx == nchunks`` at chunk.py:609 never holds -- and numpy
    clips it at d); a remainder chunk spans [floor(d/s)*s - p, d).
    """
    slices = []
    for size, pad, d in zip(plan, padding, shape):
        size, pad, d = int(size), int(pad), int(d)
        nchunks = d // size
        remainder = d % size
        start = 0
        end = 0
        dimslices = []
        for idx in range(nchunks):
            end = start + size
            left = start if idx == 0 else start - pad
            right = end + pad
            dimslices.append(slice(left, right, 1))
            start = end
        if remainder:
            dimslices.append(slice(end - pad, d, 1))
        slices.append(dimslices)
    return slices


def removepad_slices(idx, number, padding, axes=None):
    """Slices that strip padding from chunk ``idx`` (chunk.py:514-550).

    Left pad is removed unless the chunk is first, right pad unless last, only
    on ``axes`` with non-zero padding.  Returned as a tuple (the reference
    indexes with a list, which numpy >= 1.23 rejects).
    """
    if axes is None:
        axes = range(len(number))
    mask = len(number) * [False, ]
    for i in range(len(mask)):
        if i in axes and padding[i] != 0:
            mask[i] = True
    starts = [0 if (i == 0 or not m) else p for (i, m, p) in zip(idx, mask, padding)]
    stops = [None if (i == n - 1 or not m) else -p for (i, m, p, n) in zip(idx, mask, padding, number)]
    return tuple(slice(i1, i2) for (i1, i2) in zip(starts, stops))


# --------------------------------------------------------------------------
# chunk geometry -> strided copies for the pack / unpack kernels
# --------------------------------------------------------------------------

def axis_chunks(d, s, p):
    """Per-chunk (start, extent, core_offset, core_extent) along one axis.

    start/extent: the padded slice of getslices clipped to [0, d);
    core: the part removepad keeps (the chunk's own cells, chunk.py:546-550):
    [j*s, min(d, (j+1)*s)), at offset j*s - start inside the chunk.
    """
    out = []
    for j, slc in enumerate(getslices([s], [p], [d])[0]):
        start = max(0, slc.start)
        stop = min(d, slc.stop)
        core_lo = j * s
        core_hi = min(d, (j + 1) * s)
        out.append((start, stop - start, core_lo - start, core_hi - core_lo))
    return out


def _runs(chunks, s):
    """Group consecutive chunks into runs with equal extents and start step s.

    Returns a list of (j0, count, start0, extent, core_off, core_ext) whose
    members are chunks j0..j0+count-1 with start = start0 + (j-j0)*s.
    """
    runs = []
    for j, (st, ex, co, ce) in enumerate(chunks):
        if runs:
            j0, cnt, st0, ex0, co0, ce0 = runs[-1]
            if (ex, co, ce) == (ex0, co0, ce0) and st == st0 + cnt * s:
                runs[-1] = (j0, cnt + 1, st0, ex0, co0, ce0)
                continue
        runs.append((j, 1, st, ex, co, ce))
    return runs


class ChunkGeometry(object):
    """Packed layout of one record's chunks for a value shape, plan and padding.

    A record's chunks are stored back to back in C order of their chunk ids
    (the order of ``product(*slices)`` at chunk.py:132, which is also the
    sortByKey order of the chunk records); each chunk is a dense C-order box
    of its padded extent.  With E_a = sum_j extent_a[j], the record holds
    S = prod_a E_a elements and chunk j starts at
        off(j) = sum_a P_a[j_a] * prod_{b<a} extent_b[j_b] * prod_{b>a} E_b
    where P_a is the prefix sum of extents along axis a.
    """

    def __init__(self, vshape, plan, padding):
        self.vshape = tuple(int(x) for x in vshape)
        self.plan = tuple(int(x) for x in plan)
        self.padding = tuple(int(x) for x in padding)
        n = len(self.vshape)
        self.chunks = [axis_chunks(self.vshape[a], self.plan[a], self.padding[a]) for a in range(n)]
        self.nchunks = tuple(len(c) for c in self.chunks)
        self.E = [sum(c[1] for c in ch) for ch in self.chunks]
        self.P = []
        for ch in self.chunks:
            pre, acc = [], 0
            for c in ch:
                pre.append(acc)
                acc += c[1]
            self.P.append(pre)
        self.size = int(np.prod(self.E)) if n else 1
        self.runs = [_runs(self.chunks[a], self.plan[a]) for a in range(n)]

    def chunk_offset(self, j):
        n = len(self.vshape)
        off = 0
        for a in range(n):
            term = self.P[a][j[a]]
            for b in range(a):
                term *= self.chunks[b][j[b]][1]
            for b in range(a + 1, n):
                term *= self.E[b]
            off += term
        return off

    def chunk_shape(self, j):
        return tuple(self.chunks[a][j[a]][1] for a in range(len(self.vshape)))

    def chunk_ids(self):
        return list(product(*[range(k) for k in self.nchunks]))

    def combo_layout(self, combo):
        """Packed addressing of one combination of runs (one run per axis).

        Returns (base, cstr, inner): the packed offset of the combination's
        first chunk, the packed stride of the chunk index along each axis
        (linear inside a run: its chunks share one extent), and the C-order
        strides of a chunk box of the run extents.
        """
        n = len(self.vshape)
        ext = [r[3] for r in combo]
        base, cstr = 0, []
        for a, (j0, cnt, st0, ex, co, ce) in enumerate(combo):
            mult = 1
            for b in range(a):
                mult *= ext[b]
            for b in range(a + 1, n):
                mult *= self.E[b]
            base += self.P[a][j0] * mult
            cstr.append(ex * mult)
        inner = [1] * n
        for a in range(n - 2, -1, -1):
            inner[a] = inner[a + 1] * ext[a + 1]
        return base, cstr, inner

    def copies(self, unpack=False):
        """Strided copies (per record) between the dense record and the packed record.

        Each entry: (shape, dense_strides, packed_strides, dense_offset,
        packed_offset) in elements over the index space
        [count_0..count_{n-1}, extent_0..extent_{n-1}] of one run combination.
        pack copies padded boxes; unpack copies the cores (padding removed).
        """
        n = len(self.vshape)
        vstride = [1] * n
        for a in range(n - 2, -1, -1):
            vstride[a] = vstride[a + 1] * self.vshape[a + 1]
        out = []
        for combo in product(*self.runs):
            poff, cstr, inner = self.combo_layout(combo)
            shape = [r[1] for r in combo] + [(r[5] if unpack else r[3]) for r in combo]
            dstr = [self.plan[a] * vstride[a] for a in range(n)] + vstride
            pstr = cstr + inner
            doff = 0
            for a, (j0, cnt, st0, ex, co, ce) in enumerate(combo):
                doff += (st0 + (co if unpack else 0)) * vstride[a]
                if unpack:
                    poff += co * inner[a]
            out.append((shape, dstr, pstr, doff, poff))
        return out

    def record_map(self, unpack=False):
        """One record's layout change as an int32 gather map (bm_record_gather).

        pack:   map[p] = dense index of packed element p       (len = size)
        unpack: map[i] = packed index holding dense element i  (len = prod(vshape))
        Cached.
        """
        key = "_map_unpack" if unpack else "_map_pack"
        m = getattr(self, key, None)
        if m is None:
            rec = int(np.prod(self.vshape, dtype=np.int64)) if self.vshape else 1
            if unpack:
                m = copies_to_map([(sh, ps, ds, po, do) for sh, ds, ps, do, po in self.copies(True)], rec)
            else:
                m = copies_to_map(self.copies(False), self.size)
            setattr(self, key, m)
        return m

    def key(self):
        return (self.vshape, self.plan, self.padding)

    def is_identity(self):
        """True when the packed record IS the dense record: no padding growth
        and every chunk box lands at its own dense offset with dense strides
        (e.g. a plan that splits only the leading value axis, like the default
        chunk of C4's uint16 (1024, 1024) records, or a single chunk).  Packing
        and unpacking are then relabellings and move no bytes."""
        ident = getattr(self, "_identity", None)
        if ident is None:
            rec = int(np.prod(self.vshape, dtype=np.int64)) if self.vshape else 1
            ident = self.size == rec and all(
                doff == poff and all(n == 1 or a == b for n, a, b in zip(shape, dstr, pstr))
                for shape, dstr, pstr, doff, poff in self.copies(unpack=False))
            self._identity = ident
        return ident


def copies_to_map(copies, dst_len):
    """Run strided copies on index arrays: map[dst] = src, as int32.

    copies: (shape, src_strides, dst_strides, src_off, dst_off) in elements.
    Every destination element must be written exactly by the plan.
    """
    m = np.full(dst_len, -1, dtype=np.int64)
    for shape, ss, ds, so, do in copies:
        si = np.full((), so, dtype=np.int64)
        di = np.full((), do, dtype=np.int64)
        for n, a, b in zip(shape, ss, ds):
            ax = np.arange(n, dtype=np.int64)
            si = np.add.outer(si, ax * a)
            di = np.add.outer(di, ax * b)
        m[di.reshape(-1)] = si.reshape(-1)
    assert (m >= 0).all(), "copy plan does not cover the destination"
    return m.astype(np.int32)


def copies_to_scatter(copies, src_len, group=1, src_rec=None):
    """Strided copies over ``group`` consecutive source records (src_rec
    elements each, src_len = group * src_rec) -> a scatter plan
    (map_a, map_b) with

        dst(r_lo, p) = map_a[p] + r_lo * map_b[p]      (p < src_rec, r_lo < group)

    and map_a[p] = -1 where no copy reads element p (halos dropped by an
    unpack or a values_to_keys).  Returns None when the destinations are not
    affine in r_lo, or when an element is read more than once."""
    src_rec = src_len if src_rec is None else src_rec
    d = np.full(src_len, -1, dtype=np.int64)
    seen = np.zeros(src_len, dtype=np.int64)
    for shape, ss, ds, so, do in copies:
        si = np.full((), so, dtype=np.int64)
        di = np.full((), do, dtype=np.int64)
        for n, a, b in zip(shape, ss, ds):
            ax = np.arange(n, dtype=np.int64)
            si = np.add.outer(si, ax * a)
            di = np.add.outer(di, ax * b)
        si, di = si.reshape(-1), di.reshape(-1)
        if si.size and (si.min() < 0 or si.max() >= src_len):
            return None
        np.add.at(seen, si, 1)
        d[si] = di
    if (seen > 1).any():
        return None
    d = d.reshape(group, src_rec)
    used = d[0] >= 0
    if not (np.array_equal(d >= 0, np.broadcast_to(used, d.shape))):
        return None
    map_a = d[0].copy()
    map_b = np.zeros(src_rec, dtype=np.int64)
    if group > 1:
        map_b[used] = d[1, used] - d[0, used]
        want = map_a[None, :] + np.arange(group, dtype=np.int64)[:, None] * map_b[None, :]
        if not np.array_equal(d[:, used], want[:, used]):
            return None
    if map_a.max(initial=0) >= 2 ** 31 or (map_a[used] + (group - 1) * map_b[used]).max(initial=0) >= 2 ** 31:
        return None
    return map_a.astype(np.int32), map_b.astype(np.int32)


def scatter_vec(map_a, map_b, src_rec, gstride, es):
    """Elements per vector of a scatter plan: the widest v (v * es <= 16)
    such that every aligned group of v source elements is either wholly
    dropped or lands on v consecutive, v-aligned destinations with one r_lo
    step (map_b)."""
    v = max(1, 16 // es)
    while v > 1:
        if src_rec % v == 0 and gstride % v == 0:
            a = map_a.reshape(-1, v).astype(np.int64)
            b = map_b.reshape(-1, v).astype(np.int64)
            drop = a[:, 0] < 0
            ok = np.all((a < 0) == drop[:, None])
            keep = ~drop
            if ok and keep.any():
                ak, bk = a[keep], b[keep]
                ok = (np.all(ak == ak[:, :1] + np.arange(v)) and np.all(bk == bk[:, :1]) and
                      np.all(ak[:, 0] % v == 0) and np.all(bk[:, 0] % v == 0))
            if ok:
                return v
        v //= 2
    return 1


def scatter_to_runs(map_a, map_b, src_rec, gstride, es, max_runs=64, min_bytes=1024):
    """A scatter plan whose kept elements form a few long runs -> the runs
    table of bm_record_runs, or None: (runs, vec_bytes) with runs an int64
    array [s, len, a, m] x nruns in vec_bytes-byte vectors.  A run is a
    maximal stretch of source elements landing consecutively with one group
    step m.  Taken when there are at most ``max_runs`` runs of ``min_bytes``
    or more on average (C5 keys_to_values((2,)): 16 chunk boxes of 2.6-3.2 KB);
    short runs (unchunk's 128-B rows) keep the map scatter."""
    a = np.asarray(map_a, dtype=np.int64)
    b = np.asarray(map_b, dtype=np.int64)
    keep = a >= 0
    if not keep.any():
        return None
    cont = np.zeros(a.size, dtype=bool)
    cont[1:] = keep[1:] & keep[:-1] & (a[1:] == a[:-1] + 1) & (b[1:] == b[:-1])
    first = keep & ~cont
    starts = np.flatnonzero(first)
    if starts.size > max_runs:
        return None
    lens = np.bincount((np.cumsum(first) - 1)[keep], minlength=starts.size).astype(np.int64)
    if np.mean(lens) * es < min_bytes:
        return None
    runs = np.stack([starts, lens, a[starts], b[starts]], axis=1).astype(np.int64)
    vb = 16
    while vb > es and (np.any((runs * es) % vb) or (src_rec * es) % vb or (gstride * es) % vb):
        vb //= 2
    if vb < es or np.any((runs * es) % vb):
        return None
    return runs * es // vb, int(vb)


def scatter_runs_ok(map_a, map_b, es):
    """Whether a record scatter writes whole lines: its destination runs
    (consecutive kept elements landing consecutively) are all 128-B aligned
    multiples of 128 B, or 1 KiB long on average.  Short misaligned runs leave
    lines written piecewise by different waves: C5's values_to_keys as a
    scatter (144-160-B runs) ran 6.7-7.7 ms against 3.9-4.3 ms for the
    gather (profiles/r03zd_ab_scatter_c5.log)."""
    a = np.asarray(map_a, dtype=np.int64)
    b = np.asarray(map_b, dtype=np.int64)
    keep = a >= 0
    if not keep.any():
        return True
    cont = np.zeros(a.size, dtype=bool)
    cont[1:] = keep[1:] & keep[:-1] & (a[1:] == a[:-1] + 1) & (b[1:] == b[:-1])
    first = keep & ~cont
    starts = np.flatnonzero(first)
    lens = np.bincount((np.cumsum(first) - 1)[keep], minlength=starts.size)
    if np.mean(lens) * es >= 1024:
        return True
    return bool(np.all((a[starts] * es) % 128 == 0) and np.all((lens * es) % 128 == 0))


def _cstrides(shape):
    st = [1] * len(shape)
    for k in range(len(shape) - 2, -1, -1):
        st[k] = st[k + 1] * int(shape[k + 1])
    return st


def k2v_copies(old, new, kshape, kmask):
    """keys_to_values (chunk.py:202-289) as strided copies packed -> packed.

    old / new: ChunkGeometry of the value record before / after (new value
    axes = the moved keys, then the old value axes; moved keys chunked by
    ``size`` without padding, old value axes keep plan and padding).  kshape:
    this rank's key extents; kmask: moved keys.  A new chunk's box over the
    old value axes is exactly an old chunk's padded box (same slices), so
    every new chunk is a stack of old chunk boxes, one per moved-key index:
    each byte is read once from the old packing and written once.
    Entries: (shape, src_strides, dst_strides, src_off, dst_off) in elements.
    """
    ks_old = [k * old.size for k in _cstrides(kshape)]
    stat = [i for i in range(len(kshape)) if not kmask[i]]
    moved = [i for i in range(len(kshape)) if kmask[i]]
    ks_new = [k * new.size for k in _cstrides([kshape[i] for i in stat])]
    nk = len(moved)
    out = []
    for combo in product(*new.runs):
        nbase, ncstr, ninner = new.combo_layout(combo)
        obase, ocstr, oinner = old.combo_layout(combo[nk:])
        shape, ss, ds = [], [], []
        for t, i in enumerate(stat):
            shape.append(kshape[i]); ss.append(ks_old[i]); ds.append(ks_new[t])
        soff = obase
        for t, i in enumerate(moved):
            j0, cnt, st0, ex, co, ce = combo[t]
            shape.append(cnt); ss.append(new.plan[t] * ks_old[i]); ds.append(ncstr[t])
            soff += st0 * ks_old[i]
        for b in range(len(old.vshape)):
            shape.append(combo[nk + b][1]); ss.append(ocstr[b]); ds.append(ncstr[nk + b])
        for t, i in enumerate(moved):
            shape.append(combo[t][3]); ss.append(ks_old[i]); ds.append(ninner[t])
        for b in range(len(old.vshape)):
            shape.append(combo[nk + b][3]); ss.append(oinner[b]); ds.append(ninner[nk + b])
        out.append((shape, ss, ds, soff, nbase))
    return out


def v2k_copies(old, new, kshape, vmask):
    """values_to_keys (chunk.py:291-347) as strided copies packed -> packed.

    The moved value axes become trailing keys: a new record (key, b) takes,
    along each moved axis, row b of the core of the old chunk that owns b
    (removepad, chunk.py:305-312), and along the remaining value axes the
    old chunks' padded boxes unchanged (same plan and padding).  new: the
    ChunkGeometry over the remaining value axes.
    """
    nv = len(old.vshape)
    moved = [a for a in range(nv) if vmask[a]]
    rest = [a for a in range(nv) if not vmask[a]]
    mshape = [old.vshape[a] for a in moved]
    ks_old = [k * old.size for k in _cstrides(kshape)]
    nks = [k * new.size for k in _cstrides(list(kshape) + mshape)]
    nkey = len(kshape)
    out = []
    for combo in product(*old.runs):
        obase, ocstr, oinner = old.combo_layout(combo)
        nbase, ncstr, ninner = new.combo_layout(tuple(combo[a] for a in rest))
        shape, ss, ds = [], [], []
        for i in range(nkey):
            shape.append(kshape[i]); ss.append(ks_old[i]); ds.append(nks[i])
        soff, doff = obase, nbase
        for t, a in enumerate(moved):
            j0, cnt, st0, ex, co, ce = combo[a]
            shape.append(cnt); ss.append(ocstr[a]); ds.append(old.plan[a] * nks[nkey + t])
            soff += co * oinner[a]
            doff += j0 * old.plan[a] * nks[nkey + t]
        for t, a in enumerate(rest):
            shape.append(combo[a][1]); ss.append(ocstr[a]); ds.append(ncstr[t])
        for t, a in enumerate(moved):
            shape.append(combo[a][5]); ss.append(oinner[a]); ds.append(nks[nkey + t])
        for t, a in enumerate(rest):
            shape.append(combo[a][3]); ss.append(oinner[a]); ds.append(ninner[t])
        out.append((shape, ss, ds, soff, doff))
    return out


# --------------------------------------------------------------------------
# swap / transpose  (bolt/spark/array.py)
# --------------------------------------------------------------------------

def padded_strides(shape, P):
    """C-order element strides of ``shape`` with rows (the last axis) P elements
    apart: the layout of a row-padded array (array.py ROW_PITCH).  Only the
    leading stride depends on the rows' count, not on the leading extent, so
    the strides of the global shape serve every rank's slab."""
    nd = len(shape)
    st = [1] * nd
    if nd >= 2:
        st[nd - 2] = int(P)
        for k in range(nd - 3, -1, -1):
            st[k] = st[k + 1] * int(shape[k + 1])
    return st


def swap_perm(ndim, split, kaxes, vaxes):
    """Net permutation and split of BoltArraySpark.swap (array.py:716-763).

    chunk -> keys_to_values(K) -> values_to_keys(V) -> unchunk moves the key
    axes K (as a set: boolean masks, chunk.py:224/:293) to the front of the
    values and the value axes V to the end of the keys:
        P = [k not in K] + [split+v, v in V] + [k in K] + [split+v, v not in V]
        split' = split - #K + #V.
    """
    K = sorted(set(int(k) for k in kaxes))
    V = sorted(set(int(v) for v in vaxes))
    keys = list(range(split))
    vals = list(range(ndim - split))
    perm = ([k for k in keys if k not in K] + [split + v for v in V] + K +
            [split + v for v in vals if v not in V])
    return perm, split - len(K) + len(V)


def swap_shape(shape, split, kaxes, vaxes):
    """Shape and split BoltArraySpark.swap reports (array.py:758-763), or None
    where the reference's chain raises.

    The swap is chunk -> keys_to_values(K) -> values_to_keys(V + #K) ->
    unchunk, and three of those steps drop or add a unit value axis:
      * chunk of an all-key array appends a (1,) value axis (chunk.py:113-118);
      * keys_to_values of records whose values are (1,) drops that axis
        (chunk.py:284-287);
      * values_to_keys down to no value axes appends (1,) (chunk.py:342-345);
      * unchunk of records whose values are (1,) drops it (chunk.py:193-197).
    So a swap whose values end as one axis of length 1 (a (1, 5) swap((0,),
    (0,)) -> (5,)) or that moves keys next to a lone (1,) value axis loses
    that axis.  The bytes are x.transpose(swap_perm) either way: only unit
    axes differ.  None where the reference's chain raises IndexError
    (values_to_keys' mask indexes past the values left after the
    keys_to_values squeeze, chunk.py:293, or no longer fits records that
    squeeze cut short, chunk.py:329); the caller keeps numpy's shape there.
    """
    K = sorted(set(int(k) for k in kaxes))
    V = sorted(set(int(v) for v in vaxes))
    kshape = [int(d) for d in shape[:split]]
    vshape = [int(d) for d in shape[split:]] or [1]
    if K:
        squeeze = vshape == [1]
        if squeeze and any(kshape[k] == 1 for k in K):
            # numpy's squeeze drops the moved unit key's label axis from every
            # record too, and values_to_keys' mask no longer fits the records
            # (chunk.py:329, IndexError in the reference)
            return None
        vshape = [kshape[k] for k in K] + vshape
        kshape = [d for i, d in enumerate(kshape) if i not in K]
        if squeeze:
            vshape = vshape[:-1]
    Vn = [v + len(K) for v in V]
    if any(v >= len(vshape) for v in Vn):
        return None
    kshape = kshape + [vshape[v] for v in Vn]
    vshape = [d for i, d in enumerate(vshape) if i not in Vn] or [1]
    if vshape == [1]:
        vshape = []
    return tuple(kshape + vshape), len(kshape)


def transpose_split(p, split):
    """Decomposition of BoltArraySpark.transpose (array.py:788-806).

    Returns (swapping_keys, swapping_values relative to the values); the net
    result is x.transpose(p) with the split unchanged.
    """
    p = np.asarray(p)
    new_keys, new_values = p[:split], p[split:]
    swapping_keys = np.sort(new_values[new_values < split])
    swapping_values = np.sort(new_keys[new_keys >= split])
    return swapping_keys, swapping_values - split


# --------------------------------------------------------------------------
# reductions  (bolt/spark/array.py:_align, _stat, reduce)
# --------------------------------------------------------------------------

@functools.lru_cache(maxsize=1024)
def _reduce_layout(shape, axes):
    return _reduce_layout_impl(shape, axes)


def reduce_layout(shape, axes):
    """Cached front of _reduce_layout_impl (host planning stays off the critical path)."""
    return _reduce_layout(tuple(int(x) for x in shape), tuple(sorted(set(int(a) for a in axes))))


def _reduce_layout_impl(shape, axes):
    """Kernel layout for reducing ``axes`` of a C-contiguous array.

    Returns (perm, O, R, I): if ``perm`` is None the array is read in place
    as [O][R][I] (the reduced axes form one contiguous block once unit axes
    are ignored); otherwise it must first be permuted by ``perm`` (reduced
    axes first) and is then [1][R][I].  Outputs come out with the kept axes
    in ascending order, which is what _align's swap produces (array.py:85-115:
    reduced axes become the keys, kept axes the values in their order).
    """
    shape = tuple(int(x) for x in shape)
    red = set(int(a) for a in axes)
    labels = []
    for i, n in enumerate(shape):
        if n == 1:
            continue
        lab = 'R' if i in red else 'K'
        if labels and labels[-1][0] == lab:
            labels[-1][1] *= n
        else:
            labels.append([lab, n])
    nR = sum(1 for l in labels if l[0] == 'R')
    if nR == 0:
        O = int(np.prod([l[1] for l in labels])) if labels else 1
        return None, O, 1, 1
    if nR == 1:
        pos = [i for i, l in enumerate(labels) if l[0] == 'R'][0]
        O = int(np.prod([l[1] for l in labels[:pos]])) if pos else 1
        R = labels[pos][1]
        I = int(np.prod([l[1] for l in labels[pos + 1:]])) if pos + 1 < len(labels) else 1
        return None, O, R, I
    perm = [i for i in range(len(shape)) if i in red] + [i for i in range(len(shape)) if i not in red]
    R = int(np.prod([shape[i] for i in range(len(shape)) if i in red]))
    I = int(np.prod([shape[i] for i in range(len(shape)) if i not in red]))
    return perm, 1, R, I


def stat_dtype(dtype, rec_shape):
    return _stat_dtype(np.dtype(dtype), tuple(int(x) for x in rec_shape))


@functools.lru_cache(maxsize=256)
def _stat_dtype(dtype, rec_shape):
    """Result dtype of a StatCounter statistic (statcounter.py:51-59).

    The counter starts at mu = 0.0 (a Python float) and every statistic is
    built from ``value - mu``, so the result dtype is that of
    ``record - 0.0`` under the host numpy: float32 stays float32, integers
    and bool become float64; a 0-d record follows the host numpy's scalar
    casting rules.  Evaluated, not tabulated, so it matches the reference
    under whatever numpy is installed.
    """
    rec = np.zeros(tuple(rec_shape), dtype=dtype)
    if len(rec_shape) == 0:
        rec = rec[()]
    return np.asarray(rec - 0.0).dtype
