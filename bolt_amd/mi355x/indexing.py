"""Indexing of the mi355x mode: BoltArraySpark.__getitem__ (bolt/spark/array.py:480-676).

Every selection is one kernel on the dense layout, plus at most one
all-to-all when rows move between GPUs:

  basic     ints and slices (array.py:480-512): x[s_0, .., s_n] is a strided
            copy (negative steps read with negative strides) -- dist.select_sharded.
  mixed     one index list on one axis amid slices (array.py:561-593):
            x.take(idx, axis) with bm_gather_rows, then the basic selection
            of the other axes, composed exactly as the reference composes it.
  advanced  one list per axis (array.py:514-559): a point gather with
            bm_gather_rows (row = one element), in the reference's record
            order (below).

Result order of the advanced path.  The reference filters the records whose
key is listed, visits them in key order, expands each into the value
positions grouped under its key (itertools.groupby over the listed
positions: consecutive runs, a later run of the same key replaces an
earlier one) and numbers the results with zipWithIndex.  For sorted,
duplicate-free key lists that is numpy's fancy indexing; otherwise the order
(and count) differ from numpy, and this backend reproduces the reference's
order.  Where the reference's record count disagrees with the shape it
declares (its array cannot be collected) this backend raises ValueError.
"""
import numpy as np

from bolt_amd.mi355x.dist import all_to_all_bytes, _empty, _unit


def normalize(index, shape, split):
    """The reference's index normalisation and bounds checks (array.py:629-659).

    Returns (index list, int_locs, kind) with slices slicified and list
    indices as ndarrays (negatives wrapped); kind is 'basic' / 'advanced' /
    'mixed'.  Every returned slice selects indices inside its axis (below).
    """
    from bolt_amd.utils import slicify
    if isinstance(index, tuple):
        index = list(index)
    else:
        index = [index]
    int_locs = [i for i, x in enumerate(index) if isinstance(x, int)]
    ndim = len(shape)
    if len(index) > ndim:
        raise ValueError("Too many indices for array")
    if not all(isinstance(i, (slice, int, list, tuple, np.ndarray)) for i in index):
        raise ValueError("Each index must either be a slice, int, list, set, or ndarray")
    index += [slice(0, None, None)] * (ndim - len(index))
    for n, idx in enumerate(index):
        size = shape[n]
        if isinstance(idx, (slice, int)):
            slc = slicify(idx, size)
            if slc.step > 0:
                minval, maxval = slc.start, slc.stop
            else:
                minval, maxval = slc.stop, slc.start
            if minval > size - 1 or maxval < 1 or minval >= maxval:
                raise ValueError("Index {} in dimension {} with shape {} would "
                                 "produce an empty dimension".format(idx, n, size))
            if slc.step < 0 and slc.start == size:
                slc = _past_end(idx, n, size, slc, n < split)
            index[n] = slc
        else:
            adjusted = np.asarray(idx)
            neg = adjusted < 0
            if neg.any():  # copy only when negatives wrap
                adjusted = np.array(adjusted)
                adjusted[neg] += size
            if adjusted.size and (adjusted.min() < 0 or adjusted.max() > size - 1):
                raise ValueError("Index {} out of bounds in dimension {} with "
                                 "shape {}".format(idx, n, size))
            index[n] = adjusted
    if all(isinstance(i, slice) for i in index):
        kind = 'basic'
    elif all(isinstance(i, np.ndarray) for i in index):
        kind = 'advanced'
    elif sum(isinstance(i, np.ndarray) for i in index) == 1:
        kind = 'mixed'
    else:
        raise NotImplementedError("When mixing basic indexing (slices and int) with "
                                  "with advanced indexing (lists, tuples, and ndarrays), "
                                  "can only have a single advanced index")
    return index, int_locs, kind


def _past_end(idx, n, size, slc, on_key):
    """A negative-step slice that slicify leaves starting AT the end (it clamps
    only start > dim, bolt/utils.py:136).  The reference's shape counts that
    phantom element (array.py:510).  On a key axis no record carries it, so the
    records fall short of the shape and the array cannot be collected: refused.
    On a value axis numpy slices each record (array.py:505-506) from dim - 1:
    the array is numpy's selection when the two counts agree, uncollectable
    otherwise (refused).  Returns the equivalent in-bounds slice."""
    stop = None if slc.stop == -1 else slc.stop
    declared = int(np.ceil((slc.stop - slc.start) / float(slc.step)))
    if not on_key and len(range(size)[slice(slc.start, stop, slc.step)]) == declared:
        return slice(size - 1, slc.stop, slc.step)
    raise ValueError("Index {} in dimension {} with shape {} starts past the end with a negative "
                     "step: the reference's array would hold fewer elements than its shape"
                     .format(idx, n, size))


def _listify(lst, dim):
    """bolt/utils.py:85-103: integer indices, bounded by dim, flattened."""
    if len(lst) and lst.dtype != int:  # every element of an ndarray shares its dtype
        raise ValueError("indices must be integers")
    if len(lst) and np.asarray(lst).max() >= dim:
        raise ValueError("indices out of bounds for axis with size %s" % dim)
    return lst.ravel()


def advanced_points(index, shape, split):
    """Flat element offsets of the advanced selection, in the reference's order
    (array.py:514-559), and the result shape (split = its ndim).

    Positions are grouped in runs of equal key (itertools.groupby); the last
    run of each key wins (a dict keyed by key); kept runs are emitted in key
    order, each in listed order; without value axes each key yields one record.
    """
    index = [np.asarray(i) for i in index]
    ishape = index[0].shape
    if not all(i.shape == ishape for i in index):
        raise ValueError("shape mismatch: indexing arrays could not be broadcast "
                         "together with shapes " + ("%s " * len(shape)) % tuple(i.shape for i in index))
    index = [_listify(i, d).astype(np.int64, copy=False) for i, d in zip(index, shape)]
    n = int(np.prod(ishape, dtype=np.int64))
    kshape, vshape = tuple(shape[:split]), tuple(shape[split:])
    K = np.ravel_multi_index(index[:split], kshape) if split else np.zeros(n, np.int64)
    V = np.ravel_multi_index(index[split:], vshape) if vshape else np.zeros(n, np.int64)
    vsize = int(np.prod(vshape, dtype=np.int64))
    if n == 0:
        pts = np.zeros(0, np.int64)
    elif vshape and bool(np.all(K[1:] >= K[:-1])):
        # keys listed in order: one run per key, already in key order -- the
        # reference's grouping is the identity (numpy's fancy indexing)
        pts = K * vsize + V
    else:
        starts = np.flatnonzero(np.r_[True, K[1:] != K[:-1]])
        ends = np.r_[starts[1:], n]
        rk = K[starts]
        order = np.argsort(rk, kind="stable")
        last = np.r_[rk[order][1:] != rk[order][:-1], True]
        kept = order[last]
        if vshape:
            lens = ends[kept] - starts[kept]
            first = np.repeat(starts[kept] - np.r_[0, np.cumsum(lens)[:-1]], lens)
            pos = first + np.arange(int(lens.sum()), dtype=np.int64)
            pts = K[pos] * vsize + V[pos]
        else:
            pts = rk[kept]
    if pts.size != n:
        raise ValueError("the reference's advanced selection yields %d records for shape %s "
                         "(repeated key positions): not representable" % (pts.size, str(ishape)))
    return pts.astype(np.int64), tuple(int(s) for s in ishape)


def mixed_take(index, shape, split):
    """(loc, idx) of the single list index (array.py:561-593)."""
    loc = [i for i, x in enumerate(index) if isinstance(x, np.ndarray)][0]
    idx = np.asarray(index[loc])
    if idx.ndim != 1 or idx.dtype == object:  # a nested sequence (the reference checks idx[0])
        raise ValueError("When mixing basic and advanced indexing, "
                         "advanced index must be one-dimensional")
    if idx.dtype.kind not in "iu":
        raise ValueError("indices must be integers")
    idx = idx.astype(np.int64)
    if loc < split and len(np.unique(idx)) != len(idx):
        # the reference renumbers key records to the FIRST position of their
        # value (list.index): a repeated key leaves holes it cannot collect
        raise ValueError("repeated index %s on a key axis is not representable" % list(idx))
    return loc, idx


def gather_units_sharded(ctx, backend, data, nrows, unit_bytes, units_per_row, src_units, out_rows,
                         out_units_per_row):
    """This rank's slab of out[j] = in[src_units[j]] for sharded byte arrays.

    The input is ``nrows`` leading-axis rows of ``units_per_row`` units of
    ``unit_bytes`` each, sharded by rows; the output is ``out_rows`` rows of
    ``out_units_per_row`` units, sharded the same way.  One gather kernel on one
    GPU; across GPUs: gather what this rank owns per destination, one
    all-to-all, one gather into place.
    """
    src_units = np.asarray(src_units, dtype=np.int64)
    in_b = ctx.bounds(nrows)
    out_b = ctx.bounds(out_rows)
    r = ctx.rank
    lo, hi = out_b[r]
    mlo, mhi = in_b[r]
    out = _empty((hi - lo) * out_units_per_row * unit_bytes, data.device)
    if ctx.world_size == 1:
        backend.gather_rows(data, 0, out, 0, 1, nrows * units_per_row, unit_bytes, src_units)
        return out
    row_lo = np.array([b[0] for b in in_b] + [nrows], dtype=np.int64)
    owner = np.searchsorted(row_lo, src_units // units_per_row, side="right") - 1
    dest_of = np.arange(src_units.size, dtype=np.int64) // out_units_per_row
    dest_rank = np.searchsorted(np.array([b[0] for b in out_b] + [out_rows]), dest_of, side="right") - 1
    # send: units this rank owns, grouped by destination rank, in output order
    mine = np.nonzero(owner == r)[0]
    order = mine[np.argsort(dest_rank[mine], kind="stable")]
    send_counts = np.bincount(dest_rank[mine], minlength=ctx.world_size)
    send = _empty(order.size * unit_bytes, data.device)
    if order.size:
        backend.gather_rows(data, 0, send, 0, 1, (mhi - mlo) * units_per_row, unit_bytes,
                            src_units[order] - mlo * units_per_row)
    # receive: my output units, grouped by owning rank, each group in output order
    js = np.arange(lo * out_units_per_row, hi * out_units_per_row, dtype=np.int64)
    recv_order = js[np.argsort(owner[js], kind="stable")]
    recv_counts = np.bincount(owner[js], minlength=ctx.world_size) if js.size else np.zeros(ctx.world_size, int)
    u = _unit(unit_bytes)
    recv = all_to_all_bytes(ctx, send, [int(c) * unit_bytes for c in send_counts],
                            [int(c) * unit_bytes for c in recv_counts], u)
    if js.size:
        pos = np.empty(js.size, dtype=np.int64)
        pos[recv_order - js[0]] = np.arange(js.size, dtype=np.int64)
        backend.gather_rows(recv, 0, out, 0, 1, js.size, unit_bytes, pos)
    return out


def take_sharded(ctx, backend, data, shape, es, loc, idx):
    """This rank's slab of x.take(idx, axis=loc) (axis 0 moves rows across GPUs)."""
    shape = tuple(int(s) for s in shape)
    row = int(np.prod(shape[loc + 1:], dtype=np.int64)) * es
    if loc == 0:
        return gather_units_sharded(ctx, backend, data, shape[0], row, 1, idx, len(idx), 1)
    lo, hi = ctx.local_bounds(shape[0])
    n_outer = (hi - lo) * int(np.prod(shape[1:loc], dtype=np.int64))
    out = _empty(n_outer * len(idx) * row, data.device)
    if n_outer and row:
        backend.gather_rows(data, 0, out, 0, n_outer, shape[loc], row, idx)
    return out
