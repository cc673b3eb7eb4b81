"""Keys / Values views of a BoltArrayMI355X (bolt/spark/shapes.py).

transpose permutes only the key axes or only the value axes (one permute
kernel; a key permutation that moves the leading key axis exchanges records
between GPUs).  reshape is free on the dense C-order layout: it keeps the byte
sequence and only renames the shape (shapes.py:40-64, :111-134), re-slabbing
across GPUs when the leading key extent changes.
"""
from bolt_amd.mi355x.dist import redistribute_rows
from bolt_amd.utils import argpack, istransposeable, isreshapeable

import numpy as np


class Shapes(object):

    @property
    def shape(self):
        raise NotImplementedError

    @property
    def ndim(self):
        return len(self.shape)


class Keys(Shapes):

    def __init__(self, barray):
        self._barray = barray

    @property
    def shape(self):
        return self._barray.shape[:self._barray.split]

    def reshape(self, *shape):
        """Reshape the keys only (shapes.py:40-64)."""
        new = argpack(shape)
        old = self.shape
        isreshapeable(new, old)
        if new == old:
            return self._barray
        b = self._barray
        newshape = tuple(int(x) for x in new) + b.values.shape
        return _relabel(b, newshape, len(new))

    def transpose(self, *axes):
        """Permute the key axes (shapes.py:66-89)."""
        new = argpack(axes)
        old = range(self.ndim)
        istransposeable(new, old)
        if new == tuple(old):
            return self._barray
        b = self._barray
        perm = [int(i) for i in new] + list(range(b.split, b.ndim))
        return b._permute(perm, b.split)

    def __str__(self):
        return "BoltArray Keys\nshape: %s" % str(self.shape)

    def __repr__(self):
        return str(self)


class Values(Shapes):

    def __init__(self, barray):
        self._barray = barray

    @property
    def shape(self):
        return self._barray.shape[self._barray.split:]

    def reshape(self, *shape):
        """Reshape the values only (shapes.py:111-134)."""
        new = argpack(shape)
        old = self.shape
        isreshapeable(new, old)
        if new == old:
            return self._barray
        b = self._barray
        newshape = b.keys.shape + tuple(int(x) for x in new)
        return _relabel(b, newshape, b.split)

    def transpose(self, *axes):
        """Permute the value axes (shapes.py:136-159)."""
        new = argpack(axes)
        old = range(self.ndim)
        istransposeable(new, old)
        if new == tuple(old):
            return self._barray
        b = self._barray
        perm = list(range(b.split)) + [b.split + int(i) for i in new]
        return b._permute(perm, b.split)

    def __str__(self):
        return "BoltArray Values\nshape: %s" % str(self.shape)

    def __repr__(self):
        return str(self)


def _relabel(b, newshape, split):
    """``b``'s records under ``newshape`` (same C order).  A row-padded array
    whose last axis keeps its length keeps its padded rows (across GPUs only
    while the slabs stay put)."""
    d = b.__dict__
    if "_pbuf" in d and len(newshape) >= 2 and newshape[-1] == b.shape[-1] and \
            (b.context.world_size == 1 or newshape[0] == b.shape[0]):
        return b._derive_padded(d["_pbuf"], d["_pitch"], newshape, split)
    return b._like(_reslab(b, newshape), newshape, split)


def _reslab(b, newshape):
    """Same bytes under ``newshape``; re-slab across GPUs if the leading extent changes."""
    es = b.dtype.itemsize
    old_row = int(np.prod(b.shape[1:], dtype=np.int64)) * es
    new_row = int(np.prod(newshape[1:], dtype=np.int64)) * es
    if b.context.world_size == 1 or newshape[0] == b.shape[0]:
        return b._data
    return redistribute_rows(b.context, b._data, b.shape[0], old_row, newshape[0], new_row)
