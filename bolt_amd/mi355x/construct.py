"""ConstructMI355X: constructors of the 'mi355x' mode.

Mirrors ConstructSpark (bolt/spark/construct.py:10-222) with ``context`` an
``MI355XContext`` and ``npartitions`` the number of GPU shards.
"""
import numpy as np

from bolt_amd.construct import ConstructBase


class ConstructMI355X(ConstructBase):

    @staticmethod
    def array(a, context=None, axis=(0,), dtype=None, npartitions=None):
        """Create an MI355X bolt array from a local array (spark/construct.py:12-70).

        ``a`` is array-like (the full array, present on every rank) or a
        BoltArrayMI355X.  ``axis`` selects the key axes; records are sharded
        over the ranks of ``context`` along the first key axis.  Semantics,
        including the reference's handling of non-leading key axes (the data
        is transposed to key-major order but the array keeps the original
        shape, spark/construct.py:48-67), follow the reference exactly.
        """
        from bolt_amd.mi355x.array import BoltArrayMI355X
        from bolt_amd.mi355x.context import MI355XContext
        if isinstance(a, BoltArrayMI355X):
            a = a.toarray()
        if context is None:
            context = MI355XContext.default()
        if dtype is None:
            arry = np.asarray(a)
            dtype = arry.dtype
        else:
            arry = np.asarray(a, dtype)
        shape = arry.shape
        ndim = len(shape)

        axes = ConstructMI355X._format_axes(axis, arry.shape)
        key_axes = list(axes)
        value_axes = [i for i in range(ndim) if i not in axes]
        permutation = key_axes + value_axes
        split = len(axes)

        if split < 1:
            raise ValueError("split axis must be greater than 0, got %g" % split)
        if split > len(shape):
            raise ValueError("split axis must not exceed number of axes %g, got %g" % (ndim, split))

        return BoltArrayMI355X._ingest(arry, permutation, shape, split, np.dtype(dtype),
                                       context, npartitions)

    @staticmethod
    def ones(shape, context=None, axis=(0,), dtype=np.float64, npartitions=None):
        """MI355X bolt array of ones (spark/construct.py:72-102, :207-222)."""
        return ConstructMI355X._wrap(1, shape, context, axis, dtype, npartitions)

    @staticmethod
    def zeros(shape, context=None, axis=(0,), dtype=np.float64, npartitions=None):
        """MI355X bolt array of zeros (spark/construct.py:104-134, :207-222)."""
        return ConstructMI355X._wrap(0, shape, context, axis, dtype, npartitions)

    @staticmethod
    def fromshards(shard, shape, context=None, split=1, dtype=None, npartitions=None):
        """Wrap this rank's shard (rows of the leading key axis) without a host copy.

        ``shard`` is a numpy array or a device tensor holding this rank's slab
        of the global array ``shape`` (C order, leading axis sharded as
        MI355XContext.bounds says).  Not in the reference: it is how data that
        already lives in HBM (or is generated there) enters the backend.
        """
        from bolt_amd.mi355x.array import BoltArrayMI355X
        from bolt_amd.mi355x.context import MI355XContext
        if context is None:
            context = MI355XContext.default()
        return BoltArrayMI355X._from_shard(shard, tuple(int(s) for s in shape), int(split),
                                           dtype, context, npartitions)

    @staticmethod
    def concatenate(arrays, axis=0):
        """Join two arrays, at least one of them an mi355x array (spark/construct.py:136-167)."""
        from bolt_amd.mi355x.array import BoltArrayMI355X
        if not isinstance(arrays, tuple):
            raise ValueError("data type not understood")
        if not len(arrays) == 2:
            raise NotImplementedError("spark concatenation only supports two arrays")
        first, second = arrays
        if isinstance(first, BoltArrayMI355X):
            return first.concatenate(second, axis)
        elif isinstance(second, BoltArrayMI355X):
            first = ConstructMI355X.array(first, second.context)
            return first.concatenate(second, axis)
        else:
            raise ValueError("at least one array must be a spark bolt array")

    @staticmethod
    def _argcheck(*args, **kwargs):
        """True when an argument is an MI355XContext or BoltArrayMI355X (spark/construct.py:169-190)."""
        from bolt_amd.mi355x.array import BoltArrayMI355X
        from bolt_amd.mi355x.context import MI355XContext
        cond1 = any([isinstance(arg, MI355XContext) for arg in args])
        cond2 = isinstance(kwargs.get('context', None), MI355XContext)
        cond3 = any([isinstance(arg, BoltArrayMI355X) for arg in args])
        cond4 = any([any([isinstance(sub, BoltArrayMI355X) for sub in arg])
                     if isinstance(arg, (tuple, list)) else False for arg in args])
        return cond1 or cond2 or cond3 or cond4

    @staticmethod
    def _format_axes(axes, shape):
        """Normalise key axes; ValueError when out of range (spark/construct.py:192-205)."""
        if isinstance(axes, int):
            axes = (axes,)
        elif isinstance(axes, list) or hasattr(axes, '__iter__'):
            axes = tuple(axes)
        if not isinstance(axes, tuple):
            raise ValueError("axes argument %s in the constructor not specified correctly" % str(axes))
        if min(axes) < 0 or max(axes) > len(shape) - 1:
            raise ValueError("invalid key axes %s given shape %s" % (str(axes), str(shape)))
        return axes

    @staticmethod
    def _wrap(value, shape, context=None, axis=(0,), dtype=None, npartitions=None):
        """Constant-filled construction (spark/construct.py:207-222): the shape is kept as given."""
        from bolt_amd.mi355x.array import BoltArrayMI355X
        from bolt_amd.mi355x.context import MI355XContext
        if context is None:
            context = MI355XContext.default()
        if isinstance(shape, int):
            shape = (shape,)
        shape = tuple(int(s) for s in shape)
        axes = ConstructMI355X._format_axes(axis, shape)
        split = len(axes)
        return BoltArrayMI355X._filled(value, shape, split, np.dtype(dtype), context, npartitions)
