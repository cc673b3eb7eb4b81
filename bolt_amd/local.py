"""Host-side ('local' mode) array type returned by the MI355X statistics.

The reference returns statistics as ``BoltArrayLocal`` -- a numpy ndarray
subclass -- or as a numpy scalar via ``toscalar`` (bolt/spark/array.py:331,
bolt/local/array.py:8-20, :194-202).  This restates the part of it the hot
path needs, plus the numpy-backed ``ConstructLocal`` the factory routes to by
default (bolt/local/construct.py:7-83).  Inside bolt itself
bolt's own BoltArrayLocal takes this role.
"""
import numpy as np

from bolt_amd.construct import ConstructBase


class BoltArrayLocal(np.ndarray):
    """numpy ndarray carrying ``mode == 'local'`` (bolt/local/array.py:8-20)."""

    def __new__(cls, array):
        obj = np.asarray(array).view(cls)
        obj._mode = 'local'
        return obj

    def __array_finalize__(self, obj):
        if obj is None:
            return
        self._mode = getattr(obj, '_mode', 'local')

    def __array_wrap__(self, obj, context=None, return_scalar=False):
        if obj.shape == ():
            return obj[()]
        return np.ndarray.__array_wrap__(self, obj, context, return_scalar)

    @property
    def mode(self):
        return 'local'

    def toarray(self):
        return np.asarray(self)

    def toscalar(self):
        """The single element of a 0-d array, else self (bolt/local/array.py:194-202)."""
        if self.shape == ():
            return self.toarray().reshape(1)[0]
        return self

class ConstructLocal(ConstructBase):
    """numpy-backed constructors (bolt/local/construct.py:9-83)."""

    @staticmethod
    def array(a, dtype=None, order='C'):
        return BoltArrayLocal(np.asarray(a, dtype, order))

    @staticmethod
    def ones(shape, dtype=np.float64, order='C'):
        return BoltArrayLocal(np.ones(shape, dtype, order))

    @staticmethod
    def zeros(shape, dtype=np.float64, order='C'):
        return BoltArrayLocal(np.zeros(shape, dtype, order))

    @staticmethod
    def concatenate(arrays, axis=0):
        """numpy.concatenate of a tuple of arrays (bolt/local/construct.py:85-105)."""
        if not isinstance(arrays, tuple):
            raise ValueError("data type not understood")
        arrays = tuple([np.asarray(a) for a in arrays])
        return BoltArrayLocal(np.concatenate(arrays, axis))
