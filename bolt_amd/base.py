"""The bolt array interface the MI355X backend implements.

Restates the abstract ``BoltArray`` of the reference (bolt/base.py:1-158):
``_mode``, ``_metadata`` with ``__finalize__`` (bolt/base.py:6-13) and the
shape/statistics/shaping surface.  Kept local so the package runs where the
reference is not installed (the GPU box); INTEGRATION.md shows the one-line
change that makes BoltArrayMI355X a subclass of bolt.base.BoltArray instead.
"""


class BoltArray(object):

    _mode = None
    _metadata = {}

    def __finalize__(self, other):
        """Copy metadata still at its class default from ``other`` (bolt/base.py:6-13)."""
        if isinstance(other, BoltArray):
            for name in self._metadata:
                other_attr = getattr(other, name, None)
                if (other_attr is not self._metadata[name]) \
                        and (getattr(self, name, None) is self._metadata[name]):
                    object.__setattr__(self, name, other_attr)
        return self

    @property
    def mode(self):
        return self._mode

    @property
    def shape(self):
        raise NotImplementedError

    @property
    def size(self):
        raise NotImplementedError

    @property
    def ndim(self):
        raise NotImplementedError

    @property
    def dtype(self):
        raise NotImplementedError

    def sum(self, axis):
        raise NotImplementedError

    def mean(self, axis):
        raise NotImplementedError

    def var(self, axis):
        raise NotImplementedError

    def std(self, axis):
        raise NotImplementedError

    def transpose(self, axis):
        raise NotImplementedError

    @property
    def T(self):
        raise NotImplementedError

    def swapaxes(self, axis1, axis2):
        raise NotImplementedError

    def __repr__(self):
        s = "BoltArray\n"
        s += "mode: %s\n" % self._mode
        s += "shape: %s\n" % str(self.shape)
        return s
