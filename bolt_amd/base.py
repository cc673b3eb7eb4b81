"""Stand-in for bolt's ``bolt.base`` where the reference is not installed.

BoltArrayMI355X needs only the metadata protocol of bolt's abstract array:
``_mode``, ``_metadata`` and ``__finalize__`` (bolt/base.py:1-13); it
implements the shape / statistics / shaping surface itself.  Inside bolt this
module is dropped and ``bolt.base`` takes its place (INTEGRATION.md section 2;
``tests/test_reference_dropin.py`` runs the mode that way against the
reference's own test suite).
"""


class BoltArray(object):

    _mode = None
    _metadata = {}

    def __finalize__(self, other):
        """Take over metadata that is still at its class default (bolt/base.py:6-13)."""
        if isinstance(other, BoltArray):
            for name, default in self._metadata.items():
                theirs = getattr(other, name, None)
                if theirs is not default and getattr(self, name, None) is default:
                    object.__setattr__(self, name, theirs)
        return self

    @property
    def mode(self):
        return self._mode
