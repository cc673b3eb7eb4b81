"""bolt_amd -- MI355X (gfx950) execution backend for bolt's Spark-mode hot path.

Registers the 'mi355x' mode beside 'local' (bolt/factory.py:4-7):

    import bolt_amd as bolt
    ctx = bolt.MI355XContext()
    b = bolt.array(x, ctx, axis=(0,))          # or bolt.array(x, mode='mi355x')
    b.swap((0,), (0, 1)).mean(axis=2)

Hot path (HIP kernels in libbolt_mi355x.so, see include/bolt_mi355x.h):
ChunkedArray chunk/unchunk/keys_to_values/values_to_keys, swap, transpose,
sum/mean/var/std.  Multi-GPU: one process per GPU, records sharded along the
leading key axis, RCCL all-to-all for swaps and all_gather for statistics.
"""
from bolt_amd.factory import array, ones, zeros, concatenate  # noqa: F401
from bolt_amd.mi355x.context import MI355XContext  # noqa: F401
from bolt_amd.mi355x.construct import ConstructMI355X  # noqa: F401

__version__ = '0.7.1+mi355x.1'


def __getattr__(name):
    # lazy: importing the array type pulls torch
    if name == 'BoltArrayMI355X':
        from bolt_amd.mi355x.array import BoltArrayMI355X
        return BoltArrayMI355X
    if name == 'ChunkedArrayMI355X':
        from bolt_amd.mi355x.chunk import ChunkedArrayMI355X
        return ChunkedArrayMI355X
    raise AttributeError(name)
