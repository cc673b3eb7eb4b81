"""MI355XContext: the execution context of the 'mi355x' mode.

Plays the role SparkContext plays for the spark mode
(bolt/spark/construct.py:24-25, :69): it names where records live.  One
process drives one GPU; with torch.distributed initialised (backend 'nccl' =
RCCL over xGMI on MI355X) the records of every array are sharded over the
ranks along the leading key axis, in contiguous slabs as numpy.array_split
would cut them (the analogue of parallelize's contiguous partitions).
"""
import os

import numpy as np


class MI355XContext(object):

    _default = None

    def __init__(self, device=None, group=None):
        import torch
        import torch.distributed as dist
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        if self.distributed:
            self.rank = dist.get_rank(group)
            self.world_size = dist.get_world_size(group)
        else:
            self.rank, self.world_size = 0, 1
        if device is None:
            if torch.cuda.is_available():
                device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        # fail loudly here when there is no kernel backend for the device
        # (no HIP device / library): the mode has no CPU fallback
        from bolt_amd.mi355x._ops import backend_for
        self.backend = backend_for(self.device)

    @classmethod
    def default(cls):
        """A per-process context (created on first use)."""
        if cls._default is None:
            cls._default = cls()
        return cls._default

    @property
    def defaultParallelism(self):
        return self.world_size

    def bounds(self, n):
        """[(lo, hi)] of every rank's slab of an axis of length n (array_split order)."""
        g = self.world_size
        base, extra = divmod(int(n), g)
        out, lo = [], 0
        for r in range(g):
            hi = lo + base + (1 if r < extra else 0)
            out.append((lo, hi))
            lo = hi
        return out

    def local_bounds(self, n):
        return self.bounds(n)[self.rank]

    def __repr__(self):
        return "MI355XContext(device=%s, rank=%d, world_size=%d)" % (self.device, self.rank, self.world_size)


def local_shape(ctx, shape):
    if len(shape) == 0:  # a 0-d array (everything squeezed out) lives on rank 0
        return () if ctx.rank == 0 else (0,)
    lo, hi = ctx.local_bounds(shape[0])
    return (hi - lo,) + tuple(shape[1:])


def contiguous_strides(shape):
    st = [1] * len(shape)
    for k in range(len(shape) - 2, -1, -1):
        st[k] = st[k + 1] * int(shape[k + 1])
    return st


def nbytes(shape, dtype):
    return int(np.prod(shape, dtype=np.int64)) * np.dtype(dtype).itemsize if len(shape) else np.dtype(dtype).itemsize
