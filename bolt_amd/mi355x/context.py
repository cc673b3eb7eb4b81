"""MI355XContext: the execution context of the 'mi355x' mode.

Plays the role SparkContext plays for the spark mode
(bolt/spark/construct.py:24-25, :69): it names where records live.  One
process drives one GPU; with torch.distributed initialised the records of
every array are sharded over the ranks along the leading key axis, in
contiguous slabs as numpy.array_split would cut them (the analogue of
parallelize's contiguous partitions).

Transport between ranks (``transport``) is chosen by the kernel backend, not
by the process group.  The production HIP backend uses "rccl": the context
opens its own RCCL communicator in libbolt_mi355x (bm_comm_init; the id
travels through the group's rendezvous store) and every device byte between
GPUs goes through it; torch.distributed carries the rendezvous and host-side
metadata only.  The group must have an nccl device backend ('nccl' or
'cpu:gloo,cuda:nccl'; with the latter torch never builds an RCCL
communicator of its own).  Only the test executors registered through
_ops.register_backend use torch.distributed collectives ("torch", "host").

Every RCCL wait is bounded by ``comm_timeout`` seconds
(BOLT_AMD_COMM_TIMEOUT, default 600): a peer that dies or posts a mismatched
exchange raises _lib.BoltCommError and aborts the communicator.
"""
import os

import numpy as np


class MI355XContext(object):

    _default = None
    _ncomm = {}  # communicators created by this process, per rank set (names their rendezvous keys)

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
        self.comm = None
        self.comm_stream = None
        self.comm_timeout = float(os.environ.get("BOLT_AMD_COMM_TIMEOUT", "600"))
        self.transport = None
        if self.world_size > 1:
            self.transport = getattr(self.backend, "transport", "rccl")
            if self.transport == "rccl":
                pg = str(dist.get_backend(group))
                if "nccl" not in pg:
                    raise RuntimeError(
                        "bolt_amd: the mi355x mode moves records between GPUs over RCCL; initialise "
                        "torch.distributed with backend 'nccl' (or 'cpu:gloo,cuda:nccl'), not %r -- "
                        "device bytes are never staged through the host" % pg)
                # RCCL communicator of libbolt_mi355x (bm_comm_init) for the record exchanges
                self._init_comm()

    def _init_comm(self):
        """One RCCL communicator over this context's ranks: rank 0 makes the id,
        the others read it from the torch.distributed rendezvous store."""
        import ctypes
        import torch
        import torch.distributed as dist
        from bolt_amd.mi355x import _lib
        lib = _lib.load()
        key = self._comm_key(dist.get_process_group_ranks(self.group or dist.group.WORLD))
        uid = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
        store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            _lib.check(lib.bm_comm_unique_id(uid, _lib.COMM_ID_BYTES), "bm_comm_unique_id")
            store.set(key, uid.raw)
        else:
            raw = store.get(key)
            ctypes.memmove(uid, raw, _lib.COMM_ID_BYTES)
        comm = ctypes.c_void_p()
        _lib.check(lib.bm_comm_init(ctypes.byref(comm), self.world_size, uid, self.rank), "bm_comm_init")
        self.comm = comm.value
        # the exchanges run beside the pipelined pack / unpack kernels of the
        # current stream, whose grids can fill every CU: a high-priority stream
        # lets RCCL's workgroups dispatch ahead of the copies' queued ones
        self.comm_stream = torch.cuda.Stream(self.device, priority=-1)

    @classmethod
    def _comm_key(cls, ranks):
        """Rendezvous key of the next communicator over ``ranks`` (global ranks).

        Counted per rank set, so processes that open contexts over different
        subgroups in different orders still agree on every key (a single
        process-wide counter would hand a rank the id of another group)."""
        ranks = tuple(int(r) for r in ranks)
        n = cls._ncomm.get(ranks, 0) + 1
        cls._ncomm[ranks] = n
        return "bolt_amd/rccl_id/%s/%d" % (",".join(map(str, ranks)), n)

    def close(self):
        """Release the RCCL communicator (before the process group is destroyed).

        Waits (bounded, bm_comm_wait) for the exchanges still queued on the
        communicator's stream and on the current stream first; a failed
        communicator is released without raising again."""
        if self.comm is not None:
            from bolt_amd.mi355x import _lib
            import torch
            lib = _lib.load()
            comm, self.comm = self.comm, None
            try:
                for st in (self.comm_stream, torch.cuda.current_stream(self.device)):
                    _lib.check(lib.bm_comm_wait(comm, st.cuda_stream, self.comm_timeout), "bm_comm_wait")
            except _lib.BoltCommError:
                pass  # already aborted: destroy only frees the handle
            finally:
                _lib.check(lib.bm_comm_destroy(comm), "bm_comm_destroy")

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
