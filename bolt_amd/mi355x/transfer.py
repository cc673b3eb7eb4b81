"""Host <-> HBM transfers of the mi355x mode (ingest and egress).

The reference moves records driver -> executors with parallelize
(spark/construct.py:69) and back with collect (array.py:1012-1014).  Here the
path is PCIe (63 GB/s spec, MI355X_MICROARCH.md).

Ingest: the runtime's own pageable copy reaches 56 GB/s on the box, ahead of
staging through page-locked chunks (54 GB/s at 8 copy threads,
profiles/r01_transfer_*.log), so it is the default (H2D_DIRECT = False
selects the staged path).  Egress: a pageable D2H bounces through the
driver's staging at 6-8 GB/s, so large results are staged through two
page-locked chunks from torch's caching host allocator -- the host memcpy of
chunk i (split over 8 threads; numpy releases the GIL) overlaps the DMA of
chunk i+1 -- 17-18 GB/s, bound by first-touch page faults of the fresh numpy
result.  Small transfers take one pinned buffer and return a view of it.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

CHUNK = 64 << 20          # bytes per staging chunk
SMALL = 8 << 20           # below this: one pinned buffer, no pipeline
THREADS = 8               # host memcpy threads per chunk
H2D_DIRECT = True         # ingest through the runtime's pageable copy (False: staged)

# statistics results up to SMALL bytes are stored by the reduction kernel
# straight into a page-locked host buffer (no D2H copy launch)
ZERO_COPY = True

_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=THREADS, thread_name_prefix="bolt-amd-copy")
    return _POOL


def _par_copy(dst, src):
    """dst[:] = src for 1-D uint8 arrays, split over the copy threads."""
    n = src.size
    if n < (4 << 20):
        dst[:] = src
        return
    step = (n + THREADS - 1) // THREADS
    futs = [_pool().submit(np.copyto, dst[i:i + step], src[i:i + step]) for i in range(0, n, step)]
    for f in futs:
        f.result()


def to_device(host, device):
    """Contiguous host bytes (1-D uint8 ndarray) -> uint8 tensor on ``device``."""
    import torch
    host = np.ascontiguousarray(host).reshape(-1).view(np.uint8)
    if device.type != "cuda":
        return torch.from_numpy(host.copy())
    n = host.size
    if H2D_DIRECT:
        return torch.from_numpy(host).to(device)
    out = torch.empty(n, dtype=torch.uint8, device=device)
    if n == 0:
        return out
    stream = torch.cuda.current_stream(device)
    if n <= SMALL:
        pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        _par_copy(pin.numpy(), host)
        out.copy_(pin, non_blocking=True)
        stream.synchronize()
        return out
    bufs = [torch.empty(CHUNK, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    evs = [None, None]
    for i, lo in enumerate(range(0, n, CHUNK)):
        hi = min(n, lo + CHUNK)
        k = i % 2
        if evs[k] is not None:
            evs[k].synchronize()  # the DMA that last read this buffer is done
        _par_copy(bufs[k].numpy()[:hi - lo], host[lo:hi])
        out[lo:hi].copy_(bufs[k][:hi - lo], non_blocking=True)
        evs[k] = torch.cuda.Event()
        evs[k].record(stream)
    stream.synchronize()
    return out


def to_host(t, dtype, shape):
    """uint8 tensor -> host ndarray of ``dtype`` / ``shape`` (the mode's only D2H)."""
    import torch
    dtype = np.dtype(dtype)
    if t.device.type != "cuda":
        return t.numpy().view(dtype).reshape(shape)
    n = t.numel()
    if n <= SMALL:
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        if n:
            host.copy_(t, non_blocking=True)
            torch.cuda.current_stream(t.device).synchronize()
        return host.numpy().view(dtype).reshape(shape)
    out = np.empty(n, dtype=np.uint8)
    copy_to_host(t, out)
    return out.view(dtype).reshape(shape)


def staging_buffers():
    """Two page-locked CHUNK-byte buffers for copy_to_host (a caller that copies
    many windows allocates them once)."""
    import torch
    return [torch.empty(CHUNK, dtype=torch.uint8, pin_memory=True) for _ in range(2)]


def copy_to_host(t, out, staging=None, produce=None, chunk=CHUNK):
    """out[:] = the bytes of uint8 tensor ``t`` (``out`` a host uint8 ndarray of
    t.numel() bytes), staged through two page-locked chunks (``staging``, or
    two from torch's caching host allocator): the host copy out of chunk i
    overlaps the DMA of chunk i+1.

    ``produce(lo, hi, k)``, when given, replaces ``t`` (pass its device): it
    queues on the current stream whatever fills bytes [lo, hi) of the result
    into device window ``k`` (0 or 1, alternating) and returns that window's
    tensor -- a row-padded array's rows compacted window by window
    (array.py ``_padded_to_host``); ``chunk`` is then the window size."""
    import torch
    n = out.size if produce is not None else t.numel()
    if n == 0:
        return
    if t.device.type != "cuda":
        out[:] = (produce(0, n, 0) if produce is not None else t).numpy()
        return
    stream = torch.cuda.current_stream(t.device)
    src = (lambda lo, hi, k: produce(lo, hi, k)) if produce is not None else (lambda lo, hi, k: t[lo:hi])
    if n <= SMALL:
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        host.copy_(src(0, n, 0), non_blocking=True)
        stream.synchronize()
        _par_copy(out, host.numpy())
        return
    bufs = staging if staging is not None else staging_buffers()
    evs = [torch.cuda.Event(), torch.cuda.Event()]
    starts = list(range(0, n, chunk))
    # keep one DMA in flight ahead of the host copy out of the previous chunk
    for i, lo in enumerate(starts):
        hi = min(n, lo + chunk)
        k = i % 2
        bufs[k][:hi - lo].copy_(src(lo, hi, k), non_blocking=True)
        evs[k].record(stream)
        if i > 0:
            plo = starts[i - 1]
            phi = min(n, plo + chunk)
            evs[1 - k].synchronize()
            _par_copy(out[plo:phi], bufs[1 - k].numpy()[:phi - plo])
    lo = starts[-1]
    evs[(len(starts) - 1) % 2].synchronize()
    _par_copy(out[lo:n], bufs[(len(starts) - 1) % 2].numpy()[:n - lo])


def host_result(backend, nbytes, device):
    """A page-locked host buffer of ``nbytes`` that kernels on ``device`` can
    store into, or None (zero-copy results off, not a GPU, too large, or the
    allocation is not device-addressable)."""
    if not ZERO_COPY or device.type != "cuda" or not 0 < nbytes <= SMALL:
        return None
    writable = getattr(backend, "host_writable", None)
    if writable is None:
        return None
    import torch
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    # torch's caching host allocator hands the same page-locked blocks out
    # again: the check runs once per (block, size, device) (~1 us of a
    # statistic's host path, profiles/r01_host_breakdown.log)
    key = (host.data_ptr(), nbytes, device.index)
    ok = _WRITABLE.get(key)
    if ok is None:
        ok = bool(writable(host))
        if len(_WRITABLE) > 1024:
            _WRITABLE.clear()
        _WRITABLE[key] = ok
    return host if ok else None


_WRITABLE = {}  # (page-locked block address, bytes, device) -> its kernels can store into it


_STREAMS = {}  # device index -> torch Stream object of the last current stream seen


def current_stream(device):
    """torch.cuda.current_stream(device), reusing the Stream object while the
    current stream stays the same (building one costs ~4 us per statistic;
    profiles/r02x_c1_probe.log)."""
    import torch
    idx = device.index if device.index is not None else torch.cuda.current_device()
    raw = torch._C._cuda_getCurrentRawStream(idx)
    s = _STREAMS.get(idx)
    if s is None or s.cuda_stream != raw:
        s = _STREAMS[idx] = torch.cuda.current_stream(device)
    return s


def finish_host_result(host, device, dtype, shape):
    """Wait for the kernel that fills ``host`` and view it as the result."""
    current_stream(device).synchronize()
    return host.numpy().view(np.dtype(dtype)).reshape(shape)
