"""Multi-GPU data movement for the MI355X backend (one process per GPU).

The Spark path moves records with two shuffles and a driver collect
(bolt/spark/chunk.py:251-261 partitionBy in keys_to_values, chunk.py:179-191
in unchunk, array.py:1012-1014 collect).  Here records are slabs of the
leading key axis, one slab per rank, and the only exchange a swap needs is
ONE all-to-all (torch.distributed over RCCL, i.e. xGMI peer links):

  pack    local strided copy of the shard into G contiguous send blocks,
          block q = the part of the permuted array that rank q will own;
  a2a     all_to_all_single with per-peer byte counts;
  unpack  local strided copy of each received block into its place.

A permutation that keeps the leading axis (perm[0] == 0) needs no exchange.
Statistics exchange only small per-output states (all_gather), see array.py.
"""
import numpy as np

from bolt_amd.mi355x.context import contiguous_strides


def _empty(nbytes, device):
    import torch
    return torch.empty(max(0, int(nbytes)), dtype=torch.uint8, device=device)


def to_host(t, dtype, shape):
    """Device bytes -> host ndarray of ``dtype``/``shape`` (the only D2H of the mode).

    GPU tensors go through a page-locked staging buffer from torch's caching
    host allocator (a DMA, no pageable bounce) on the current stream; the
    returned array owns that buffer.
    """
    import torch
    dtype = np.dtype(dtype)
    if t.device.type != "cuda":
        return t.numpy().view(dtype).reshape(shape)
    host = torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True)
    if t.numel():
        host.copy_(t, non_blocking=True)
        torch.cuda.current_stream(t.device).synchronize()
    return host.numpy().view(dtype).reshape(shape)


# Optional phase timing of the exchange (bench.py sets it to a dict):
# name -> list of (start, end) torch.cuda.Event pairs on the current stream.
PROFILE = None


class _phase(object):
    def __init__(self, name, device):
        self.name, self.device = name, device

    def __enter__(self):
        if PROFILE is not None and self.device.type == "cuda":
            import torch
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()
        return self

    def __exit__(self, *exc):
        if PROFILE is not None and self.device.type == "cuda":
            self.ev[1].record()
            PROFILE.setdefault(self.name, []).append(self.ev)
        return False


def _wide(t, sizes, unit):
    """View a byte tensor as elements of ``unit`` bytes (1/2/4/8) so RCCL counts
    stay small for multi-GB exchanges.  ``unit`` must be the same on every rank
    (it is derived from global quantities: the element size, the row size)."""
    import torch
    if unit not in (4, 8):  # (gloo has no 16-bit collectives)
        unit = 1
    dt = {8: torch.int64, 4: torch.int32, 1: torch.uint8}[unit]
    return t.view(dt), [int(s) // unit for s in sizes]


def _unit(nbytes):
    """Largest power of two <= 8 dividing ``nbytes`` (a global quantity)."""
    u = 8
    while u > 1 and int(nbytes) % u:
        u //= 2
    return u


def all_gather_bytes(ctx, local, sizes):
    """Concatenate every rank's byte tensor (sizes[r] bytes from rank r) on every rank."""
    import torch
    import torch.distributed as dist
    if ctx.world_size == 1:
        return local
    m = max(sizes) if sizes else 0
    m = (m + 7) // 8 * 8
    buf = _empty(m, local.device)
    if local.numel():
        buf[:local.numel()].copy_(local)
    outs = [_empty(m, local.device) for _ in range(ctx.world_size)]
    wb, _ = _wide(buf, [m], 8)
    wo = [_wide(o, [m], 8)[0] for o in outs]
    dist.all_gather(wo, wb, group=ctx.group)
    return torch.cat([o[:s] for o, s in zip(outs, sizes)]) if m else _empty(0, local.device)


def all_to_all_bytes(ctx, send, send_sizes, recv_sizes, unit=1):
    """Variable-size all-to-all of byte blocks; every size is a multiple of ``unit``."""
    import torch.distributed as dist
    recv = _empty(sum(recv_sizes), send.device)
    ws, ss = _wide(send, send_sizes, unit)
    wr, rs = _wide(recv, recv_sizes, unit)
    with _phase("all_to_all", send.device):
        dist.all_to_all_single(wr, ws, output_split_sizes=rs, input_split_sizes=ss, group=ctx.group)
    return recv


def permute_sharded(ctx, backend, data, shape, perm, es):
    """This rank's shard of x.transpose(perm) for a sharded x of global ``shape``.

    ``data`` holds this rank's slab of x's leading axis.  Returns the byte
    tensor of this rank's slab of the result's leading axis.
    """
    shape = tuple(int(s) for s in shape)
    nd = len(shape)
    out_shape = tuple(shape[p] for p in perm)
    in_b = ctx.bounds(shape[0])
    out_b = ctx.bounds(out_shape[0])
    r = ctx.rank
    in_lo, in_hi = in_b[r]
    loc_in = (in_hi - in_lo,) + shape[1:]
    sin = contiguous_strides(loc_in)

    if perm[0] == 0 or ctx.world_size == 1:
        lo, hi = out_b[r]
        loc_out = (hi - lo,) + out_shape[1:]
        out = _empty(int(np.prod(loc_out)) * es, data.device)
        if out.numel():
            backend.permute(data, loc_in, perm, es, out)
        return out

    a = perm[0]          # input axis that becomes the output's leading axis
    j = perm.index(0)    # where the input's leading axis lands
    blocks = []
    for q in range(ctx.world_size):
        qlo, qhi = out_b[q]
        bshape = list(out_shape)
        bshape[0] = qhi - qlo
        bshape[j] = in_hi - in_lo
        blocks.append((qlo, bshape))
    send_sizes = [int(np.prod(b)) * es for _, b in blocks]
    send = _empty(sum(send_sizes), data.device)
    off = 0
    with _phase("pack", data.device):
        for (qlo, bshape), nb in zip(blocks, send_sizes):
            if nb:
                sstr = [sin[p] for p in perm]
                backend.copy_strided(data, qlo * sin[a] * es, send, off, bshape, sstr,
                                     contiguous_strides(bshape), es)
            off += nb

    lo, hi = out_b[r]
    loc_out = (hi - lo,) + out_shape[1:]
    recv_sizes = []
    rblocks = []
    for s in range(ctx.world_size):
        slo, shi = in_b[s]
        bshape = list(loc_out)
        bshape[j] = shi - slo
        rblocks.append((slo, bshape))
        recv_sizes.append(int(np.prod(bshape)) * es)
    recv = all_to_all_bytes(ctx, send, send_sizes, recv_sizes, _unit(es))

    out = _empty(int(np.prod(loc_out)) * es, data.device)
    tstr = contiguous_strides(loc_out)
    off = 0
    with _phase("unpack", data.device):
        for (slo, bshape), nb in zip(rblocks, recv_sizes):
            if nb:
                backend.copy_strided(recv, off, out, slo * tstr[j] * es, bshape,
                                     contiguous_strides(bshape), tstr, es)
            off += nb
    return out


def redistribute_rows(ctx, data, old_rows, old_rowbytes, new_rows, new_rowbytes):
    """Re-shard a flat byte array whose leading-axis extent changes (same bytes, new slabs).

    Used where only the key shape changes (Keys.reshape); the global byte
    sequence is unchanged, only which rank owns which bytes.
    """
    if ctx.world_size == 1:
        return data
    ob = [(lo * old_rowbytes, hi * old_rowbytes) for lo, hi in ctx.bounds(old_rows)]
    nb = [(lo * new_rowbytes, hi * new_rowbytes) for lo, hi in ctx.bounds(new_rows)]
    r = ctx.rank
    mlo, mhi = ob[r]
    send_sizes = [max(0, min(mhi, qhi) - max(mlo, qlo)) for qlo, qhi in nb]
    tlo, thi = nb[r]
    recv_sizes = [max(0, min(thi, shi) - max(tlo, slo)) for slo, shi in ob]
    return all_to_all_bytes(ctx, data, send_sizes, recv_sizes, _unit(np.gcd(old_rowbytes, new_rowbytes)))
