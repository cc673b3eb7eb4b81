"""Multi-GPU data movement for the MI355X backend (one process per GPU).

The Spark path moves records with two shuffles and a driver collect
(bolt/spark/chunk.py:251-261 partitionBy in keys_to_values, chunk.py:179-191
in unchunk, array.py:1012-1014 collect).  Here records are slabs of the
leading key axis, one slab per rank, and the only exchange a swap needs is
ONE all-to-all over RCCL (xGMI peer links), issued by libbolt_mi355x itself
(bm_alltoallv / bm_allgatherv on the context's communicator; torch only owns
the buffers and streams):

  pack    local strided copy of the shard into G contiguous send blocks,
          block q = the part of the permuted array that rank q will own;
  a2a     bm_alltoallv with per-peer byte counts (one RCCL group of
          ncclSend / ncclRecv pairs, every link at once; the self block is a
          local device copy);
  unpack  local strided copy of each received block into its place.

The transport is the context's (MI355XContext.transport), chosen by the kernel
backend, never by the process group: the production HIP backend always uses
the library's RCCL communicator ("rccl").  Only the test executors registered
through _ops.register_backend select torch.distributed collectives: "torch"
(the numpy executor on CPU tensors over gloo) and "host" (the one-GPU
multi-rank rehearsal, device bytes staged through the host over gloo).

Every RCCL exchange ends in a bounded host wait (bm_comm_wait): a peer that
died or posted a mismatched exchange raises BoltCommError instead of hanging.

A permutation that keeps the leading axis (perm[0] == 0) needs no exchange.
Statistics exchange only small per-output states (all_gather), see array.py.
"""
import numpy as np

from bolt_amd.mi355x.context import contiguous_strides


def _empty(nbytes, device):
    import torch
    return torch.empty(max(0, int(nbytes)), dtype=torch.uint8, device=device)


from bolt_amd.mi355x.transfer import to_host  # noqa: E402,F401  (re-exported)


# Pipeline depth of the swap exchange: K = per-peer bytes // stage_bytes(G),
# clamped to [1, 8] (STAGES overrides; tests set it to exercise the stages).
# Stage i's exchange overlaps stage i-1's unpack and stage i+1's pack; the
# first pack and the last unpack do not overlap, so deeper is better (each is
# 1/K of the local work) until a stage's per-peer message gets too small for
# RCCL to keep a link at its plateau.  The local work moves 2x a stage's bytes
# through HBM at ~5.8 TB/s (profiles/r01_exchange_local.log) while the links
# move them at (G-1)*153 GB/s per rank, so at every G the exchange, not the
# pack/unpack, is the critical path.  The floor per world size is the
# smallest per-peer message that keeps K = 8 at the BASELINE sizes while
# staying >= 8 MiB per peer (a send/recv pair is near its plateau from a few
# MiB); larger worlds split each rank's bytes over more peers, so the floor
# shrinks with G:
#   G = 2: 1 peer,  32 MiB     G = 4: 3 peers, 16 MiB     G = 8: 7 peers, 8 MiB
# (C2 per rank: 1.05 / 0.52 / 0.26 GB per peer -> K = 8 at every G.)
STAGES = None
STAGE_BYTES_BY_WORLD = {2: 32 << 20, 4: 16 << 20, 8: 8 << 20}
STAGE_BYTES = None  # override for every world size (tests lower it)


def stage_bytes(world):
    if STAGE_BYTES is not None:
        return STAGE_BYTES
    for g in sorted(STAGE_BYTES_BY_WORLD, reverse=True):
        if world >= g:
            return STAGE_BYTES_BY_WORLD[g]
    return STAGE_BYTES_BY_WORLD[2]


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
    if t.numel() == 0:  # an empty slab may carry any stride
        return torch.empty(0, dtype=dt, device=t.device), [0 for _ in sizes]
    return t.view(dt), [int(s) // unit for s in sizes]


def _unit(nbytes):
    """Largest power of two <= 8 dividing ``nbytes`` (a global quantity)."""
    u = 8
    while u > 1 and int(nbytes) % u:
        u //= 2
    return u


class _Work(object):
    """An exchange running on the context's RCCL stream: wait() orders the
    caller's current stream after it (the host never blocks)."""

    def __init__(self, done):
        self.done = done

    def wait(self):
        import torch
        torch.cuda.current_stream().wait_event(self.done)


def _offsets(sizes):
    return [int(v) for v in np.r_[0, np.cumsum([int(v) for v in sizes])][:-1]]


def _drain_local(device):
    """Wait (unbounded) for the local work queued on the current stream, so that
    the bounded wait after an exchange times the exchange alone: a long
    legitimate compute queue must not read as a failed peer."""
    import torch
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(device))
    ev.synchronize()


def _rccl_all_gather(ctx, local, sizes):
    """bm_allgatherv on the current stream (include/bolt_mi355x.h), then a
    bounded wait for it (bm_comm_wait)."""
    import torch
    from bolt_amd.mi355x import _lib
    recv = _empty(sum(sizes), local.device)
    _drain_local(local.device)
    stream = torch.cuda.current_stream(local.device).cuda_stream
    sp = local.data_ptr() if local.numel() else None
    rp = recv.data_ptr() if recv.numel() else None
    _lib.check(_lib.load().bm_allgatherv(ctx.comm, sp, int(sizes[ctx.rank]), rp, _lib.i64_array(sizes),
                                         _lib.i64_array(_offsets(sizes)), stream), "bm_allgatherv")
    comm_wait(ctx, stream)
    return recv


def comm_wait(ctx, stream):
    """Host wait for ``stream`` (a raw hipStream_t or a torch Stream) bounded by
    ctx.comm_timeout; an RCCL error or a timeout aborts the communicator and
    raises _lib.BoltCommError (bm_comm_wait)."""
    from bolt_amd.mi355x import _lib
    raw = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    _lib.check(_lib.load().bm_comm_wait(ctx.comm, raw, float(ctx.comm_timeout)), "bm_comm_wait")


def _rccl_all_to_all(ctx, send, send_sizes, recv_sizes, async_op):
    """bm_alltoallv; async: on the context's RCCL stream, fenced by events."""
    import torch
    from bolt_amd.mi355x import _lib
    recv = _empty(sum(recv_sizes), send.device)
    cur = torch.cuda.current_stream(send.device)
    stream = ctx.comm_stream if async_op else cur
    if not async_op:
        _drain_local(send.device)
    if async_op:
        ready = torch.cuda.Event()
        ready.record(cur)
        stream.wait_event(ready)
        # the buffers are used on the RCCL stream: keep the allocator from
        # reusing them before it is done
        send.record_stream(stream)
        recv.record_stream(stream)
    sp = send.data_ptr() if send.numel() else None
    rp = recv.data_ptr() if recv.numel() else None
    if PROFILE is not None:  # the RCCL group alone, on the stream it runs on
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record(stream)
    _lib.check(_lib.load().bm_alltoallv(ctx.comm, sp, _lib.i64_array(send_sizes), _lib.i64_array(_offsets(send_sizes)),
                                        rp, _lib.i64_array(recv_sizes), _lib.i64_array(_offsets(recv_sizes)),
                                        stream.cuda_stream), "bm_alltoallv")
    if PROFILE is not None:
        ev[1].record(stream)
        PROFILE.setdefault("rccl", []).append(ev)
    if not async_op:
        comm_wait(ctx, stream)
        return recv
    done = torch.cuda.Event()
    done.record(stream)
    return recv, _Work(done)


def all_gather_bytes(ctx, local, sizes):
    """Concatenate every rank's byte tensor (sizes[r] bytes from rank r) on every rank."""
    if ctx.world_size == 1:
        return local
    if ctx.transport == "rccl":
        return _rccl_all_gather(ctx, local, sizes)
    return _test_all_gather(ctx, local, sizes)


def all_to_all_bytes(ctx, send, send_sizes, recv_sizes, unit=1, async_op=False):
    """Variable-size all-to-all of byte blocks; every size is a multiple of ``unit``.

    With async_op the call returns (recv, work): the exchange runs on the
    collective's own stream and ``work.wait()`` orders the caller's stream
    after it (no host block on RCCL)."""
    if ctx.transport == "rccl":
        return _rccl_all_to_all(ctx, send, send_sizes, recv_sizes, async_op)
    return _test_all_to_all(ctx, send, send_sizes, recv_sizes, unit, async_op)


# Egress across GPUs moves the global byte sequence in windows of at most this
# many bytes: each window is one all_gather into a window-sized device buffer,
# then a staged D2H into its place in the host result -- device memory per rank
# stays at its slab plus one window, never the whole array (the reference
# collects to the driver, bolt/spark/array.py:1006-1014).
EGRESS_WINDOW = None  # None: 2 x the staging chunk (transfer.CHUNK); tests lower it


def egress_window():
    from bolt_amd.mi355x import transfer
    return int(EGRESS_WINDOW) if EGRESS_WINDOW else 2 * transfer.CHUNK


def gather_to_host(ctx, local, sizes, out=None, rows=None):
    """The concatenation of every rank's bytes (``sizes[r]`` bytes from rank r,
    in rank order) as a host uint8 ndarray on every rank, gathered window by
    window (EGRESS_WINDOW).  ``out``: a host uint8 array to fill instead.
    ``rows``: (row bytes R*es, pitch bytes P*es, backend) when ``local`` holds
    row-padded rows: each window's rows are compacted on the way (no dense
    copy of the slab)."""
    from bolt_amd.mi355x.transfer import copy_to_host
    sizes = [int(v) for v in sizes]
    if out is None:
        out = np.empty(sum(sizes), dtype=np.uint8)
    if ctx.world_size == 1 and rows is None:
        copy_to_host(local, out)
        return out
    return gather_windows(ctx, local, sizes, out, all_gather_bytes, rows)


def gather_windows(ctx, local, sizes, out, gather, rows=None):
    """gather_to_host's windows: each window of the global byte sequence is one
    ``gather`` (all_gather_bytes) into a window-sized device buffer, then a
    staged D2H into its place in ``out``; the two page-locked staging buffers
    are allocated once for all windows.  With ``rows`` the windows are whole
    rows and this rank's piece of each is compacted from its padded rows into
    one window-sized device buffer first."""
    from bolt_amd.mi355x.transfer import SMALL, copy_to_host, staging_buffers
    total = sum(sizes)
    offs = np.r_[0, np.cumsum(sizes)].astype(np.int64)
    me = ctx.rank
    w = max(1, egress_window())
    win = None
    if rows is not None:
        rb, pb, be = rows
        w = max(rb, w // rb * rb)  # windows of whole rows (every slab is whole rows too)
        win = _empty(min(w, max(sizes[me], 0)), local.device) if sizes[me] else None
    staging = staging_buffers() if local.device.type == "cuda" and min(w, total) > SMALL else None
    for g0 in range(0, total, w):
        g1 = min(total, g0 + w)
        part = [max(0, min(g1, int(offs[r + 1])) - max(g0, int(offs[r]))) for r in range(len(sizes))]
        lo = max(g0, int(offs[me])) - int(offs[me])
        if not part[me]:
            piece = local[:0]
        elif rows is None:
            piece = local[lo:lo + part[me]]
        else:
            n = part[me] // rb
            be.copy_strided(local, (lo // rb) * pb, win, 0, [n, rb], [pb, 1], [rb, 1], 1)
            piece = win[:part[me]]
        buf = gather(ctx, piece, part)
        copy_to_host(buf, out[g0:g1], staging)
        del buf
    return out


# --- test executors only (transport "torch" / "host"; see the module docstring)

def _check_test_transport(ctx, t):
    if ctx.transport not in ("torch", "host"):
        raise RuntimeError("bolt_amd: transport %r has no torch.distributed path" % (ctx.transport,))
    if t.device.type == "cuda" and ctx.transport != "host":
        raise RuntimeError("bolt_amd: device bytes never take the torch.distributed path "
                           "(the mi355x mode exchanges them over RCCL)")


def _test_all_gather(ctx, local, sizes):
    import torch
    import torch.distributed as dist
    _check_test_transport(ctx, local)
    if ctx.transport == "host" and local.device.type == "cuda":
        return _test_all_gather(ctx, local.cpu(), sizes).to(local.device)
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


def _test_all_to_all(ctx, send, send_sizes, recv_sizes, unit, async_op):
    import torch.distributed as dist
    _check_test_transport(ctx, send)
    if ctx.transport == "host" and send.device.type == "cuda":
        recv = _test_all_to_all(ctx, send.cpu(), send_sizes, recv_sizes, unit, False).to(send.device)
        return (recv, None) if async_op else recv
    recv = _empty(sum(recv_sizes), send.device)
    ws, ss = _wide(send, send_sizes, unit)
    wr, rs = _wide(recv, recv_sizes, unit)
    work = dist.all_to_all_single(wr, ws, output_split_sizes=rs, input_split_sizes=ss, group=ctx.group,
                                  async_op=async_op)
    return (recv, work) if async_op else recv


def permute_sharded(ctx, backend, data, shape, perm, es, src_pitch=None, out_pitch=None):
    """This rank's shard of x.transpose(perm) for a sharded x of global ``shape``.

    ``data`` holds this rank's slab of x's leading axis.  Returns the byte
    tensor of this rank's slab of the result's leading axis.  ``src_pitch`` /
    ``out_pitch``: elements between the rows (last axis) of a row-padded
    source / result (array.py ROW_PITCH); the exchange's pack reads the padded
    source rows in place and its unpack writes the padded result rows.
    """
    from bolt_amd.mi355x.plan import padded_strides
    if ctx.world_size == 1 and src_pitch is None and out_pitch is None:  # one GPU: one kernel
        out = _empty(data.numel(), data.device)
        if out.numel():
            backend.permute(data, shape, perm, es, out)
        return out
    shape = tuple(int(s) for s in shape)
    nd = len(shape)
    out_shape = tuple(shape[p] for p in perm)
    in_b = ctx.bounds(shape[0])
    out_b = ctx.bounds(out_shape[0])
    r = ctx.rank
    in_lo, in_hi = in_b[r]
    loc_in = (in_hi - in_lo,) + shape[1:]
    sin = contiguous_strides(loc_in) if src_pitch is None else padded_strides(loc_in, src_pitch)
    lo, hi = out_b[r]
    loc_out = (hi - lo,) + out_shape[1:]
    if out_pitch is None:
        out = _empty(int(np.prod(loc_out)) * es, data.device)
        tstr = contiguous_strides(loc_out)
    else:
        out = _empty(int(np.prod(loc_out[:-1])) * int(out_pitch) * es, data.device)
        tstr = padded_strides(loc_out, out_pitch)

    if perm[0] == 0 or ctx.world_size == 1:
        if out.numel() and int(np.prod(loc_out)):
            if src_pitch is None and out_pitch is None:
                backend.permute(data, loc_in, perm, es, out)
            else:
                backend.copy_strided(data, 0, out, 0, list(loc_out), [sin[p] for p in perm], tstr, es)
        return out

    a = perm[0]          # input axis that becomes the output's leading axis
    j = perm.index(0)    # where the input's leading axis lands
    G = ctx.world_size
    sstr = [sin[p] for p in perm]
    # Pipeline the exchange in K stages: stage k packs its sub-blocks, starts
    # its all-to-all asynchronously (RCCL stream) and, while that runs, the
    # current stream unpacks stage k-1 and packs k+1.  The stages split the
    # output's leading axis (every peer's rows in K parts) -- unless that axis
    # is the source-contiguous one (a .T: C3 / C5), whose rows per peer and
    # stage would be a few elements (16-B source segments, 0.11 of HBM peak in
    # the r05a rehearsal): the stages then split the largest other output axis
    # that is not the exchanged one, and each pack reads whole source rows.
    stage_ax = None
    if sin[a] == 1 and nd >= 3:
        cand = [k for k in range(1, nd) if k != j and out_shape[k] > 1]
        if cand:
            stage_ax = max(cand, key=lambda k: (out_shape[k], -k))
    # K must agree on every rank (each stage is one collective), so it comes
    # from global quantities only: the largest slab's per-peer block
    max_rows = max(hi_ - lo_ for lo_, hi_ in in_b)
    per_peer = max_rows * int(np.prod(shape[1:])) * es // G
    K = STAGES if STAGES else int(max(1, min(8, per_peer // stage_bytes(G))))
    if stage_ax is None:
        K = max(1, min(K, min(b - a_ for a_, b in out_b) or 1))
    else:
        K = max(1, min(K, out_shape[stage_ax]))

    def sub(q, k):
        """(output rows of peer q, range of the stage axis or None) in stage k."""
        qlo, qhi = out_b[q]
        if stage_ax is None:
            n = qhi - qlo
            return (qlo + k * n // K, qlo + (k + 1) * n // K), None
        n = out_shape[stage_ax]
        return (qlo, qhi), (k * n // K, (k + 1) * n // K)

    # equal slabs on every rank (the weak-scaling benches): one pack and one
    # unpack launch per stage instead of one per peer
    even_out = G > 1 and out_shape[0] % G == 0
    even_in = G > 1 and shape[0] % G == 0

    with _phase("exchange", data.device):
        pending = None
        for k in range(K):
            send_sizes, parts = [], []
            for q in range(G):
                (slo_q, shi_q), sr = sub(q, k)
                bshape = list(out_shape)
                bshape[0] = shi_q - slo_q
                bshape[j] = in_hi - in_lo
                off = slo_q * sin[a]                   # source element offset of the block
                if sr is not None:
                    bshape[stage_ax] = sr[1] - sr[0]
                    off += sr[0] * sstr[stage_ax]
                parts.append((off, bshape))
                send_sizes.append(int(np.prod(bshape)) * es)
            send = _empty(sum(send_sizes), data.device)
            if even_out and send_sizes[0]:
                # every peer's block has one shape and the sources are evenly
                # spaced along axis a: the G packs are one strided copy
                bshape = parts[0][1]
                backend.copy_strided(data, parts[0][0] * es, send, 0, [G] + bshape,
                                     [parts[1][0] - parts[0][0]] + sstr,
                                     [send_sizes[0] // es] + contiguous_strides(bshape), es)
            else:
                off = 0
                for (soff, bshape), nb in zip(parts, send_sizes):
                    if nb:
                        backend.copy_strided(data, soff * es, send, off, bshape, sstr,
                                             contiguous_strides(bshape), es)
                    off += nb
            (mlo, mhi), sr = sub(r, k)
            recv_sizes, rparts = [], []
            for s_ in range(G):
                slo, shi = in_b[s_]
                bshape = list(loc_out)
                bshape[0] = mhi - mlo
                bshape[j] = shi - slo
                doff = (mlo - lo) * tstr[0] + slo * tstr[j]   # destination element offset
                if sr is not None:
                    bshape[stage_ax] = sr[1] - sr[0]
                    doff += sr[0] * tstr[stage_ax]
                rparts.append((doff, bshape))
                recv_sizes.append(int(np.prod(bshape)) * es)
            recv, work = all_to_all_bytes(ctx, send, send_sizes, recv_sizes, _unit(es), async_op=True)
            if pending is not None:
                _unpack(backend, pending, out, tstr, es, even_in)
            pending = (recv, work, send, rparts, recv_sizes)
        _unpack(backend, pending, out, tstr, es, even_in)
        if ctx.transport == "rccl":
            # bounded host wait for the last exchange (the final unpack is
            # already queued behind it): a failed peer raises, never hangs
            comm_wait(ctx, ctx.comm_stream)
    return out


def _unpack(backend, pending, out, tstr, es, even=False):
    recv, work, send, rparts, recv_sizes = pending
    if work is not None:
        work.wait()  # the current stream waits for this stage's all-to-all
    if even and recv_sizes[0]:
        # equal blocks from every rank, landing evenly spaced along axis j: one copy
        doff, bshape = rparts[0]
        G = len(rparts)
        backend.copy_strided(recv, 0, out, doff * es, [G] + bshape,
                             [recv_sizes[0] // es] + contiguous_strides(bshape),
                             [rparts[1][0] - doff] + tstr, es)
    else:
        off = 0
        for (doff, bshape), nb in zip(rparts, recv_sizes):
            if nb:
                backend.copy_strided(recv, off, out, doff * es, bshape, contiguous_strides(bshape), tstr, es)
            off += nb
    del send


def select_sharded(ctx, backend, data, shape, starts, steps, out_shape, es, src_strides=None):
    """This rank's slab of x[start_k :: step_k] (basic slicing) for a sharded x.

    Output row i of the leading axis is input row starts[0] + i*steps[0].  On
    one GPU this is a single strided copy; across GPUs each rank packs, for
    every destination, the selected rows it holds (they form one run of
    output rows), one all-to-all moves them, and they land in order.
    ``src_strides``: element strides of a source that is not C-contiguous (a
    row-padded array: plan.padded_strides of the global shape, which are also
    every slab's).
    """
    shape = tuple(int(x) for x in shape)
    out_shape = tuple(int(x) for x in out_shape)
    for d, n, s0, st in zip(shape, out_shape, starts, steps):
        # every selected index inside its axis: the copies below read through
        # raw device pointers
        if n > 0 and not (0 <= s0 < d and 0 <= s0 + (n - 1) * st < d):
            raise ValueError("selection %d::%d of %d elements leaves an axis of %d" % (s0, st, n, d))
    in_b = ctx.bounds(shape[0])
    out_b = ctx.bounds(out_shape[0])
    r = ctx.rank
    mlo, mhi = in_b[r]
    sin = contiguous_strides((mhi - mlo,) + shape[1:])
    if src_strides is not None:
        sin = [int(v) for v in src_strides]
    sstr = [sin[k] * steps[k] for k in range(len(shape))]
    inner_off = sum(starts[k] * sin[k] for k in range(1, len(shape)))
    lo, hi = out_b[r]
    loc_out = (hi - lo,) + out_shape[1:]
    out = _empty(int(np.prod(loc_out)) * es, data.device)
    ostr = contiguous_strides(loc_out)

    def rows_from(src_lo, src_hi, q_lo, q_hi):
        """Output rows i in [q_lo, q_hi) whose input row lies in [src_lo, src_hi)."""
        s0, st = starts[0], steps[0]
        ilo, ihi = q_lo, q_hi
        if st > 0:
            ilo = max(ilo, -((s0 - src_lo) // st))          # ceil((src_lo - s0) / st)
            ihi = min(ihi, -((s0 - src_hi) // st))
        else:
            ilo = max(ilo, (s0 - src_hi) // (-st) + 1)        # s0 + i*st <= src_hi - 1
            ihi = min(ihi, (s0 - src_lo) // (-st) + 1)        # s0 + i*st >= src_lo
        return ilo, max(ilo, ihi)

    def copy_rows(i0, i1, dst, dst_off, dst_strides):
        n = i1 - i0
        if n <= 0:
            return 0
        src_row = starts[0] + i0 * steps[0] - mlo
        shp = (n,) + out_shape[1:]
        backend.copy_strided(data, (src_row * sin[0] + inner_off) * es, dst, dst_off, shp, sstr,
                             dst_strides, es)
        return int(np.prod(shp)) * es

    if ctx.world_size == 1:
        copy_rows(0, out_shape[0], out, 0, ostr)
        return out
    send_sizes, blocks = [], []
    for q in range(ctx.world_size):
        qlo, qhi = out_b[q]
        i0, i1 = rows_from(mlo, mhi, qlo, qhi)
        blocks.append((i0, i1))
        send_sizes.append((i1 - i0) * int(np.prod(out_shape[1:])) * es)
    send = _empty(sum(send_sizes), data.device)
    off = 0
    for (i0, i1), nb in zip(blocks, send_sizes):
        if nb:
            copy_rows(i0, i1, send, off, contiguous_strides((i1 - i0,) + out_shape[1:]))
        off += nb
    recv_sizes, rblocks = [], []
    for s_ in range(ctx.world_size):
        slo, shi = in_b[s_]
        i0, i1 = rows_from(slo, shi, lo, hi)
        rblocks.append((i0, i1))
        recv_sizes.append((i1 - i0) * int(np.prod(out_shape[1:])) * es)
    recv = all_to_all_bytes(ctx, send, send_sizes, recv_sizes, _unit(es))
    off = 0
    for (i0, i1), nb in zip(rblocks, recv_sizes):
        if nb:
            out[(i0 - lo) * ostr[0] * es:(i1 - lo) * ostr[0] * es].copy_(recv[off:off + nb])
        off += nb
    return out


def reslab_counts(ctx, data, counts, rowbytes):
    """Rows held raggedly (rank r holds counts[r] consecutive rows, in rank
    order) -> the standard slabs ctx.bounds(sum(counts)).  One all-to-all."""
    if ctx.world_size == 1:
        return data
    starts = np.r_[0, np.cumsum(counts)].astype(np.int64)
    ob = [(int(starts[q]) * rowbytes, int(starts[q + 1]) * rowbytes) for q in range(ctx.world_size)]
    nb = [(lo * rowbytes, hi * rowbytes) for lo, hi in ctx.bounds(int(starts[-1]))]
    r = ctx.rank
    mlo, mhi = ob[r]
    send_sizes = [max(0, min(mhi, qhi) - max(mlo, qlo)) for qlo, qhi in nb]
    tlo, thi = nb[r]
    recv_sizes = [max(0, min(thi, shi) - max(tlo, slo)) for slo, shi in ob]
    return all_to_all_bytes(ctx, data, send_sizes, recv_sizes, _unit(rowbytes))


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


def concat_rows_sharded(ctx, a, a_rows, b, b_rows, rowbytes):
    """This rank's slab of concatenate((A, B), axis=0) for row-sharded A and B.

    The global byte sequence is A's then B's; every rank sends each peer the
    parts of its two slabs that fall in the peer's output slab (one
    all-to-all) and places what it receives by global offset.
    """
    out_rows = a_rows + b_rows
    if ctx.world_size == 1:
        out = _empty(out_rows * rowbytes, a.device)
        out[:a.numel()].copy_(a)
        out[a.numel():].copy_(b)
        return out
    r = ctx.rank
    ab, bb, ob = ctx.bounds(a_rows), ctx.bounds(b_rows), ctx.bounds(out_rows)

    def pieces(s, q):
        """(global row lo, hi, source tensor, source row lo) sent from rank s to rank q."""
        qlo, qhi = ob[q]
        out = []
        lo, hi = max(ab[s][0], qlo), min(ab[s][1], qhi)
        if hi > lo:
            out.append((lo, hi, "a", lo - ab[s][0]))
        lo, hi = max(a_rows + bb[s][0], qlo), min(a_rows + bb[s][1], qhi)
        if hi > lo:
            out.append((lo, hi, "b", lo - a_rows - bb[s][0]))
        return out

    src = {"a": a, "b": b}
    send_parts, send_sizes = [], []
    for q in range(ctx.world_size):
        ps = pieces(r, q)
        send_sizes.append(sum(hi - lo for lo, hi, _, _ in ps) * rowbytes)
        send_parts += [src[t][o * rowbytes:(o + hi - lo) * rowbytes] for lo, hi, t, o in ps]
    import torch
    send = torch.cat(send_parts) if send_parts else _empty(0, a.device)
    recv_pieces = [pieces(s_, r) for s_ in range(ctx.world_size)]
    recv_sizes = [sum(hi - lo for lo, hi, _, _ in ps) * rowbytes for ps in recv_pieces]
    recv = all_to_all_bytes(ctx, send, send_sizes, recv_sizes, _unit(rowbytes))
    mlo = ob[r][0]
    out = _empty((ob[r][1] - mlo) * rowbytes, a.device)
    off = 0
    for ps in recv_pieces:
        for lo, hi, _, _ in ps:
            n = (hi - lo) * rowbytes
            out[(lo - mlo) * rowbytes:(lo - mlo) * rowbytes + n].copy_(recv[off:off + n])
            off += n
    return out
