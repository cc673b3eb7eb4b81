"""Benchmark of the mi355x mode's hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C1|C3|C4|C5|target64]

One "step" = one pass of the hot path over one batch of synthetic input,
resident in HBM before timing starts.  Default workload (BASELINE.json
configs[1], "C2"): float32 (2000, 512, 512) time series per GPU, key = time
(split 1); swap((0,), (0,1)) to key = voxel, then mean and std over time
(axis 2) -- the three calls a bolt user makes, each returning its result to
the host as the reference does.

`value` = algorithmic bytes of all ranks / wall time of K steps (max over
ranks), GB/s:  swap 2*N*s, each stat N*s + outputs.  `roofline` is the
dominant kernel (the swap's permute) measured with hipEvents on the stream it
runs on; `stats_roofline` the same for the reduction kernels of mean / std;
traffic comes from rocprofv3 --pmc child runs (FETCH_SIZE, WRITE_SIZE).

Sub-records of the default run (same JSON line; `value` stays C2's):
  configs   C1, C3, C4 and C5 (BASELINE configs[0], [2..4]) on their GLOBAL
            shapes (strong scaling: N slabs of the leading axis), a few steps
            each: value, per-op time, fraction of HBM peak, PMC traffic;
  target64  BASELINE.json's target, swap + mean/std of a 64 GiB float32 4-D
            array (1 GPU only).
Every op of every step is checked after timing (`ck`): permutes, chunk /
unchunk / keys_to_values / values_to_keys bit for bit against torch on the
global array rebuilt from each rank's seed, statistics against a float64
truth at the stated tolerance.  `cpu_baseline` times the oracle's restatement
of the reference Spark path and the local mode's numpy calls in a child
process that never touches the GPU.

The line holds numbers and short codes only (profiles/BENCH_FIELDS.md is the
legend), ordered so that the driver's kept tail holds every sub-record; the
prose goes to the detail file named in `detail`.

N GPUs: `python bench.py --gpus N` starts the N rank processes itself (one
per GPU, before anything touches the GPU; rank 0's JSON line is relayed), or
runs as one rank of `torch.distributed.run --nproc-per-node N ... --gpus N`.
A --gpus that differs from WORLD_SIZE, or more GPUs than are visible, exits 2.
The headline scales weakly (the leading axis grows with N); the swap becomes
pack -> all-to-all -> unpack over RCCL, sharded-axis statistics all_gather
their partial states.  Rank 0 runs under rocprofv3 --kernel-trace --stats
(rocprof_rank0) and a marked pass attributes its kernels to op calls.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBPS = 6290.0      # measured float4 copy on MI355X (MI355X_MICROARCH.md), SURVEY 8(d)
XGMI_LINK_GBPS = 153.0      # per link, per direction
METRIC = "swap/transpose GB/s + stat-reduce GB/s, % of HBM/xGMI roofline, 1-8 GPUs"

CONFIGS = {
    # name: (shape, dtype, split, scaling, short workload code)
    #   weak:   ``shape`` is one rank's slab; the global leading axis is shape[0] * N
    #   strong: ``shape`` is BASELINE.json's global array, cut into N slabs of
    #           its leading axis (construct.py:66-69 partitions a fixed array)
    "C1": ((100, 64, 64), np.float64, 1, "strong",
           "C1 f64 (100,64,64) key 0: swap((0,),(0,)) + sum/mean/var/std at axis None and (0,)"),
    "C2": ((2000, 512, 512), np.float32, 1, "weak",
           "C2 f32 (2000,512,512)/GPU key=time: swap((0,),(0,1)) + mean/std(axis=2)"),
    "C3": ((4096, 256, 256, 32), np.float32, 2, "strong",
           "C3 f32 (4096,256,256,32) keys (0,1): swap((0,),(0,)) + .T"),
    "C4": ((10000, 1024, 1024), np.uint16, 1, "strong",
           "C4 u16 (10000,1024,1024) key 0: swap((0,),(0,)) + chunk('150') -> unchunk + var(axis=0)"),
    "C5": ((64, 64, 64, 64, 64), np.float64, 3, "strong",
           "C5 f64 64^5 keys (0,1,2): .T + transpose(2,0,4,1,3) + chunk((16,16),pad 2) -> unchunk / "
           "keys_to_values((2,)) / values_to_keys((0,))"),
    "target64": ((8192, 256, 256, 32), np.float32, 2, "weak",
                 "target64 f32 (8192,256,256,32)=64 GiB/GPU keys (0,1): swap((0,),(0,)) + mean/std(axis=0)"),
}
SUB_CONFIGS = ("C1", "C3", "C4", "C5")  # sub-records of the default run


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) to measure on; without WORLD_SIZE in the environment, N > 1 "
                         "starts the N rank processes itself (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=None)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc traffic passes")
    ap.add_argument("--no-rocprof", action="store_true",
                    help="N > 1: do not run rank 0 under rocprofv3 --kernel-trace --stats")
    ap.add_argument("--no-target64", action="store_true",
                    help="skip the 64 GiB north_star sub-record of the default (C2, 1 GPU) run")
    ap.add_argument("--target-steps", type=int, default=5)
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C1/C3/C4/C5 sub-records of the default (C2) run")
    ap.add_argument("--config-steps", type=int, default=3)
    ap.add_argument("--no-checks", action="store_true", help="skip the post-timing result checks")
    ap.add_argument("--no-sweeps", action="store_true",
                    help="N > 1: skip the all-to-all size sweep and the swap's pipeline-depth sweep")
    ap.add_argument("--detail", default=None,
                    help="file for the full record with its prose (default gpurun_out/bench_detail_n<N>.json)")
    # internal: rocprofv3 child, CPU-baseline child, rehearsal shapes (JSON {config: shape}: a weak
    # config's per-rank slab, a strong config's global array)
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--shapes", "--shard-shapes", dest="shapes", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def config_of(args, cfg, world=1):
    """(global shape, dtype, split, scaling, workload code) of a config at
    ``world`` ranks; --shapes (rehearsals on small data) overrides the shape."""
    shape, dtype, split, scaling, desc = CONFIGS[cfg]
    if args.shapes:
        over = json.loads(args.shapes)
        if cfg in over:
            shape = tuple(int(s) for s in over[cfg])
            desc = "REHEARSAL %s: %s" % (str(shape).replace(" ", ""), desc)
    if scaling == "weak":
        shape = (shape[0] * world,) + tuple(shape[1:])
    return tuple(shape), dtype, split, scaling, desc


def slab_shapes(gshape, world):
    """Every rank's slab shape of a global array (MI355XContext.bounds: array_split order)."""
    base, extra = divmod(int(gshape[0]), world)
    return [(base + (1 if r < extra else 0),) + tuple(gshape[1:]) for r in range(world)]


# ----------------------------------------------------------------- launcher --

def rehearsal_knobs():
    """BOLT_AMD_BENCH_BACKEND=gloo with BOLT_AMD_BENCH_DEVICE=<cuda index | cpu>:
    several ranks on one device, records exchanged through the host by a test
    executor (RCCL refuses two ranks on one GPU) -- a rehearsal of the N-GPU
    code path, never a measurement."""
    return (os.environ.get("BOLT_AMD_BENCH_BACKEND", "nccl") != "nccl"
            and "BOLT_AMD_BENCH_DEVICE" in os.environ)


def visible_gpus():
    import torch
    return torch.cuda.device_count()  # counts devices without initialising HIP (this image)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) without WORLD_SIZE: start N fresh rank
    processes of this script, rank r on GPU r, rendezvous on 127.0.0.1 --
    before this process touches the GPU.  Rank 0's stdout (the JSON line) is
    relayed; the exit status is the worst rank's.  If a rank fails, the others
    are stopped after a grace period (a peer blocked in an exchange would
    otherwise wait out its communicator timeout)."""
    import signal
    import subprocess
    import threading
    if not rehearsal_knobs():
        ndev = visible_gpus()
        if n > ndev:
            sys.stderr.write("bench.py: --gpus %d asked, %d GPU(s) visible: refusing to measure fewer GPUs "
                             "than asked (rehearsals on one GPU set BOLT_AMD_BENCH_BACKEND=gloo and "
                             "BOLT_AMD_BENCH_DEVICE)\n" % (n, ndev))
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", ROLE_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   BOLT_AMD_BENCH_LAUNCHER="bench.py --gpus %d" % n)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    out = []
    reader = threading.Thread(target=lambda: out.extend(procs[0].stdout.read().decode().splitlines(True)))
    reader.start()

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    prev = signal.signal(signal.SIGTERM, lambda *_: (stop(), sys.exit(143)))
    failed_at = None
    try:
        while any(p.poll() is None for p in procs):
            if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
                failed_at = time.time()
                sys.stderr.write("bench.py: a rank failed; stopping the others in 30 s\n")
            if failed_at is not None and time.time() - failed_at > 30:
                stop()
                if time.time() - failed_at > 45:
                    for p in procs:
                        if p.poll() is None:
                            p.kill()
            time.sleep(0.2)
    finally:
        signal.signal(signal.SIGTERM, prev)
    reader.join()
    sys.stdout.write("".join(out))
    sys.stdout.flush()
    worst = 0
    for p in procs:
        rc = p.returncode if p.returncode >= 0 else 128 - p.returncode
        worst = max(worst, rc)
    return worst


# -------------------------------------------------------------- the steps --

def synth_shard(torch, shape, dtype, device, seed):
    """Synthetic input generated in HBM (no host copy): imaging-like floats or random ints."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if np.dtype(dtype) == np.float32:
        t = torch.randn(shape, generator=g, device=device, dtype=torch.float32)
        return t.mul_(50.0).add_(1000.0)
    if np.dtype(dtype) == np.float64:
        return torch.randn(shape, generator=g, device=device, dtype=torch.float64)
    if np.dtype(dtype) == np.uint16:
        t = torch.randint(0, 65536, shape, generator=g, device=device, dtype=torch.int32)
        return t.to(torch.int16)  # same bits as uint16
    raise ValueError(dtype)


def steps_of(cfg, b, world=1):
    """The step of a config as (name, call, algorithmic bytes per rank) in order.

    The first op is the swap / transpose whose kernel is the roofline line.
    Bytes: permute 2*N*s; statistic N*s + outputs; chunk pack
    N*s + packed bytes, unchunk packed bytes + N*s.
    """
    n = int(np.prod(b.shape)) // world   # elements per rank (weak scaling: equal slabs)
    s = b.dtype.itemsize
    N = n * s
    if cfg == "C2":
        out = b.shape[1] * b.shape[2] * 4 // world
        sw = {}
        return [("swap", lambda: sw.__setitem__("s", b.swap((0,), (0, 1))), 2 * N),
                ("mean", lambda: sw["s"].mean(axis=2), N + out),
                ("std", lambda: sw["s"].std(axis=2), N + out)]
    if cfg == "C1":
        sw = {}
        ops = [("swap", lambda: sw.__setitem__("s", b.swap((0,), (0,))), 2 * N)]
        for name in ("sum", "mean", "var", "std"):
            for ax in (None, (0,)):
                nout = 1 if ax is None else n * world // b.shape[1]
                k = 2 if name in ("var", "std") else 1
                ops.append(("%s_%s" % (name, "all" if ax is None else "0"),
                            (lambda name=name, ax=ax: getattr(sw["s"], name)(axis=ax)), N + nout * s * k))
        return ops
    if cfg == "target64":
        out = (n * world // b.shape[0]) * s
        return [("swap", lambda: b.swap((0,), (0,)), 2 * N),
                ("mean", lambda: b.mean(axis=0), N + out),
                ("std", lambda: b.std(axis=0), N + out)]
    if cfg == "C3":
        return [("swap", lambda: b.swap((0,), (0,)), 2 * N),
                ("T", lambda: b.T, 2 * N)]
    if cfg == "C4":
        from bolt_amd.mi355x.plan import ChunkGeometry, getplan
        plan, pad = getplan(b.shape[1:], b.dtype, "150")
        geom = ChunkGeometry(b.shape[1:], plan, pad)
        P = geom.size * (b.shape[0] // world) * s
        # chunk('150') splits only the leading value axis of the (1024, 1024)
        # records: the packed layout IS the dense one, chunk / unchunk are
        # relabellings that move no bytes (ChunkGeometry.is_identity)
        moved = 0 if geom.is_identity() else N + P
        ck = {}
        return [("swap", lambda: b.swap((0,), (0,)), 2 * N),
                ("chunk", lambda: ck.__setitem__("c", b.chunk("150")), moved),
                ("unchunk", lambda: ck.pop("c").unchunk(), moved),
                ("var", lambda: b.var(axis=0), N + (n * world // b.shape[0]) * 8)]
    if cfg == "C5":
        from bolt_amd.mi355x.plan import ChunkGeometry
        P = ChunkGeometry(b.shape[3:], (16, 16), (2, 2)).size * (n // int(np.prod(b.shape[3:]))) * s
        # values_to_keys((0,)): every record's 64 core rows become records of the
        # remaining axis, chunked 16 with padding 2 (76 elements each)
        Pv = ChunkGeometry(b.shape[4:], (16,), (2,)).size * b.shape[3] * (n // int(np.prod(b.shape[3:]))) * s
        ck = {}
        return [("T", lambda: b.T, 2 * N),
                ("transpose", lambda: b.transpose(2, 0, 4, 1, 3), 2 * N),
                ("chunk", lambda: ck.__setitem__("c", b.chunk((16, 16), padding=2)), N + P),
                ("unchunk", lambda: ck["c"].unchunk(), P + N),
                ("keys_to_values", lambda: ck["c"].keys_to_values((2,)), 2 * P),
                ("values_to_keys", lambda: ck.pop("c").values_to_keys((0,)), P + Pv)]
    raise ValueError(cfg)


# ------------------------------------------------------------------ checks --

def checks_of(cfg, b):
    """One check per op of the config's step (steps_of), as (name, call, spec):
      ("perm", perm)             the call returns x.transpose(perm): bit for bit;
      ("stat", name, axis, pre)  a statistic over ``axis`` of x.transpose(pre)
                                 (pre None: of x) against a float64 truth;
      ("packed", vshape, plan, pad)  the call returns a chunked array whose
                                 records are x.reshape(-1, *vshape): its packed
                                 buffer against the reference's slice rule
                                 (chunk.py:574-618) applied with torch slicing,
                                 and its plan / padding.
    x is the global array rebuilt from every rank's seed."""
    from bolt_amd.mi355x.plan import swap_perm, getplan
    nd = len(b.shape)
    rev = list(range(nd))[::-1]
    ident = list(range(nd))
    if cfg == "C1":
        p = swap_perm(nd, b.split, (0,), (0,))[0]
        out = [("swap", lambda: b.swap((0,), (0,)), ("perm", p))]
        for name in ("sum", "mean", "var", "std"):
            for ax in (None, (0,)):
                out.append(("%s_%s" % (name, "all" if ax is None else "0"),
                            lambda name=name, ax=ax: getattr(b.swap((0,), (0,)), name)(axis=ax),
                            ("stat", name, ax, p)))
        return out
    if cfg == "C2":
        # mean / std over time (axis 2) of the swapped array = over axis 0 of x
        return [("swap", lambda: b.swap((0,), (0, 1)), ("perm", swap_perm(nd, b.split, (0,), (0, 1))[0])),
                ("mean", lambda: b.swap((0,), (0, 1)).mean(axis=2), ("stat", "mean", (0,), None)),
                ("std", lambda: b.swap((0,), (0, 1)).std(axis=2), ("stat", "std", (0,), None))]
    if cfg == "C3":
        return [("swap", lambda: b.swap((0,), (0,)), ("perm", swap_perm(nd, b.split, (0,), (0,))[0])),
                ("T", lambda: b.T, ("perm", rev))]
    if cfg == "C4":
        vshape = tuple(b.shape[1:])
        plan, pad = getplan(vshape, b.dtype, "150")
        return [("swap", lambda: b.swap((0,), (0,)), ("perm", swap_perm(nd, b.split, (0,), (0,))[0])),
                ("chunk", lambda: b.chunk("150"), ("packed", vshape, tuple(plan), tuple(pad))),
                ("unchunk", lambda: b.chunk("150").unchunk(), ("perm", ident)),
                ("var", lambda: b.var(axis=0), ("stat", "var", (0,), None))]
    if cfg == "C5":
        v = tuple(b.shape[3:])
        return [("T", lambda: b.T, ("perm", rev)),
                ("transpose", lambda: b.transpose(2, 0, 4, 1, 3), ("perm", [2, 0, 4, 1, 3])),
                ("chunk", lambda: b.chunk((16, 16), padding=2), ("packed", v, (16, 16), (2, 2))),
                ("unchunk", lambda: b.chunk((16, 16), padding=2).unchunk(), ("perm", ident)),
                # keys (k0, k1), values (k2, v0, v1): the moved key is one whole chunk
                ("keys_to_values", lambda: b.chunk((16, 16), padding=2).keys_to_values((2,)),
                 ("packed", (b.shape[2],) + v, (b.shape[2], 16, 16), (0, 2, 2))),
                # keys (k0, k1, k2, v0), values (v1,)
                ("values_to_keys", lambda: b.chunk((16, 16), padding=2).values_to_keys((0,)),
                 ("packed", v[1:], (16,), (2,)))]
    if cfg == "target64":
        return [("swap", lambda: b.swap((0,), (0,)), ("perm", swap_perm(nd, b.split, (0,), (0,))[0])),
                ("mean", lambda: b.mean(axis=0), ("stat", "mean", (0,), None)),
                ("std", lambda: b.std(axis=0), ("stat", "std", (0,), None))]
    raise ValueError(cfg)


def _int_type(torch, itemsize):
    return {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[itemsize]


def _empty_cache(torch, dev):
    if dev.type == "cuda":
        torch.cuda.empty_cache()


CHECK_CHUNK = 4 << 30  # bytes of the rebuilt array compared / reduced at a time


def perm_check(torch, res, perm, gshape, dtype, ctx, dev):
    """True if this rank's slab of ``res`` equals x.transpose(perm), x the
    global array ``gshape`` whose rank-r slab is synth_shard(seed 1234 + r)."""
    world, es = ctx.world_size, np.dtype(dtype).itemsize
    idt = _int_type(torch, es)
    slabs = slab_shapes(gshape, world)
    oshape = [gshape[p] for p in perm]
    got = res._data.view(idt)
    a, j = perm[0], perm.index(0)
    if world == 1 or a == 0:
        # this rank's own rows, permuted: compared in chunks of output rows
        x = synth_shard(torch, slabs[ctx.rank], dtype, dev, 1234 + ctx.rank).view(idt).permute(*perm)
        row = int(np.prod(x.shape[1:]))
        step = max(1, CHECK_CHUNK // max(1, row * es))
        ok = got.numel() == x.numel()
        for lo in range(0, x.shape[0], step):
            hi = min(x.shape[0], lo + step)
            ok = ok and bool(torch.equal(got[lo * row:hi * row], x[lo:hi].contiguous().reshape(-1)))
        del x
        return ok
    lo, hi = ctx.bounds(oshape[0])[ctx.rank]
    want = torch.empty([hi - lo] + oshape[1:], dtype=idt, device=dev)
    for r, (rlo, rhi) in enumerate(ctx.bounds(gshape[0])):
        x = synth_shard(torch, slabs[r], dtype, dev, 1234 + r).view(idt)
        want.narrow(j, rlo, rhi - rlo).copy_(x.narrow(a, lo, hi - lo).permute(*perm))
        del x
    ok = got.numel() == want.numel() and bool(torch.equal(got, want.reshape(-1)))
    del want
    return ok


def _axis_slices(d, s, p):
    """getslices (chunk.py:574-618) on one axis: chunk j = [j s - (j>0) p, j s + s + p) clipped."""
    out, j = [], 0
    while j * s < d:
        out.append(slice(max(0, j * s - (p if j else 0)), min(d, j * s + s + p)))
        j += 1
    return out


def packed_ref(torch, rec, vshape, plan, pad):
    """(records, *vshape) tensor -> its packed chunk layout by torch slicing:
    each record's chunks back to back in chunk-id (product) order, each a
    dense box (test_gpu_large.py's rule, independent of plan.ChunkGeometry)."""
    from itertools import product
    sl = [_axis_slices(vshape[k], plan[k], pad[k]) for k in range(len(vshape))]
    parts = [rec[(slice(None),) + tuple(c)].reshape(rec.shape[0], -1) for c in product(*sl)]
    return torch.cat(parts, dim=1).reshape(-1)


def packed_check(torch, res, vshape, plan, pad, gshape, dtype, ctx, dev):
    """True if the chunked array ``res`` has plan / padding (plan, pad) and
    this rank's packed bytes equal the slice rule on its records of x (records
    never cross GPUs), compared in batches of records."""
    if tuple(res.plan) != tuple(plan) or tuple(res.padding) != tuple(pad):
        return False
    es = np.dtype(dtype).itemsize
    idt = _int_type(torch, es)
    slab = slab_shapes(gshape, ctx.world_size)[ctx.rank]
    x = synth_shard(torch, slab, dtype, dev, 1234 + ctx.rank).view(idt).reshape((-1,) + tuple(vshape))
    got = res._packed.view(idt)
    rec = int(np.prod(vshape))
    batch = max(1, CHECK_CHUNK // max(1, 2 * rec * es))
    ok, off = True, 0
    for lo in range(0, x.shape[0], batch):
        want = packed_ref(torch, x[lo:lo + batch], vshape, plan, pad)
        n = want.numel()
        ok = ok and off + n <= got.numel() and bool(torch.equal(got[off:off + n], want))
        off += n
        del want
    del x
    return ok and off == got.numel()


def _as_f64(torch, t, dtype):
    if np.dtype(dtype) == np.uint16:
        return (t.to(torch.int32) & 0xFFFF).to(torch.float64)
    return t.to(torch.float64)


def stat_truth(torch, name, axis, pre, gshape, dtype, world, dev):
    """(float64 truth, scale) of statistic ``name`` over ``axis`` of
    x.transpose(pre) on the device, x the global array rebuilt from every
    rank's seed.  Small arrays are rebuilt whole; otherwise (pre None, axis
    (0,)) each rank's rows are regenerated and reduced in chunks, merged with
    Chan's update.  ``scale`` is the tolerance's absolute term: max|x| (mean),
    sum|x| (sum), max|truth| (var / std)."""
    slabs = slab_shapes(gshape, world)
    total = int(np.prod(gshape)) * 8
    if total <= (1 << 30):
        x = torch.cat([_as_f64(torch, synth_shard(torch, slabs[r], dtype, dev, 1234 + r), dtype)
                       for r in range(world)], 0)
        if pre is not None:
            x = x.permute(*pre)
        dims = tuple(range(x.dim())) if axis is None else tuple(axis)
        if name == "sum":
            return x.sum(dims), x.abs().sum(dims)
        if name == "mean":
            return x.mean(dims), x.abs().max()
        v = x.var(dims, unbiased=False)
        t = v if name == "var" else v.sqrt()
        return t, t.abs().max()
    if pre is not None or tuple(axis or ()) != (0,) or name not in ("mean", "var", "std"):
        raise ValueError("stat_truth: a large array is reduced over its leading axis only")
    row = int(np.prod(gshape[1:]))
    step = max(1, CHECK_CHUNK // (row * 8))
    n, mean, m2, xmax = 0, None, None, 0.0
    for r in range(world):
        x = synth_shard(torch, slabs[r], dtype, dev, 1234 + r)
        for lo in range(0, slabs[r][0], step):
            c = _as_f64(torch, x[lo:lo + step], dtype)
            k = c.shape[0]
            cm = c.mean(0)
            cq = ((c - cm) ** 2).sum(0)
            xmax = max(xmax, float(c.abs().max()))
            if mean is None:
                n, mean, m2 = k, cm, cq
            else:
                tot = n + k
                d = cm - mean
                mean = mean + d * (k / tot)
                m2 = m2 + cq + d * d * (n * k / tot)
                n = tot
            del c, cq
        del x
    if name == "mean":
        return mean, xmax
    v = m2 / n
    t = v if name == "var" else v.sqrt()
    return t, float(t.abs().max())


def stat_within(got, truth, scale, name):
    """The parity rule of SURVEY.md 8(c) against a float64 truth:
    |got - truth| <= rtol*|truth| + rtol*scale, rtol 1e-12 for float64 outputs
    and 1e-6 for float32; for var / std the absolute term is eps-sized
    (rtol*eps*max|truth|), so the bar stays relative.  Returns (ok, max error
    relative to rtol*|truth| + atol)."""
    got = np.asarray(got)
    rtol = 1e-12 if got.dtype == np.float64 else 1e-6
    t = np.asarray(truth, dtype=np.float64).reshape(got.shape)
    sc = float(np.max(np.asarray(scale, dtype=np.float64)))
    if name in ("var", "std"):
        atol = rtol * np.finfo(got.dtype).eps * sc
    elif name == "sum":
        atol = rtol * np.asarray(scale, dtype=np.float64).reshape(got.shape)
    else:
        atol = rtol * sc
    err = np.abs(got.astype(np.float64) - t)
    bar = rtol * np.abs(t) + atol
    return bool(np.all(err <= bar)), float(np.max(err / np.maximum(bar, 1e-300))) if err.size else 0.0


def run_checks(torch, cfg, b, ctx, dev, gshape, dtype, world):
    """Every check of checks_of(cfg) on this rank -> ({name: verdict}, all ok);
    all ranks' verdicts merged (a mismatch on any rank is a mismatch).
    Verdicts: "exact" / "MISMATCH" (data movement), "ok <e>" / "FAIL <e>"
    (statistics; e = largest error as a fraction of the tolerance bar)."""
    res = {}
    for name, call, spec in checks_of(cfg, b):
        r = call()
        if spec[0] == "perm":
            ok = perm_check(torch, r, spec[1], gshape, dtype, ctx, dev)
            detail = "exact" if ok else "MISMATCH"
        elif spec[0] == "packed":
            ok = packed_check(torch, r, spec[1], spec[2], spec[3], gshape, dtype, ctx, dev)
            detail = "exact" if ok else "MISMATCH"
        else:
            _, stat, axis, pre = spec
            truth, scale = stat_truth(torch, stat, axis, pre, gshape, dtype, world, dev)
            ok, worst = stat_within(r, truth.cpu().numpy(), scale.cpu().numpy() if hasattr(scale, "cpu") else scale,
                                    stat)
            detail = "%s %.3g" % ("ok" if ok else "FAIL", worst)
        del r
        _empty_cache(torch, dev)
        res[name] = (ok, detail)
    if world > 1:
        import torch.distributed as dist
        flags = torch.tensor([0.0 if ok else 1.0 for ok, _ in res.values()], dtype=torch.float64)
        dist.all_reduce(flags, op=dist.ReduceOp.MAX)
        for (name, (ok, detail)), f in zip(list(res.items()), flags.tolist()):
            if f and ok:
                res[name] = (False, "MISMATCH on another rank")
    return {name: detail for name, (ok, detail) in res.items()}, all(ok for ok, _ in res.values())


def exchange_check(torch, cfg, b, ctx, dev, gshape, dtype):
    """Bit-exact check of the first op of the step (the swap / .T that crosses
    GPUs): True if every byte of this rank's slab agrees with the global array
    rebuilt from every rank's seed."""
    name, call, spec = checks_of(cfg, b)[0]
    r = call()
    ok = perm_check(torch, r, spec[1], gshape, dtype, ctx, dev)
    del r
    return ok


# ------------------------------------------------------------ PMC traffic --

def run_child(cmd, timeout, capture=False):
    """Run ``cmd`` in its own process group and return (rc, stdout bytes); on
    timeout the whole group is killed (a profiler's or a worker pool's
    grandchildren included), and the rc is -9."""
    import signal
    import subprocess
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE if capture else subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout)
        return p.returncode, out or b""
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.communicate()
        return -9, b""


def _library_kernel(name):
    import re
    return re.search(r"(?<![A-Za-z0-9_])k_(transpose|rowcopy|generic|red|recmap|record|gather)", name) is not None


def pmc_traffic(cfg, args, nops, warmup=1, steps=2):
    """HBM bytes per call of each op of a config's step, from rocprofv3 PMC counters.

    Two child runs of this script (--pmc-child: the whole step, warmup+steps
    times, a torch spin kernel dispatched before every op as a marker), one
    counter each (FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2: they do not fit
    one pass), with nothing but --pmc on the rocprofv3 line.  The library's
    kernels between two markers belong to one op call.  gfx950 correction
    (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of wide
    streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B stores.
    Counters are in KiB.  Returns ([bytes per call of op k] or None, note).
    """
    import csv
    import glob
    import shutil
    import tempfile
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None, "rocprofv3 not found"
    per = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        out = tempfile.mkdtemp(prefix="bm_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [rp, "--pmc", ctr, "-d", out, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--config", cfg, "--steps", str(steps),
               "--warmup", str(warmup), "--pmc-child"]
        if args.shapes:
            cmd += ["--shapes", args.shapes]
        try:
            rc, _ = run_child(cmd, timeout=600)
        except OSError as e:  # profiler unavailable: report null
            rc = "%s" % type(e).__name__
        if rc != 0:
            shutil.rmtree(out, ignore_errors=True)
            return None, "rocprofv3 --pmc %s failed: %s" % (ctr, rc)
        disp = {}  # dispatch id -> [kernel name, counter value in bytes]
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                d = disp.setdefault(int(r.get("Dispatch_Id") or len(disp)), [r.get("Kernel_Name", ""), 0.0])
                if r.get("Counter_Name") == ctr:
                    d[1] += float(r["Counter_Value"]) * 1024
        shutil.rmtree(out, ignore_errors=True)
        seg, vals = -1, []
        for _, (name, v) in sorted(disp.items()):
            if "spin_kernel" in name:
                seg += 1
                vals.append(0.0)
            elif seg >= 0 and _library_kernel(name):
                vals[seg] += v
        if len(vals) != (warmup + steps) * nops:
            return None, "%s: %d op segments, expected %d" % (ctr, len(vals), (warmup + steps) * nops)
        per[ctr] = [float(np.median(vals[k::nops])) for k in range(nops)]
    traffic = [2.0 * f + w for f, w in zip(per["FETCH_SIZE"], per["WRITE_SIZE"])]
    return traffic, "per call: 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE over the library's kernels"


# ------------------------------------------------ rocprofv3 at N > 1 ranks --

PROFILED_ENV = "BOLT_AMD_BENCH_PROFILED"  # set in rank 0's profiled child: its trace directory


def rocprof_path():
    import shutil
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return rp if os.path.exists(rp) else None


def rocprof_wanted(args, world, where):
    """True on EVERY rank of an N-rank GPU run whose rank 0 runs under
    rocprofv3 (all ranks then run the marked pass, which holds collectives)."""
    return (world > 1 and not args.no_rocprof and not args.pmc_child and where != "cpu"
            and os.environ.get("BOLT_AMD_BENCH_ROCPROF", "1") != "0" and rocprof_path() is not None)


def _die_with_parent():
    """preexec: the child gets SIGKILL when the wrapper dies (PR_SET_PDEATHSIG)."""
    import ctypes
    import signal
    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGKILL), 0, 0, 0)
    except OSError:
        pass


def rocprof_rank0(argv, world):
    """Rank 0 of an N-rank run, before anything touches the GPU: run this
    script again as rank 0 (same environment: it joins the rendezvous) under
    ``rocprofv3 --kernel-trace --stats`` -- a fresh child, the program after
    ``--`` -- then add the trace's numbers (rocprof_windows) to its JSON line
    and relay it.  Exit status: the child's."""
    import glob
    import shutil
    import signal
    import subprocess
    import tempfile
    out = tempfile.mkdtemp(prefix="bm_rocprof_", dir=os.environ.get("TMPDIR", "/tmp"))
    env = dict(os.environ)
    env[PROFILED_ENV] = out
    cmd = [rocprof_path(), "--kernel-trace", "--stats", "-d", out, "-o", "rank0", "--output-format", "csv",
           "--", sys.executable, os.path.abspath(__file__)] + list(argv)
    progress("rank 0 under rocprofv3 --kernel-trace --stats (%s)" % out)
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, preexec_fn=_die_with_parent)
    prev = signal.signal(signal.SIGTERM, lambda *_: p.terminate())
    try:
        raw, _ = p.communicate()
    finally:
        signal.signal(signal.SIGTERM, prev)
    text = raw.decode("utf-8", "replace")
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        sys.stdout.write(text)
        sys.stdout.flush()
        shutil.rmtree(out, ignore_errors=True)
        return p.returncode or 1
    line = json.loads(lines[-1])
    marks = line.pop("rocprof_marks", None)
    info = line.pop("rocprof_info", {})
    try:
        traces = sorted(glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True))
        if not traces:
            raise RuntimeError("no kernel trace written")
        kept = None
        stats = sorted(glob.glob(os.path.join(out, "**", "*kernel_stats.csv"), recursive=True))
        if stats:
            keep_dir = os.path.join(HERE, "gpurun_out")
            os.makedirs(keep_dir, exist_ok=True)
            kept = os.path.join(keep_dir, "bench_rocprof_n%d_kernel_stats.csv" % world)
            shutil.copyfile(stats[0], kept)
            kept = os.path.relpath(kept, HERE)
        merge_rocprof(line, rocprof_windows(traces[0], marks, info, world), kept)
    except Exception as e:  # the measurement stands; the profile is reported missing
        line["rocprof"] = {"error": "%s: %s" % (type(e).__name__, e)}
    shutil.rmtree(out, ignore_errors=True)
    if line.get("detail"):
        try:
            path = os.path.join(HERE, line["detail"])
            d = json.load(open(path))
            d["rocprof"] = line.get("rocprof")
            json.dump(d, open(path, "w"), indent=1)
        except (OSError, ValueError):
            pass
    sys.stdout.write(json.dumps(line, separators=(",", ":")) + "\n")
    sys.stdout.flush()
    return 0


def _short_kernel(name):
    n = name.replace("(anonymous namespace)::", "")
    return n[5:] if n.startswith("void ") else n


def kernel_class(name):
    """'marker' (torch's spin kernel), 'rccl' (RCCL's device kernels,
    ncclDevKernel_* / ncclKernel_*), 'lib' (libbolt_mi355x), 'blit' (the HIP
    runtime's copy / fill kernels: hipMemcpyAsync on a shader), 'torch' (at::)
    or 'other' (counted with RCCL's time: within a swap call nothing else
    launches kernels)."""
    import re
    n = _short_kernel(name)
    if "spin_kernel" in n:
        return "marker"
    if re.search(r"nccl|rccl", n, re.I):
        return "rccl"
    if re.match(r"k_[a-z]", n):
        return "lib"
    if "rocclr" in n or "__amd" in n:
        return "blit"
    if n.startswith("at::") or "at::native" in n or "at::cuda" in n:
        return "torch"
    return "other"


def _union_ms(iv):
    """Length of the union of [start, end) intervals (ns) in ms."""
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur is not None:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur is not None:
        tot += cur[1] - cur[0]
    return tot / 1e6


def rocprof_windows(trace_csv, marks, info, world):
    """Per op of the marked pass, from rank 0's kernel trace: the kernels that
    ran between the op call's two marker kernels (on the current stream; the
    exchange's RCCL kernels on the RCCL stream start after the call's first
    marker and end before its last unpack, so before the second marker).

    ``marks``: [[cfg, [op, ...], steps], ...] in the order the marked pass ran;
    ``info``: {"cfg.op": [peer payload bytes per rank, pack+unpack bytes]}.
    Returns {"cfg.op": {"n": calls, "span": ms between the markers, "rccl":
    union of the RCCL kernels' intervals (ms per call), "rccl_n": RCCL kernels
    per call, "lib": summed library kernel ms per call, "blit": runtime copy
    kernels, and for an exchanging op "xgmi_GBs"/"xgmi_frac" (payload over the
    RCCL time, of (G-1) x 153 GB/s) and "pu_frac" (pack + unpack bytes over the
    library kernels' time, of 8 TB/s)}}."""
    import csv
    rows = []
    for r in csv.DictReader(open(trace_csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kernel_class(r["Kernel_Name"])))
    rows.sort()
    markers = [(a, b) for a, b, c in rows if c == "marker"]
    calls = [("%s.%s" % (cfg, op)) for cfg, ops, steps in (marks or []) for _ in range(int(steps)) for op in ops]
    if len(markers) != 2 * len(calls):
        raise RuntimeError("%d marker kernels in the trace, %d expected" % (len(markers), 2 * len(calls)))
    others = [(a, b, c) for a, b, c in rows if c != "marker"]
    acc = {}
    lo = 0
    for k, label in enumerate(calls):
        w0, w1 = markers[2 * k][1], markers[2 * k + 1][0]
        while lo < len(others) and others[lo][0] < w0:
            lo += 1
        ks = []
        i = lo
        while i < len(others) and others[i][0] < w1:
            ks.append(others[i])
            i += 1
        a = acc.setdefault(label, {"n": 0, "span": 0.0, "rccl": 0.0, "rccl_n": 0, "lib": 0.0, "blit": 0.0})
        a["n"] += 1
        a["span"] += (w1 - w0) / 1e6
        a["rccl"] += _union_ms([(s, e) for s, e, c in ks if c in ("rccl", "other")])
        a["rccl_n"] += sum(1 for _, _, c in ks if c in ("rccl", "other"))
        a["lib"] += sum(e - s for s, e, c in ks if c == "lib") / 1e6
        a["blit"] += sum(e - s for s, e, c in ks if c == "blit") / 1e6
    out = {}
    peak = (world - 1) * XGMI_LINK_GBPS
    for label, a in acc.items():
        n = a["n"]
        o = {"n": n, "span": round(a["span"] / n, 3), "rccl": round(a["rccl"] / n, 3),
             "lib": round(a["lib"] / n, 3)}
        if a["rccl_n"]:
            o["rccl_n"] = round(a["rccl_n"] / float(n), 1)
        if a["blit"]:
            o["blit"] = round(a["blit"] / n, 3)
        payload, local = (info or {}).get(label, (0, 0))
        if payload and o["rccl"] > 0:
            o["xgmi_GBs"] = round(payload / (o["rccl"] / 1e3) / 1e9, 1)
            o["xgmi_frac"] = round(o["xgmi_GBs"] / peak, 4)
        if payload and local and o["lib"] > 0:
            o["pu_frac"] = round(local / (o["lib"] / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
        out[label] = o
    return out


def merge_rocprof(line, ops, stats_file):
    """rocprof_windows' numbers into the record: ``rocprof`` (every op of
    every config, keyed "cfg.op") and the headline swap's RCCL time into
    ``xgmi``."""
    line["rocprof"] = {"rank": 0, "stats": stats_file, "ops": ops}
    head = "%s.%s" % (line.get("config", {}).get("name", "C2"), next(iter(line.get("ops", {"swap": 0}))))
    h = ops.get(head)
    if h and "xgmi" in line:
        line["xgmi"]["rocprof_ms"] = h["rccl"]
        if "xgmi_GBs" in h:
            line["xgmi"]["rocprof_achieved"] = h["xgmi_GBs"]
            line["xgmi"]["rocprof_frac"] = h["xgmi_frac"]
        if "pu_frac" in h:
            line["xgmi"]["pack_unpack_frac"] = h["pu_frac"]


# ------------------------------------------------------------ CPU baseline --

# leading-axis rows of the per-GPU shard timed by local_numpy_baseline (~0.5-1 GB)
LOCAL_SAMPLE_ROWS = {"C3": 64, "C4": 256, "C5": 8, "target64": 64}
C2_SAMPLE_ROWS = 500     # time points of the C2 oracle / numpy / local[8] sample (0.5 GB)
REPS = 3                 # best of 3 after 1 warm-up


def best_of(f, reps=REPS):
    """Best of ``reps`` timed runs of f() after one warm-up: (seconds, result of the best run)."""
    f()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = f()
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, r)
    return best


def local_numpy_baseline(cfg, shape, dtype):
    """The reference local mode's numpy calls (bolt/local/array.py) for the
    config's permute and statistic ops, one host thread, on a slab of the
    leading axis; chunk/unchunk have no local-mode counterpart and are left out."""
    rows = min(shape[0], LOCAL_SAMPLE_ROWS[cfg])
    sample_shape = (rows,) + tuple(shape[1:])
    rng = np.random.default_rng(0)
    if np.dtype(dtype).kind == "u":
        x = rng.integers(0, np.iinfo(dtype).max + 1, size=sample_shape, dtype=dtype)
    else:
        x = rng.standard_normal(sample_shape).astype(dtype)
    nd = x.ndim
    swap01 = (1, 0) + tuple(range(2, nd))
    ops = {"C3": [("swap", lambda: np.ascontiguousarray(x.transpose(1, 2, 0, 3))),
                  ("T", lambda: np.ascontiguousarray(x.T))],
           "C4": [("swap", lambda: np.ascontiguousarray(x.transpose(swap01))),
                  ("var", lambda: x.var(axis=0))],
           "C5": [("T", lambda: np.ascontiguousarray(x.T)),
                  ("transpose", lambda: np.ascontiguousarray(x.transpose(2, 0, 4, 1, 3)))],
           "target64": [("swap", lambda: np.ascontiguousarray(x.transpose(1, 2, 0, 3))),
                        ("mean", lambda: x.mean(axis=0)),
                        ("std", lambda: x.std(axis=0))]}[cfg]
    N = x.nbytes

    def step():
        parts, total = [], 0
        for name, f in ops:
            u = time.perf_counter()
            r = f()
            parts.append("%s %.2fs" % (name, time.perf_counter() - u))
            total += 2 * N if r.size == x.size else N + r.nbytes
            del r
        return parts, total
    el, (parts, total) = best_of(step)
    return {"value": total / el / 1e9, "unit": "GB/s", "cores": 1, "kind": "port", "reps": REPS,
            "brief": "numpy local mode, %s %s slab, 1 core, best of 3" % (np.dtype(dtype).name,
                                                                        str(sample_shape).replace(" ", "")),
            "sample": "the reference local mode's numpy calls on %s %s (a leading-axis slab of the "
                      "shard; chunk/unchunk not included), best of %d after 1 warm-up: %s"
                      % (np.dtype(dtype).name, str(sample_shape), REPS, " + ".join(parts)),
            "host_cpus": os.cpu_count()}


def c1_cpu_baseline(shape, dtype):
    """C1 in full on one host core: the oracle's record-level restatement of
    the reference Spark path (8 partitions) and the reference local mode's
    numpy calls; each timed run repeats the step ~3 s (spark) / ~1 s (numpy),
    best of 3 after 1 warm-up."""
    from oracle import bolt_oracle as O
    rng = np.random.default_rng(0)
    x = rng.standard_normal(shape).astype(dtype)
    N = x.nbytes
    total = 2 * N + 8 * N  # swap + 8 statistics reading the array (outputs are < 33 KB)

    def spark():
        rs = O.parallelize(x, axis=(0,), npartitions=8)
        s = O.swap(rs, (0,), (0,))
        O.sum_(s, None)
        O.sum_(s, (0,))
        for name in ("mean", "variance", "stdev"):
            O.stat(s, name, None)
            O.stat(s, name, (0,))

    def local():
        y = np.ascontiguousarray(x.transpose(1, 0, 2))
        for f in (y.sum, y.mean, y.var, y.std):
            f()
            f(axis=0)

    out = {}
    for name, f, budget in (("spark", spark, 3.0), ("local", local, 1.0)):
        t0, k = time.perf_counter(), 0
        while time.perf_counter() - t0 < budget / 4:  # size a run
            f()
            k += 1
        reps = max(1, int(k * 4))
        el, _ = best_of(lambda: [f() for _ in range(reps)])
        out[name] = (total * reps / el / 1e9, reps)
    return {"value": out["spark"][0], "unit": "GB/s", "cores": 1, "kind": "port", "reps": REPS,
            "brief": "oracle Spark-path port, whole C1, 1 core, best of 3",
            "sample": "oracle/bolt_oracle.py record-level Spark path (8 partitions) on the whole C1 input, "
                      "swap + sum/mean/var/std at axis=None and axis=(0,), %d steps per timed run, best of %d "
                      "after 1 warm-up" % (out["spark"][1], REPS),
            "host_cpus": os.cpu_count(),
            "local_numpy": {"value": round(out["local"][0], 3), "unit": "GB/s", "cores": 1, "reps": REPS,
                            "brief": "numpy local mode, whole C1, 1 core",
                            "sample": "the reference local mode's numpy calls on the same input, %d steps per "
                                      "timed run, best of %d after 1 warm-up" % (out["local"][1], REPS)}}


def cpu_baseline(cfg, shape, dtype, rows):
    """Oracle (record-level restatement of the reference Spark path), 1 core,
    bounded sample, best of 3 after 1 warm-up; C2 adds the local
    mode's numpy calls and an OpenMP line on the WHOLE C2 input, and the Spark
    local[8] analogue on the oracle's sample."""
    from oracle import bolt_oracle as O
    if cfg == "C1":
        return c1_cpu_baseline(shape, dtype)
    if cfg != "C2":
        return local_numpy_baseline(cfg, shape, dtype)
    rows = rows or C2_SAMPLE_ROWS
    rng = np.random.default_rng(0)
    full = (1000 + 50 * rng.standard_normal(tuple(shape), dtype=np.float32)).astype(dtype, copy=False)
    x = np.ascontiguousarray(full[:rows])
    sample_shape = x.shape
    rs = O.parallelize(x, axis=(0,), npartitions=8)

    def spark():
        t0 = time.perf_counter()
        s = O.swap(rs, (0,), (0, 1))
        t1 = time.perf_counter()
        O.stat(s, 'mean', axis=2)
        t2 = time.perf_counter()
        O.stat(s, 'stdev', axis=2)
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2

    def local():
        # the reference's local mode (bolt/local/array.py) runs the same three
        # calls as numpy on one host thread: ascontiguousarray(transpose) + mean / std
        u0 = time.perf_counter()
        xs = np.ascontiguousarray(full.transpose(1, 2, 0))
        u1 = time.perf_counter()
        xs.mean(axis=2)
        u2 = time.perf_counter()
        xs.std(axis=2)
        u3 = time.perf_counter()
        del xs
        return u1 - u0, u2 - u1, u3 - u2

    def step_bytes(a):
        N = a.nbytes
        return 2 * N + 2 * (N + a.shape[1] * a.shape[2] * 4)
    ts, tp = best_of(spark)
    ls, lp = best_of(local)
    out = {"value": step_bytes(x) / ts / 1e9, "unit": "GB/s", "cores": 1, "kind": "port", "reps": REPS,
           "brief": "oracle Spark-path port, f32 %s, 1 core, best of 3" % str(sample_shape).replace(" ", ""),
           "sample": "oracle/bolt_oracle.py record-level Spark path (8 partitions) on float32 %s (the first %d "
                     "time points of C2), best of %d after 1 warm-up: swap((0,),(0,1)) %.2fs + mean(axis=2) "
                     "%.2fs + std(axis=2) %.2fs" % ((str(sample_shape), rows, REPS) + tp),
           "host_cpus": os.cpu_count(),
           "local_numpy": {"value": round(step_bytes(full) / ls / 1e9, 3), "unit": "GB/s", "cores": 1,
                           "reps": REPS, "brief": "numpy local mode, whole C2 f32 %s, 1 core, best of 3"
                                                  % str(full.shape).replace(" ", ""),
                           "sample": "the reference local mode's numpy calls on the whole C2 input float32 %s, "
                                     "best of %d after 1 warm-up: transpose %.2fs + mean %.2fs + std %.2fs"
                                     % ((str(full.shape), REPS) + lp)}}
    del rs
    out["spark_local8"] = spark_local8_baseline(x, dtype)
    out["openmp"] = openmp_baseline(full)
    return out


def host_cpu_share():
    """(threads to use, note): the CPUs this process may run on and the
    cgroup's CPU quota.  On the GPU pool one GPU's job gets a share of a large
    host (OMP_NUM_THREADS is set to that share); os.cpu_count() counts the
    whole machine, shared with other jobs."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = omp or (int(quota) if quota else aff)
    note = ("OMP_NUM_THREADS=%d (the CPU share the GPU pool gives one GPU's job; it is set by the pool and "
            "left as is)" % omp if omp else "cgroup CPU quota %.1f" % quota if quota else "CPU affinity")
    return max(1, n), {"host_cpus": os.cpu_count(), "affinity_cpus": aff,
                       "cgroup_cpu_quota": quota, "threads_from": note}


def openmp_baseline(x):
    """The local mode's three calls as OpenMP C on the host cores
    (oracle/c/local_step.c, a port: SURVEY 8(d)'s optional multi-core line),
    on the whole C2 shard; best of 3 after one warm-up."""
    import ctypes
    path = os.path.join(HERE, "oracle", "c", "liblocal_step.so")
    if not os.path.exists(path):
        return {"value": None, "note": "oracle/c/liblocal_step.so not built"}
    lib = ctypes.CDLL(path)
    f32p = ctypes.POINTER(ctypes.c_float)
    for fn in (lib.local_swap, lib.local_mean, lib.local_std):
        fn.argtypes = [f32p, f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    T = x.shape[0]
    P = int(np.prod(x.shape[1:]))
    threads, share = host_cpu_share()
    xc = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty((P, T), np.float32)
    m = np.empty(P, np.float32)
    sd = np.empty(P, np.float32)
    ptr = lambda a: a.ctypes.data_as(f32p)  # noqa: E731

    def step():
        t0 = time.perf_counter()
        lib.local_swap(ptr(xc), ptr(y), T, P, threads)
        t1 = time.perf_counter()
        lib.local_mean(ptr(y), ptr(m), T, P, threads)
        t2 = time.perf_counter()
        lib.local_std(ptr(y), ptr(sd), T, P, threads)
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2
    el, parts = best_of(step)
    N = xc.nbytes
    total = 2 * N + 2 * (N + P * 4)
    out = {"value": round(total / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port", "reps": REPS,
           "brief": "OpenMP local step, %d threads, f32 %s" % (threads, str(x.shape).replace(" ", "")),
           "sample": "oracle/c/local_step.c (OpenMP, the local mode's ascontiguousarray(transpose) + mean + "
                     "std) on float32 %s, best of %d after 1 warm-up: swap %.3fs + mean %.3fs + std %.3fs"
                     % ((str(x.shape), REPS) + parts)}
    out.update(share)
    if threads < (os.cpu_count() or threads):
        out["cores_reason"] = ("%d threads, not os.cpu_count() = %d: %s" % (threads, os.cpu_count(),
                                                                            share["threads_from"]))
    return out


def spark_local8_baseline(x, dtype, workers=8):
    """The Spark local[8] analogue (oracle/spark_local.py): the oracle's record-level
    C2 step with Spark's stage structure on 8 host processes -- 8 map tasks, one
    reduce task per chunk group, and the statistics' single task (their _align
    shuffle has one group) -- shuffles pickled through the parent.  Best of 3
    after 1 warm-up.  Runs in bench.py's CPU-baseline child, which never
    initialises the GPU, so its forked workers inherit no HIP runtime."""
    from oracle import spark_local as SL
    x = np.ascontiguousarray(x)
    el, (t, tasks) = best_of(lambda: SL.c2_step(x, workers=workers)[2:])
    N = x.nbytes
    out = x.shape[1] * x.shape[2] * 4
    total = 2 * N + 2 * (N + out)
    return {"value": round(total / t["total"] / 1e9, 4), "unit": "GB/s", "cores": workers, "reps": REPS,
            "brief": "Spark local[%d] analogue, %d processes, f32 %s" % (workers, workers,
                                                                        str(x.shape).replace(" ", "")),
            "kind": "port, local[%d] analogue" % workers, "host_cpus": os.cpu_count(),
            "sample": "oracle/spark_local.py on float32 %s, best of %d after 1 warm-up: stage 1 (%d map tasks: "
                      "chunk + relabel) %.2fs, stage 2 (%d reduce tasks: rebuild + values_to_keys + unchunk) "
                      "%.2fs, mean(axis=2) %.2fs + std(axis=2) %.2fs (one task each: _align's shuffle has a "
                      "single group, as in the reference)" % (str(x.shape), REPS, tasks["stage1"], t["stage1"],
                                                              tasks["stage2"], t["stage2"], t["mean"], t["std"])}


def cpu_baseline_in_child(args, cfg):
    """cpu_baseline() in a fresh child process of this script that never
    touches the GPU (its local[8] analogue forks workers: never from a process
    with a live HIP runtime)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--config", cfg]
    if args.cpu_sample_rows:
        cmd += ["--cpu-sample-rows", str(args.cpu_sample_rows)]
    if args.shapes:
        cmd += ["--shapes", args.shapes]
    rc, out = run_child(cmd, timeout=900, capture=True)
    try:
        if rc != 0:
            raise RuntimeError("exit status %d" % rc)
        return json.loads(out.decode().strip().splitlines()[-1])
    except (RuntimeError, ValueError, IndexError) as e:
        return {"value": None, "note": "CPU baseline child failed: %s" % e}


# ------------------------------------------------------------------ timing --

class HostEvent(object):
    """torch.cuda.Event's timing interface on the host clock (the CPU rehearsal)."""

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, end):
        return (end.t - self.t) * 1e3


def make_event(dev):
    import torch
    return torch.cuda.Event(enable_timing=True) if dev.type == "cuda" else HostEvent()


LAUNCHES = ("permute", "copy_strided", "gather_rows", "record_gather", "record_scatter", "record_runs", "reduce",
            "reduce_rows", "reduce_state", "reduce_combine")


class KernelClock(object):
    """hipEvent pairs around the library launches of a kernel backend, on the
    stream they run on (torch's current stream), attributed to ``op`` (None:
    not timed).  Event pairs come from a pool made before the timed region."""

    def __init__(self, backend, dev, methods, pool=0):
        self.be, self.dev, self.op = backend, dev, None
        self.pairs = {}
        self.pool = [(make_event(dev), make_event(dev)) for _ in range(pool)]
        self.methods = [m for m in methods if hasattr(backend, m)]
        for m in self.methods:
            setattr(backend, m, self._wrap(getattr(backend, m)))

    def _wrap(self, f):
        def timed(*a, **k):
            if self.op is None:
                return f(*a, **k)
            e0, e1 = self.pool.pop() if self.pool else (make_event(self.dev), make_event(self.dev))
            e0.record()
            r = f(*a, **k)
            e1.record()
            self.pairs.setdefault(self.op, []).append((e0, e1))
            return r
        return timed

    def close(self):
        for m in self.methods:
            self.be.__dict__.pop(m, None)

    def ms(self, op, steps):
        pairs = self.pairs.get(op)
        return sum(a.elapsed_time(z) for a, z in pairs) / steps if pairs else None

    def launches(self, op, steps):
        return len(self.pairs.get(op, ())) / float(steps)


def live_copy_gbps(be, dev, nbytes, reps=7):
    """The box's copy ceiling for the headline kernel's byte count, measured
    here: the library's contiguous copy (bm_copy_strided -> 16-B rowcopy) of
    ``nbytes`` into a second buffer, hipEvents on the launch stream, median of
    ``reps`` after one untimed call.  Algorithmic bytes 2 * nbytes.  None off
    the GPU.  (Run after the timed region; its buffers are freed.)"""
    import torch
    if dev.type != "cuda" or nbytes < (1 << 20):
        return None
    n4 = int(nbytes) // 4
    src = torch.empty(n4 * 4, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1)
    ms = []
    for i in range(reps + 1):
        e0, e1 = make_event(dev), make_event(dev)
        e0.record()
        be.copy_strided(src, 0, dst, 0, [n4], [1], [1], 4)
        e1.record()
        e1.synchronize()
        if i:
            ms.append(e0.elapsed_time(e1))
    del src, dst
    _empty_cache(torch, dev)
    ms.sort()
    return 2.0 * n4 * 4 / (ms[len(ms) // 2] / 1e3) / 1e9


def _stdout_to_stderr(fn):
    """Run fn with file descriptor 1 pointed at 2: the process group's
    transports print connection chatter on stdout ("[Gloo] Rank 0 is connected
    to 7 peer ranks ..."), and stdout must carry only the one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def progress(msg):
    sys.stderr.write("[bench %s] %s\n" % (time.strftime("%H:%M:%S"), msg))
    sys.stderr.flush()


DTYPE_NAMES = {"float32": "f32", "float64": "f64", "uint16": "u16"}
LEGEND = "profiles/BENCH_FIELDS.md"   # what every field of the record means (the prose lives there)


def op_rec(nb, ms, launches=None):
    """Compact per-op record: B algorithmic bytes per rank and call, ms per
    call, frac of the 8 TB/s HBM peak, nl launches per call."""
    o = {"B": int(nb), "ms": round(ms, 4) if ms else None}
    if ms and nb:
        o["frac"] = round(nb / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
    if launches is not None:
        o["nl"] = round(launches, 2)
    return o


def compact_cpu(cb):
    """The CPU baseline's numbers for the stdout record (its prose goes to the detail file)."""
    if not isinstance(cb, dict) or cb.get("value") is None:
        return cb
    out = {"value": round(cb["value"], 4), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
           "sample": cb.get("brief", "")}
    for k in ("local_numpy", "spark_local8", "openmp"):
        v = cb.get(k)
        if isinstance(v, dict):
            out[k] = {"value": v.get("value"), "cores": v.get("cores"), "sample": v.get("brief", "")}
    return out


def detail_path(args, world):
    p = args.detail or os.path.join("gpurun_out", "bench_detail_n%d.json" % world)
    return p if os.path.isabs(p) else os.path.join(HERE, p)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.cpu_baseline_child:
        gshape, dtype, _, _, _ = config_of(args, args.config)
        print(json.dumps(cpu_baseline(args.config, gshape, dtype, args.cpu_sample_rows)), flush=True)
        return 0
    if env_world is None and (args.gpus or 1) > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%d: refusing to measure a different number of "
                         "GPUs than asked\n" % (args.gpus, world))
        return 2
    rank = int(os.environ.get("RANK", "0"))
    # rehearsal knobs (not the measured configuration): several ranks on one
    # device over gloo, exchanges staged through the host by a test executor
    # of tests/cpu_backend.py (RCCL refuses two ranks on one GPU)
    backend = os.environ.get("BOLT_AMD_BENCH_BACKEND", "nccl")
    where = os.environ.get("BOLT_AMD_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not rehearsal_knobs() and world > visible_gpus():
        sys.stderr.write("bench.py: WORLD_SIZE=%d but %d GPU(s) visible\n" % (world, visible_gpus()))
        return 2
    # a stalled exchange ends the run with BoltCommError well inside any
    # driver's limit (a legitimate exchange here takes milliseconds)
    os.environ.setdefault("BOLT_AMD_COMM_TIMEOUT", "180")
    profiling = rocprof_wanted(args, world, where)
    if profiling and rank == 0 and not os.environ.get(PROFILED_ENV):
        return rocprof_rank0(sys.argv[1:], world)
    import torch
    import torch.distributed as dist
    if where == "cpu":
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", int(where))
        torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            # gloo for the host-side barrier / timing max / metadata, nccl only
            # as the group's device backend: no device_id, no eager torch RCCL
            # communicator -- the one RCCL communicator per rank is the
            # library's (MI355XContext, bm_comm_init through the group's store)
            _stdout_to_stderr(lambda: dist.init_process_group("cpu:gloo,cuda:nccl"))
        else:
            _stdout_to_stderr(lambda: dist.init_process_group(backend))
    if dev.type == "cpu" or (world > 1 and backend != "nccl"):
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import cpu_backend
        if dev.type == "cpu":
            cpu_backend.install()
        else:
            cpu_backend.install_host_staged_gpu()

    import bolt_amd as bolt
    from bolt_amd import MI355XContext
    from bolt_amd.mi355x import dist as bdist
    from bolt_amd.mi355x._ops import backend_for
    ctx = _stdout_to_stderr(lambda: MI355XContext(device=dev))
    assert ctx.world_size == world
    if world > 1:
        _stdout_to_stderr(dist.barrier)  # (a lazily connecting transport talks here)
    be = backend_for(dev)
    marks, marks_info = [], {}
    prose = {}   # the detail file's descriptions

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def barrier():
        sync()
        if world > 1:
            dist.barrier()  # over gloo (host)
        sync()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64)  # host tensor: over gloo
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def build(cfg):
        gshape, dtype, split, scaling, desc = config_of(args, cfg, world)
        shard = synth_shard(torch, slab_shapes(gshape, world)[rank], dtype, dev, 1234 + rank)
        b = bolt.ConstructMI355X.fromshards(shard, gshape, context=ctx, split=split, dtype=dtype)
        del shard
        return b, gshape, dtype, split, scaling, desc

    def release():
        import gc
        gc.collect()
        _empty_cache(torch, dev)

    def timed_steps(ops, steps, clock=None, call_events=None, op_filter=None):
        """K steps between barriers; the clock / call events (when given) time the
        ops op_filter admits.  Returns the max-over-ranks wall time."""
        barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            for name, call, _ in ops:
                on = op_filter is None or name in op_filter
                if clock is not None and on:
                    clock.op = name
                if call_events is not None and on:
                    e0, e1 = make_event(dev), make_event(dev)
                    e0.record()
                r = call()
                if call_events is not None and on:
                    e1.record()
                    call_events.setdefault(name, []).append((e0, e1))
                if clock is not None:
                    clock.op = None
                del r
        barrier()
        return max_over_ranks(time.perf_counter() - t0)

    def per_op_ms(ops, steps):
        """{op: (ms per call, launches per call)}: one GPU, the library launches'
        own hipEvents; N GPUs, hipEvents around each call (its exchange
        included).  K more steps, outside the timed region."""
        if world == 1:
            clock = KernelClock(be, dev, LAUNCHES, pool=steps * len(ops) * 4)
            try:
                timed_steps(ops, steps, clock=clock)
            finally:
                clock.close()
            return {name: (clock.ms(name, steps), clock.launches(name, steps)) for name, _, _ in ops}
        calls = {}
        timed_steps(ops, steps, call_events=calls)
        return {name: (float(np.mean([a.elapsed_time(z) for a, z in calls[name]])) if calls.get(name) else None,
                       None) for name, _, _ in ops}

    def marked_pass(cfg, b, ops, steps):
        """N ranks under rocprof: K more steps with torch's spin kernel as a
        marker before and after every op call (every rank runs it: the ops
        hold collectives); rank 0's trace attributes kernels to calls."""
        if not profiling:
            return
        specs = {n: sp for n, _, sp in checks_of(cfg, b)}
        for name, _, nb in ops:
            sp = specs.get(name)
            payload = 0
            if sp and sp[0] == "perm" and sp[1][0] != 0:
                payload = int(nb / 2 * (world - 1) / world)   # the permuted slab's bytes sent to peers
            marks_info["%s.%s" % (cfg, name)] = [payload, int(2 * nb) if payload else 0]
        progress("%s: marked pass (%d steps) for the kernel trace" % (cfg, steps))
        barrier()
        for _ in range(steps):
            for name, call, _ in ops:
                torch.cuda._sleep(1)
                r = call()
                del r
                torch.cuda._sleep(1)
        barrier()
        marks.append([cfg, [n for n, _, _ in ops], steps])

    def call_ms(call, reps):
        """Mean ms of ``reps`` calls between events on the current stream after
        one warm-up call (a swap's events bracket its whole exchange: the last
        unpack waits for the last all-to-all), max over ranks."""
        r = call()
        del r
        barrier()
        evs = []
        for _ in range(reps):
            e0, e1 = make_event(dev), make_event(dev)
            e0.record()
            r = call()
            e1.record()
            del r
            evs.append((e0, e1))
        barrier()
        return max_over_ranks(float(np.mean([a.elapsed_time(z) for a, z in evs])))

    def stage_sweep(swap_call, reps=3):
        """The swap's exchange time at pipeline depths K = 1..16 (dist.STAGES):
        tuning data for dist.STAGE_BYTES_BY_WORLD from the run itself."""
        out = {}
        try:
            for k in (1, 2, 4, 8, 16):
                bdist.STAGES = k
                out[str(k)] = round(call_ms(swap_call, reps), 3)
        finally:
            bdist.STAGES = None
        progress("swap exchange ms by pipeline depth: %s" % out)
        return out

    def a2a_sweep(reps=5):
        """The xGMI all-to-all itself: bm_alltoallv (RCCL send / recv group) of
        B bytes to every peer, no pack / unpack; per size [ms, GB/s each rank
        sends, fraction of (G-1) x 153 GB/s]."""
        out = {}
        G = world
        for mib in (4, 16, 64):
            per = mib << 20
            send = torch.empty(per * G, dtype=torch.uint8, device=dev)
            sizes = [per] * G

            def xchg():
                recv, work = bdist.all_to_all_bytes(ctx, send, sizes, sizes, 8, async_op=True)
                if work is not None:
                    work.wait()
                return recv
            ms = call_ms(xchg, reps)
            gbs = per * (G - 1) / (ms / 1e3) / 1e9
            out["%dM" % mib] = [round(ms, 4), round(gbs, 1), round(gbs / ((G - 1) * XGMI_LINK_GBPS), 4)]
            del send
        progress("all-to-all per peer size -> [ms, GB/s, frac]: %s" % out)
        return out

    def run_all_checks(cfg, b, gshape, dtype, rec_ops):
        """Checks of every op (run_checks) into rec_ops[name]["ck"]; returns all-ok (None: skipped)."""
        if args.no_checks:
            return None
        progress("%s: checks" % cfg)
        det, ok = run_checks(torch, cfg, b, ctx, dev, gshape, dtype, world)
        for name, v in det.items():
            rec_ops.setdefault(name, {})["ck"] = v
        return ok

    def measure_main(cfg, steps, warmup):
        """The headline record: wall time of K steps, the permute kernel's own
        hipEvents (one GPU) or the exchange's (N GPUs), per-op times, checks."""
        b, gshape, dtype, split, scaling, desc = build(cfg)
        ops = steps_of(cfg, b, world)
        if args.pmc_child:  # profiled child of pmc_traffic(): the step, a marker before every op
            for _ in range(warmup + steps):
                for _, call, _ in ops:
                    torch.cuda._sleep(1)
                    r = call()
                    del r
            sync()
            return None
        progress("%s: %d warm-up + %d timed steps on %d rank(s)" % (cfg, warmup, steps, world))
        for _ in range(warmup):
            for _, call, _ in ops:
                r = call()
                del r
        # hipEvents bracketing the permute kernel's own launch, on the stream it
        # runs on (one permute launch per swap on one GPU; the pipelined
        # multi-GPU swap launches more and draws extra pairs)
        # permute; copy_strided when the result is stored at a padded row pitch
        clock = KernelClock(be, dev, ("permute", "copy_strided"), pool=steps)
        swap_ev = {} if world > 1 else None
        if world > 1:
            bdist.PROFILE = {}  # hipEvent pairs around pack / all_to_all / unpack
        try:
            elapsed = timed_steps(ops, steps, clock=clock, call_events=swap_ev, op_filter=(ops[0][0],))
        finally:
            clock.close()
        phases, rccl_ms = {}, None
        if bdist.PROFILE is not None:
            for k, evs in bdist.PROFILE.items():
                phases[k] = float(np.mean([a.elapsed_time(z) for a, z in evs]))
            if bdist.PROFILE.get("rccl"):
                # the RCCL groups alone (all pipeline stages of a swap), per swap
                rccl_ms = float(np.sum([a.elapsed_time(z) for a, z in bdist.PROFILE["rccl"]])) / steps
            bdist.PROFILE = None
        # On one GPU the swap call is the one permute launch, so only the kernel's
        # own event pair is recorded (each extra stream event adds a few us between
        # the kernels); across GPUs the call's pair brackets the whole exchange.
        kern_ms = clock.ms(ops[0][0], steps)
        swap_ms = (float(np.mean([a.elapsed_time(z) for a, z in swap_ev[ops[0][0]]])) if world > 1
                   else kern_ms)
        if kern_ms is None:  # (no permute launch in the op: the step's wall time bounds it)
            kern_ms = swap_ms if swap_ms is not None else elapsed / steps * 1e3
            swap_ms = kern_ms
        per = {name: nb * world for name, _, nb in ops}
        value = sum(per.values()) * steps / elapsed / 1e9
        swap_bytes_rank = ops[0][2]
        achieved = swap_bytes_rank / (kern_ms / 1e3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": DTYPE_NAMES[np.dtype(dtype).name],
            "data": "synthetic, generated in HBM",
            "config": {"name": cfg, "workload": desc, "global_shape": list(gshape), "split": split,
                       "parallelism": "dp%d" % world,
                       "collectives": ("none" if world == 1 else "rccl" if ctx.comm
                                       else "%s host-staged (rehearsal)" % backend),
                       "bytes_per_step": {k: int(v) for k, v in per.items()}},
            "legend": LEGEND,
            "roofline": {
                "bound": "hbm",
                "kernel": ("bm_permute / bm_copy_strided (%s)" % ops[0][0]) if world == 1 else "swap exchange per rank",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": None,
                "avg_ms": round(kern_ms, 4),
                "bytes_per_launch": int(swap_bytes_rank),
            },
        }
        if os.environ.get("BOLT_AMD_BENCH_LAUNCHER"):
            line["launcher"] = os.environ["BOLT_AMD_BENCH_LAUNCHER"]
        if world > 1:
            G = world
            n_rank = ops[0][2] / 2                        # bytes held per rank
            payload = n_rank * (G - 1) / G                # bytes each rank sends to its peers
            ex = phases.get("exchange")
            if ex:  # the swap across GPUs: pipelined pack -> RCCL all-to-all -> unpack
                line["roofline"].update({"achieved": round(2 * n_rank / (ex / 1e3) / 1e9, 1),
                                         "avg_ms": round(ex, 4), "bytes_per_launch": int(2 * n_rank)})
                line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBPS, 4)
            peak = (G - 1) * XGMI_LINK_GBPS
            x = {"payload_bytes_per_rank": int(payload), "avg_ms": round(ex, 4) if ex else None,
                 "achieved": round(payload / (ex / 1e3) / 1e9, 1) if ex else None, "peak": peak,
                 "unit": "GB/s per rank (egress)",
                 "frac": round(payload / (ex / 1e3) / 1e9 / peak, 4) if ex else None,
                 "phases_ms": {k: round(v, 4) for k, v in phases.items()}}
            if rccl_ms:
                # isolated: hipEvents around each bm_alltoallv on the RCCL stream
                # (stages overlap pack / unpack, so this is the links' own time)
                x["rccl_ms_per_swap"] = round(rccl_ms, 4)
                x["rccl_achieved"] = round(payload / (rccl_ms / 1e3) / 1e9, 1)
                x["rccl_frac"] = round(payload / (rccl_ms / 1e3) / 1e9 / peak, 4)
            line["xgmi"] = x
            if ctx.comm:
                import ctypes
                from bolt_amd.mi355x import _lib
                r_, w_ = ctypes.c_int(), ctypes.c_int()
                lib_path = ctypes.create_string_buffer(512)
                _lib.check(_lib.load().bm_comm_info(ctx.comm, ctypes.byref(r_), ctypes.byref(w_), lib_path, 512),
                           "bm_comm_info")
                line["rccl_ranks"] = int(w_.value)
                prose.setdefault("rccl_lib", lib_path.value.decode("utf-8", "replace"))
            else:
                line["rccl_ranks"] = None
        line["roofline"]["frac_of_measured_copy"] = round(line["roofline"]["achieved"] / HBM_COPY_GBPS, 4)
        # this box's own copy ceiling for the same bytes (boxes differ by up to
        # ~25% on the same kernel, profiles/r06zk_pack_expand.log)
        copy_live = live_copy_gbps(be, dev, ops[0][2] // 2) if world == 1 else None
        if copy_live:
            line["roofline"]["copy_live"] = round(copy_live, 1)
            line["roofline"]["frac_of_live_copy"] = round(line["roofline"]["achieved"] / copy_live, 4)
        stat_ops = [name for name, _, _ in ops[1:] if name in ("mean", "std", "var")]
        if stat_ops and world == 1:
            # the reduction kernels' own hipEvents, in K more steps (kept out of the
            # timed region above: every extra event adds a few us to the step)
            clock = KernelClock(be, dev, ("reduce", "reduce_rows", "reduce_state", "reduce_combine"),
                                pool=steps * len(stat_ops))
            try:
                timed_steps(ops, steps, clock=clock, op_filter=stat_ops)
            finally:
                clock.close()
            sr = {}
            nbs = dict((n, v) for n, _, v in ops)
            for name in stat_ops:
                ms = clock.ms(name, steps)
                sr[name] = op_rec(nbs[name], ms, clock.launches(name, steps))
            line["stats_roofline"] = sr
        if not args.pmc_child:
            # every op's own time, in K more steps (outside the timed region)
            times = per_op_ms(ops, steps)
            line["ops"] = {name: op_rec(nb, *times[name]) for name, _, nb in ops}
        marked_pass(cfg, b, ops, steps)
        if world > 1 and not args.no_sweeps:
            line["xgmi"]["stages_ms"] = stage_sweep(ops[0][1])
            line["a2a"] = a2a_sweep()
        ok = run_all_checks(cfg, b, gshape, dtype, line.setdefault("ops", {}))
        line["checks_ok"] = ok
        if world > 1:
            line["exchange_check"] = line["ops"].get(ops[0][0], {}).get("ck")
        del b, ops
        release()
        return line

    def measure_sub(cfg, steps, warmup):
        """A sub-record: K steps of a config; per op the library launches' own
        hipEvents (one GPU) or each call's (N GPUs: the exchange included)."""
        b, gshape, dtype, split, scaling, desc = build(cfg)
        ops = steps_of(cfg, b, world)
        progress("%s: %d warm-up + %d timed steps on %d rank(s)" % (cfg, warmup, steps, world))
        for _ in range(warmup):
            for _, call, _ in ops:
                r = call()
                del r
        clock, calls = None, None
        if world == 1:
            clock = KernelClock(be, dev, LAUNCHES, pool=steps * len(ops) * 4)
        else:
            calls = {}
        try:
            elapsed = timed_steps(ops, steps, clock=clock, call_events=calls)
        finally:
            if clock is not None:
                clock.close()
        per = {name: nb * world for name, _, nb in ops}
        rec = {"value": round(sum(per.values()) * steps / elapsed / 1e9, 2),
               "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps, "scaling": scaling,
               "global_shape": list(gshape), "dtype": DTYPE_NAMES[np.dtype(dtype).name], "ops": {}}
        prose.setdefault("workloads", {})[cfg] = desc
        for name, _, nb in ops:
            if clock is not None:
                ms, nl = clock.ms(name, steps), clock.launches(name, steps)
            else:
                evs = calls.get(name, [])
                ms, nl = (float(np.mean([a.elapsed_time(z) for a, z in evs])) if evs else None), None
            rec["ops"][name] = op_rec(nb, ms, nl)
        timed = [(o["ms"], n) for n, o in rec["ops"].items() if o["ms"]]
        rec["dominant"] = max(timed)[1] if timed else None
        marked_pass(cfg, b, ops, steps)
        rec["ok"] = run_all_checks(cfg, b, gshape, dtype, rec["ops"])
        del b, ops
        release()
        return rec

    def add_traffic(cfg, names, recs):
        """PMC traffic per op call (rank 0, one GPU): "tr" = traffic / algorithmic bytes."""
        progress("%s: rocprofv3 --pmc passes" % cfg)
        traffic, note = pmc_traffic(cfg, args, len(names))
        prose.setdefault("traffic", note)
        for k, name in enumerate(names):
            for rec in recs.get(name, ()):
                nb = rec.get("B", rec.get("bytes_per_launch"))
                if traffic and nb:
                    rec["tr"] = round(traffic[k] / nb, 4)
        return traffic

    line = measure_main(args.config, args.steps, args.warmup)
    if line is None:
        return 0
    one = rank == 0 and world == 1 and dev.type == "cuda"
    if one and not args.no_pmc:
        names = list(line["config"]["bytes_per_step"])
        recs = {n: [line["ops"][n]] for n in names if n in line["ops"]}
        recs.setdefault(names[0], []).append(line["roofline"])
        for n, v in line.get("stats_roofline", {}).items():
            recs.setdefault(n, []).append(v)
        traffic = add_traffic(args.config, names, recs)
        if traffic:
            line["roofline"]["traffic"] = int(traffic[0])
            line["roofline"]["traffic_ratio"] = line["roofline"].pop("tr", None)
    target = None
    if world == 1 and args.config == "C2" and not args.no_target64:
        # BASELINE.json's target sentence: swap and statistics of a 64 GiB
        # float32 4-D array on one GPU at >= 60% of the HBM roofline
        t = measure_main("target64", args.target_steps, 1)
        target = {"value": t["value"], "frac_of_hbm_peak": round(t["value"] / HBM_PEAK_GBPS, 4),
                  "ms_per_step": t["ms_per_step"], "steps": t["steps"], "global_shape": t["config"]["global_shape"],
                  "target": "value >= 0.60 x 8 TB/s on one GPU",
                  "roofline": {k: t["roofline"][k] for k in ("achieved", "frac", "avg_ms", "bytes_per_launch")},
                  "ops": t["ops"], "ok": t["checks_ok"]}
        prose.setdefault("workloads", {})["target64"] = t["config"]["workload"]
        if one and not args.no_pmc:
            names = list(t["config"]["bytes_per_step"])
            recs = {n: [target["ops"][n]] for n in names if n in target["ops"]}
            recs[names[0]].append(target["roofline"])
            add_traffic("target64", names, recs)
            target["roofline"]["traffic_ratio"] = target["roofline"].pop("tr", None)
    configs = None
    if args.config == "C2" and not args.no_configs:
        configs = {}
        for cfg in SUB_CONFIGS:
            rec = measure_sub(cfg, args.config_steps, 1)
            if one and not args.no_pmc:
                add_traffic(cfg, list(rec["ops"]), {n: [o] for n, o in rec["ops"].items()})
            configs[cfg] = rec
    cpu = None
    if one and not args.no_cpu_baseline:
        progress("%s: CPU baseline (child process)" % args.config)
        cpu = cpu_baseline_in_child(args, args.config)
    # the stdout record: the driver keeps its tail, so the numbers come after
    # the contract keys in this order and the prose goes to the detail file
    out = dict(line)
    stats_roofline = out.pop("stats_roofline", None)
    ops = out.pop("ops", None)
    checks_ok = out.pop("checks_ok", None)
    if cpu is not None:
        out["cpu_baseline"] = compact_cpu(cpu)
    out["ops"] = ops
    if configs is not None:
        out["configs"] = configs
    if target is not None:
        out["target64"] = target
    if stats_roofline is not None:
        out["stats_roofline"] = stats_roofline
    out["checks_ok"] = checks_ok
    if profiling:
        out["rocprof_marks"] = marks
        out["rocprof_info"] = marks_info
    if rank == 0:
        path = detail_path(args, world)
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            d = dict(out)
            d.pop("rocprof_marks", None)
            d.pop("rocprof_info", None)
            prose.setdefault("workloads", {})[args.config] = line["config"]["workload"]
            d["prose"] = prose
            if cpu is not None:
                d["cpu_baseline"] = cpu
            with open(path, "w") as f:
                json.dump(d, f, indent=1)
            out["detail"] = os.path.relpath(path, HERE)
        except OSError as e:
            out["detail"] = "not written: %s" % e
        print(json.dumps(out, separators=(",", ":")), flush=True)
    if world > 1:
        barrier()
        ctx.close()  # the library's RCCL communicator, before the process group
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
