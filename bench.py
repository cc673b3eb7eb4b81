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
`traffic` comes from rocprofv3 --pmc child runs (FETCH_SIZE, WRITE_SIZE).

Sub-records of the default run (same JSON line; `value` stays C2's):
  target64  BASELINE.json's target, swap + mean/std of a 64 GiB float32 4-D
            array (1 GPU only);
  configs   C1, C3, C4 and C5 (BASELINE configs[0], [2..4]), a few steps
            each: value, per-op hipEvents time, fraction of HBM peak and PMC
            traffic.
`checks` compares the results of every permute (bit for bit) and of every
statistic over the sharded axis (float64 truth, stated tolerance) with the
global array rebuilt from each rank's seed; `cpu_baseline` times the oracle's
restatement of the reference Spark path and the local mode's numpy calls in a
child process that never touches the GPU.

N GPUs: `python bench.py --gpus N` starts the N rank processes itself (one
per GPU, before anything touches the GPU; rank 0's JSON line is relayed), or
runs as one rank of `torch.distributed.run --nproc-per-node N ... --gpus N`.
A --gpus that differs from WORLD_SIZE, or more GPUs than are visible, exits 2.
Weak scaling: the leading axis grows with N, the swap becomes pack ->
all-to-all -> unpack over RCCL, sharded-axis statistics all_gather their
partial states.
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
    # name: (per-GPU shape, dtype, split, description)
    "C1": ((100, 64, 64), np.float64, 1,
           "C1: float64 (100,64,64), key 0; swap((0,),(0,)) then sum/mean/var/std at axis=None and "
           "axis=(0,) of the swapped array (the reference's CPU-runnable case)"),
    "C2": ((2000, 512, 512), np.float32, 1,
           "C2: float32 (2000,512,512) per GPU, key=time; swap((0,),(0,1)) + mean/std over time"),
    "C3": ((4096, 256, 256, 32), np.float32, 2,
           "C3: float32 (4096,256,256,32) per GPU, keys (0,1); swap((0,),(0,)) + .T"),
    "C4": ((10000, 1024, 1024), np.uint16, 1,
           "C4: uint16 (10000,1024,1024) per GPU, key 0; swap((0,),(0,)) + chunk('150') -> unchunk "
           "(plan (73, 1024): the packed layout is the dense one, no bytes move) + float64 var over axis 0"),
    "C5": ((64, 64, 64, 64, 64), np.float64, 3,
           "C5: float64 64^5 per GPU, keys (0,1,2); .T + transpose(2,0,4,1,3) + "
           "chunk((16,16), padding=2) -> unchunk / keys_to_values((2,)) / values_to_keys((0,))"),
    "target64": ((8192, 256, 256, 32), np.float32, 2,
                 "64 GiB float32 4-D per GPU, keys (0,1); swap((0,),(0,)) + mean/std over axis 0"),
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
    ap.add_argument("--no-target64", action="store_true",
                    help="skip the 64 GiB north_star sub-record of the default (C2, 1 GPU) run")
    ap.add_argument("--target-steps", type=int, default=5)
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C1/C3/C4/C5 sub-records of the default (C2) run")
    ap.add_argument("--config-steps", type=int, default=3)
    ap.add_argument("--no-checks", action="store_true", help="skip the post-timing result checks")
    # internal: rocprofv3 child, CPU-baseline child, rehearsal shapes (JSON {config: per-rank shape})
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--shard-shapes", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def config_of(args, cfg):
    """(per-rank shape, dtype, split, description) of a config; --shard-shapes
    (rehearsals on small data) overrides the shape."""
    shape, dtype, split, desc = CONFIGS[cfg]
    if args.shard_shapes:
        over = json.loads(args.shard_shapes)
        if cfg in over:
            shape = tuple(int(s) for s in over[cfg])
            desc = "REHEARSAL SHAPE %s -- %s" % (str(shape), desc)
    return shape, dtype, split, desc


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
    """The results the bench checks after timing, as (name, call, spec):
    spec ("perm", perm) -- the call returns x.transpose(perm), compared bit for
    bit; spec ("stat", name, axis, pre) -- a statistic over ``axis`` of
    x.transpose(pre) (pre None: of x) that reduces the sharded leading axis
    (reduce_state -> all_gather -> ordered Chan combine across GPUs)."""
    from bolt_amd.mi355x.plan import swap_perm
    nd = len(b.shape)
    rev = list(range(nd))[::-1]
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
        return [("swap", lambda: b.swap((0,), (0, 1)), ("perm", swap_perm(nd, b.split, (0,), (0, 1))[0]))]
    if cfg == "C3":
        return [("swap", lambda: b.swap((0,), (0,)), ("perm", swap_perm(nd, b.split, (0,), (0,))[0])),
                ("T", lambda: b.T, ("perm", rev))]
    if cfg == "C4":
        return [("swap", lambda: b.swap((0,), (0,)), ("perm", swap_perm(nd, b.split, (0,), (0,))[0])),
                ("var", lambda: b.var(axis=0), ("stat", "var", (0,), None))]
    if cfg == "C5":
        return [("T", lambda: b.T, ("perm", rev)),
                ("transpose", lambda: b.transpose(2, 0, 4, 1, 3), ("perm", [2, 0, 4, 1, 3]))]
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


def perm_check(torch, res, perm, shape, dtype, ctx, dev):
    """True if this rank's slab of ``res`` equals x.transpose(perm), x the
    global array whose rank-r rows are synth_shard(seed 1234 + r)."""
    world, es = ctx.world_size, np.dtype(dtype).itemsize
    idt = _int_type(torch, es)
    gshape = (shape[0] * world,) + tuple(shape[1:])
    oshape = [gshape[p] for p in perm]
    got = res._data.view(idt)
    a, j = perm[0], perm.index(0)
    if world == 1 or a == 0:
        # this rank's own rows, permuted: compared in chunks of output rows
        x = synth_shard(torch, shape, dtype, dev, 1234 + ctx.rank).view(idt).permute(*perm)
        row = int(np.prod(x.shape[1:]))
        step = max(1, CHECK_CHUNK // max(1, row * es))
        ok = True
        for lo in range(0, x.shape[0], step):
            hi = min(x.shape[0], lo + step)
            ok = ok and bool(torch.equal(got[lo * row:hi * row], x[lo:hi].contiguous().reshape(-1)))
        del x
        return ok
    lo, hi = ctx.bounds(oshape[0])[ctx.rank]
    want = torch.empty([hi - lo] + oshape[1:], dtype=idt, device=dev)
    for r, (rlo, rhi) in enumerate(ctx.bounds(gshape[0])):
        x = synth_shard(torch, shape, dtype, dev, 1234 + r).view(idt)
        want.narrow(j, rlo, rhi - rlo).copy_(x.narrow(a, lo, hi - lo).permute(*perm))
        del x
    ok = bool(torch.equal(got, want.reshape(-1)))
    del want
    return ok


def _as_f64(torch, t, dtype):
    if np.dtype(dtype) == np.uint16:
        return (t.to(torch.int32) & 0xFFFF).to(torch.float64)
    return t.to(torch.float64)


def stat_truth(torch, name, axis, pre, shape, dtype, world, dev):
    """(float64 truth, scale) of statistic ``name`` over ``axis`` of
    x.transpose(pre) on the device, x the global array rebuilt from every
    rank's seed.  Small arrays are rebuilt whole; otherwise (pre None, axis
    (0,)) each rank's rows are regenerated and reduced in chunks, merged with
    Chan's update.  ``scale`` is the tolerance's absolute term: max|x| (mean),
    sum|x| (sum), max|truth| (var / std)."""
    es = np.dtype(dtype).itemsize
    total = int(np.prod(shape)) * world * 8
    if total <= (1 << 30):
        x = torch.cat([_as_f64(torch, synth_shard(torch, shape, dtype, dev, 1234 + r), dtype)
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
    row = int(np.prod(shape[1:]))
    step = max(1, CHECK_CHUNK // (row * 8))
    n, mean, m2, xmax = 0, None, None, 0.0
    for r in range(world):
        x = synth_shard(torch, shape, dtype, dev, 1234 + r)
        for lo in range(0, shape[0], step):
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
    del es
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


def run_checks(torch, cfg, b, ctx, dev, shape, dtype, world):
    """Every check of checks_of(cfg) on this rank -> {name: result}, all ranks'
    verdicts merged (a mismatch on any rank is a mismatch)."""
    res = {}
    for name, call, spec in checks_of(cfg, b):
        r = call()
        if spec[0] == "perm":
            ok = perm_check(torch, r, spec[1], shape, dtype, ctx, dev)
            detail = "bit-exact" if ok else "MISMATCH"
        else:
            _, stat, axis, pre = spec
            truth, scale = stat_truth(torch, stat, axis, pre, shape, dtype, world, dev)
            ok, worst = stat_within(r, truth.cpu().numpy(), scale.cpu().numpy() if hasattr(scale, "cpu") else scale,
                                    stat)
            detail = ("within %s (max error %.3g of the bar)" % (
                "rtol 1e-12" if np.asarray(r).dtype == np.float64 else "rtol 1e-6", worst) if ok else
                "OUT OF TOLERANCE (max error %.3g of the bar)" % worst)
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


def exchange_check(torch, cfg, b, ctx, dev, shape=None, dtype=None, split=None):
    """Bit-exact check of the first op of the step (the swap / .T that crosses
    GPUs): True if every byte of this rank's slab agrees with the global array
    rebuilt from every rank's seed."""
    if shape is None:
        shape, dtype, split, _ = CONFIGS[cfg]
    name, call, spec = checks_of(cfg, b)[0]
    r = call()
    ok = perm_check(torch, r, spec[1], shape, dtype, ctx, dev)
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
        if args.shard_shapes:
            cmd += ["--shard-shapes", args.shard_shapes]
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
            "sample": "oracle/bolt_oracle.py record-level Spark path (8 partitions) on the whole C1 input, "
                      "swap + sum/mean/var/std at axis=None and axis=(0,), %d steps per timed run, best of %d "
                      "after 1 warm-up" % (out["spark"][1], REPS),
            "host_cpus": os.cpu_count(),
            "local_numpy": {"value": round(out["local"][0], 3), "unit": "GB/s", "cores": 1, "reps": REPS,
                            "sample": "the reference local mode's numpy calls on the same input, %d steps per "
                                      "timed run, best of %d after 1 warm-up" % (out["local"][1], REPS)}}


def cpu_baseline(cfg, shape, dtype, rows):
    """Oracle (record-level restatement of the reference Spark path), 1 core,
    bounded sample, best of 3 after 1 warm-up; C2 adds the local
    mode's numpy calls, the Spark local[8] analogue and an OpenMP line."""
    from oracle import bolt_oracle as O
    if cfg == "C1":
        return c1_cpu_baseline(shape, dtype)
    if cfg != "C2":
        return local_numpy_baseline(cfg, shape, dtype)
    rows = rows or C2_SAMPLE_ROWS
    rng = np.random.default_rng(0)
    sample_shape = (rows,) + tuple(shape[1:])
    x = (1000 + 50 * rng.standard_normal(sample_shape)).astype(dtype)
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
        xs = np.ascontiguousarray(x.transpose(1, 2, 0))
        u1 = time.perf_counter()
        xs.mean(axis=2)
        u2 = time.perf_counter()
        xs.std(axis=2)
        u3 = time.perf_counter()
        return u1 - u0, u2 - u1, u3 - u2
    N = int(np.prod(sample_shape)) * np.dtype(dtype).itemsize
    out_b = sample_shape[1] * sample_shape[2] * 4
    total = 2 * N + 2 * (N + out_b)
    ts, tp = best_of(spark)
    ls, lp = best_of(local)
    out = {"value": total / ts / 1e9, "unit": "GB/s", "cores": 1, "kind": "port", "reps": REPS,
           "sample": "oracle/bolt_oracle.py record-level Spark path (8 partitions) on float32 %s, best of %d "
                     "after 1 warm-up: swap((0,),(0,1)) %.2fs + mean(axis=2) %.2fs + std(axis=2) %.2fs"
                     % ((str(sample_shape), REPS) + tp),
           "host_cpus": os.cpu_count(),
           "local_numpy": {"value": round(total / ls / 1e9, 3), "unit": "GB/s", "cores": 1, "reps": REPS,
                           "sample": "the reference local mode's numpy calls on the same input, best of %d "
                                     "after 1 warm-up: transpose %.2fs + mean %.2fs + std %.2fs" % ((REPS,) + lp)}}
    del rs
    out["spark_local8"] = spark_local8_baseline(x, dtype)
    out["openmp"] = openmp_baseline(np.ascontiguousarray(
        (1000 + 50 * rng.standard_normal((shape[0],) + tuple(shape[1:]), dtype=np.float32))))
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
    if args.shard_shapes:
        cmd += ["--shard-shapes", args.shard_shapes]
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
            "reduce_state", "reduce_combine")


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


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.cpu_baseline_child:
        shape, dtype, split, _ = config_of(args, args.config)
        print(json.dumps(cpu_baseline(args.config, shape, dtype, args.cpu_sample_rows)), flush=True)
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
        shape, dtype, split, desc = config_of(args, cfg)
        gshape = (shape[0] * world,) + tuple(shape[1:])
        shard = synth_shard(torch, shape, dtype, dev, 1234 + rank)
        b = bolt.ConstructMI355X.fromshards(shard, gshape, context=ctx, split=split, dtype=dtype)
        del shard
        return b, shape, dtype, split, desc, gshape

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

    def checks(cfg, b, shape, dtype):
        if args.no_checks:
            return None
        progress("%s: checks" % cfg)
        det, ok = run_checks(torch, cfg, b, ctx, dev, shape, dtype, world)
        det["all"] = ("every result matches (permutes bit-exact, sharded-axis statistics within tolerance) "
                      "against the global array rebuilt from each rank's seed" if ok else "FAILED")
        return det

    def measure_main(cfg, steps, warmup):
        """The headline line: wall time of K steps, the permute kernel's own
        hipEvents (one GPU) or the exchange's (N GPUs)."""
        b, shape, dtype, split, desc, gshape = build(cfg)
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
        clock = KernelClock(be, dev, ("permute",), pool=steps)
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPE_NAMES[np.dtype(dtype).name],
            "data": "synthetic (generated in HBM: 1000+50*N(0,1) float32 / N(0,1) float64 / uniform uint16)",
            "config": {"workload": desc, "global_shape": list(gshape), "split": split,
                       "parallelism": "dp%d (records sharded on the leading key axis)" % world,
                       "collectives": ("none (single GPU)" if world == 1 else
                                       "RCCL via libbolt_mi355x (bm_alltoallv / bm_allgatherv)" if ctx.comm
                                       else "%s, host-staged (one-device rehearsal, not a measurement)" % backend),
                       "bytes_per_step": {k: int(v) for k, v in per.items()}},
            "roofline": {
                "bound": "hbm",
                "kernel": "bm_permute for the %s" % ops[0][0] if world == 1 else
                          "swap = pack + all_to_all + unpack (per rank)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": None,
                "avg_ms": round(kern_ms, 4),
                "swap_call_ms": round(swap_ms, 4),
                "bytes_per_launch": int(swap_bytes_rank),
            },
        }
        if os.environ.get("BOLT_AMD_BENCH_LAUNCHER"):
            line["launcher"] = os.environ["BOLT_AMD_BENCH_LAUNCHER"] + " (rank processes started by bench.py)"
        if world > 1:
            G = world
            xport = "RCCL" if ctx.comm else "%s (host-staged rehearsal)" % backend
            n_rank = ops[0][2] / 2                        # bytes held per rank
            payload = n_rank * (G - 1) / G                # bytes each rank sends to its peers
            ex = phases.get("exchange")
            if ex:  # the swap across GPUs: pipelined pack -> RCCL all-to-all -> unpack
                line["roofline"].update({"kernel": "swap exchange per rank (pack + %s all_to_all + unpack, "
                                                   "pipelined)" % xport,
                                         "achieved": round(2 * n_rank / (ex / 1e3) / 1e9, 1),
                                         "avg_ms": round(ex, 4), "bytes_per_launch": int(2 * n_rank)})
                line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBPS, 4)
            peak = (G - 1) * XGMI_LINK_GBPS
            line["xgmi"] = {"op": ("RCCL send/recv group (bm_alltoallv)" if ctx.comm else
                                   "%s all_to_all" % xport) + " inside the pipelined swap exchange "
                                  "(achieved = peer payload / whole exchange time: a lower bound)",
                            "payload_bytes_per_rank": int(payload),
                            "avg_ms": round(ex, 4) if ex else None,
                            "achieved": round(payload / (ex / 1e3) / 1e9, 1) if ex else None,
                            "peak": peak, "unit": "GB/s per rank (egress)",
                            "frac": round(payload / (ex / 1e3) / 1e9 / peak, 4) if ex else None,
                            "phases_ms": {k: round(v, 4) for k, v in phases.items()}}
            if rccl_ms:
                # isolated: hipEvents around each bm_alltoallv on the RCCL stream
                # (stages overlap pack / unpack, so this is the links' own time)
                line["xgmi"]["rccl_ms_per_swap"] = round(rccl_ms, 4)
                line["xgmi"]["rccl_achieved"] = round(payload / (rccl_ms / 1e3) / 1e9, 1)
                line["xgmi"]["rccl_frac"] = round(payload / (rccl_ms / 1e3) / 1e9 / peak, 4)
            if ctx.comm:
                import ctypes
                from bolt_amd.mi355x import _lib
                r_, w_ = ctypes.c_int(), ctypes.c_int()
                lib_path = ctypes.create_string_buffer(512)
                _lib.check(_lib.load().bm_comm_info(ctx.comm, ctypes.byref(r_), ctypes.byref(w_), lib_path, 512),
                           "bm_comm_info")
                line["rccl_ranks"] = int(w_.value)
                line["rccl_lib"] = lib_path.value.decode("utf-8", "replace")
            else:
                line["rccl_ranks"] = None
        line["roofline"]["frac_of_measured_copy"] = round(line["roofline"]["achieved"] / HBM_COPY_GBPS, 4)
        line["roofline"]["measured_copy_peak"] = HBM_COPY_GBPS
        stat_ops = [name for name, _, _ in ops[1:] if name in ("mean", "std", "var")]
        if stat_ops and world == 1:
            # the reduction kernels' own hipEvents, in K more steps (kept out of the
            # timed region above: every extra event adds a few us to the step)
            clock = KernelClock(be, dev, ("reduce", "reduce_state", "reduce_combine"), pool=steps * len(stat_ops))
            try:
                timed_steps(ops, steps, clock=clock, op_filter=stat_ops)
            finally:
                clock.close()
            sr = {"kernel": "bm_reduce (k_red_rows / k_red_cols) per statistic", "bound": "hbm",
                  "peak": HBM_PEAK_GBPS, "unit": "GB/s"}
            for name in stat_ops:
                ms = clock.ms(name, steps)
                nb = dict((n, v) for n, _, v in ops)[name]
                sr[name] = {"avg_ms": round(ms, 4), "bytes_per_launch": int(nb),
                            "launches_per_call": clock.launches(name, steps),
                            "achieved": round(nb / (ms / 1e3) / 1e9, 1),
                            "frac": round(nb / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None}
            line["stats_roofline"] = sr
        if world == 1 and not args.pmc_child:
            # every op's own library launches, in K more steps (per-op detail of
            # the step; outside the timed region for the same reason)
            clock = KernelClock(be, dev, LAUNCHES, pool=steps * len(ops) * 4)
            try:
                timed_steps(ops, steps, clock=clock)
            finally:
                clock.close()
            line["ops"] = {}
            for name, _, nb in ops:
                ms = clock.ms(name, steps)
                o = {"bytes": int(nb), "ms": round(ms, 4) if ms else None,
                     "launches_per_call": clock.launches(name, steps)}
                if ms and nb:
                    o["achieved"] = round(nb / (ms / 1e3) / 1e9, 1)
                    o["frac"] = round(o["achieved"] / HBM_PEAK_GBPS, 4)
                line["ops"][name] = o
        line["checks"] = checks(cfg, b, shape, dtype)
        if world > 1:
            line["exchange_check"] = (line["checks"] or {}).get(ops[0][0])
        del b, ops
        release()
        return line

    def measure_sub(cfg, steps, warmup):
        """A sub-record: K steps of a config; per op the library launches' own
        hipEvents (one GPU) or each call's (N GPUs: the exchange included)."""
        b, shape, dtype, split, desc, gshape = build(cfg)
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
        rec = {"workload": desc, "global_shape": list(gshape), "split": split,
               "dtype": DTYPE_NAMES[np.dtype(dtype).name],
               "value": round(sum(per.values()) * steps / elapsed / 1e9, 2), "unit": "GB/s",
               "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps, "warmup": warmup,
               "timing": ("hipEvents around each library launch on its stream, summed per op call" if world == 1
                          else "hipEvents around each call on the current stream (the RCCL exchange included)"),
               "ops": {}}
        for name, _, nb in ops:
            if clock is not None:
                ms = clock.ms(name, steps)
                nl = clock.launches(name, steps)
            else:
                evs = calls.get(name, [])
                ms = float(np.mean([a.elapsed_time(z) for a, z in evs])) if evs else None
                nl = None
            o = {"bytes": int(nb), "ms": round(ms, 4) if ms else None, "launches_per_call": nl}
            if ms and nb:
                o["achieved"] = round(nb / (ms / 1e3) / 1e9, 1)
                o["frac"] = round(o["achieved"] / HBM_PEAK_GBPS, 4)
            rec["ops"][name] = o
        timed = [(o["ms"], n) for n, o in rec["ops"].items() if o["ms"]]
        rec["dominant"] = max(timed)[1] if timed else None
        rec["checks"] = checks(cfg, b, shape, dtype)
        del b, ops
        release()
        return rec

    def add_traffic(cfg, names, into):
        """PMC traffic per op call (rank 0, one GPU), into {name: record}."""
        progress("%s: rocprofv3 --pmc passes" % cfg)
        traffic, note = pmc_traffic(cfg, args, len(names))
        for k, name in enumerate(names):
            rec = into.get(name)
            if rec is None:
                continue
            rec["traffic"] = int(traffic[k]) if traffic else None
            nb = rec.get("bytes", rec.get("bytes_per_launch"))
            if traffic and nb:
                rec["traffic_ratio"] = round(traffic[k] / nb, 4)
        return note

    line = measure_main(args.config, args.steps, args.warmup)
    if line is None:
        return 0
    one = rank == 0 and world == 1 and dev.type == "cuda"
    if one and not args.no_pmc:
        names = list(line["config"]["bytes_per_step"])
        recs = {names[0]: line["roofline"]}
        recs.update({n: v for n, v in line.get("stats_roofline", {}).items() if isinstance(v, dict)})
        # every other op of the step: its traffic against its algorithmic bytes
        recs.update({n: o for n, o in line.get("ops", {}).items() if n not in recs})
        line["roofline"]["traffic_note"] = add_traffic(args.config, names, recs)
        for n, o in line.get("ops", {}).items():
            src = recs.get(n)
            if src is not o and src is not None and "traffic" in src:
                o["traffic"] = src["traffic"]
                if "traffic_ratio" in src:
                    o["traffic_ratio"] = src["traffic_ratio"]
    if world == 1 and args.config == "C2" and not args.no_target64:
        # BASELINE.json's target sentence: swap and statistics of a 64 GiB
        # float32 4-D array on one GPU at >= 60% of the HBM roofline
        t = measure_main("target64", args.target_steps, 1)
        sub = {"workload": t["config"]["workload"], "value": t["value"], "unit": "GB/s",
               "ms_per_step": t["ms_per_step"], "steps": t["steps"], "warmup": t["warmup"],
               "global_shape": t["config"]["global_shape"], "bytes_per_step": t["config"]["bytes_per_step"],
               "frac_of_hbm_peak": round(t["value"] / HBM_PEAK_GBPS, 4),
               "target": "swap + mean/std of 64 GiB on 1 GPU at >= 0.60 of HBM (swap <= 28.6 ms)",
               "roofline": t["roofline"], "stats_roofline": t.get("stats_roofline"), "checks": t["checks"]}
        if one and not args.no_pmc:
            names = list(t["config"]["bytes_per_step"])
            recs = {names[0]: sub["roofline"]}
            recs.update({n: v for n, v in (sub["stats_roofline"] or {}).items() if isinstance(v, dict)})
            sub["roofline"]["traffic_note"] = add_traffic("target64", names, recs)
        line["target64"] = sub
    if args.config == "C2" and not args.no_configs:
        line["configs"] = {}
        for cfg in SUB_CONFIGS:
            rec = measure_sub(cfg, args.config_steps, 1)
            if one and not args.no_pmc:
                rec["traffic_note"] = add_traffic(cfg, list(rec["ops"]), rec["ops"])
            line["configs"][cfg] = rec
    if one and not args.no_cpu_baseline:
        progress("%s: CPU baseline (child process)" % args.config)
        line["cpu_baseline"] = cpu_baseline_in_child(args, args.config)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        barrier()
        ctx.close()  # the library's RCCL communicator, before the process group
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
