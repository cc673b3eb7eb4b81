"""Benchmark of the mi355x mode's hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5|target64]

The default run (C2 on one GPU) also times BASELINE.json's target -- swap +
mean/std of a 64 GiB float32 (8192,256,256,32) array -- and reports it as the
`target64` sub-record of the same JSON line (`value` stays C2's).

One "step" = one pass of the hot path over one batch of synthetic input,
resident in HBM before timing starts.  Default workload (BASELINE.json
configs[1], "C2"): float32 (2000, 512, 512) time series per GPU, key = time
(split 1); swap((0,), (0,1)) to key = voxel, then mean and std over time
(axis 2) -- the three calls a bolt user makes, each returning its result to
the host as the reference does.

`value` = algorithmic bytes of all ranks / wall time of K steps (max over
ranks), GB/s:  swap 2*N*s, each stat N*s + outputs.  `roofline` is the
dominant kernel (the swap's permute) measured with hipEvents on the stream it
runs on; `cpu_baseline` times the oracle's record-level restatement of the
reference Spark path (oracle/bolt_oracle.py) on a bounded sample on the host.

For N > 1 (torch.distributed.run, one rank per GPU, RCCL): weak scaling, the
time axis grows with N (2000*N), the swap becomes pack -> all-to-all ->
unpack, the statistics reduce locally and all_gather their outputs.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=None)
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-target64", action="store_true",
                    help="skip the 64 GiB north_star sub-record of the default (C2, 1 GPU) run")
    ap.add_argument("--target-steps", type=int, default=5)
    return ap.parse_args()


ROOFLINE_KERNEL = {"C1": "k_rowcopy", "C2": "k_transpose", "C5": "k_transpose", "C3": "k_rowcopy", "C4": "k_rowcopy",
                   "target64": "k_rowcopy"}


def pmc_traffic(cfg, kernel_substr=None):
    """HBM bytes per launch of the dominant kernel from rocprofv3 PMC counters.

    Two separate child runs of this script (swap only), one counter each
    (FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2: they do not fit one pass),
    with nothing but --pmc on the rocprofv3 line.  gfx950 correction
    (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports half the bytes of wide
    streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B stores.
    Counters are in KiB.  Returns (bytes or None, note).
    """
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    kernel_substr = kernel_substr or ROOFLINE_KERNEL[cfg]
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        out = tempfile.mkdtemp(prefix="bm_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [rp, "--pmc", ctr, "-d", out, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--config", cfg, "--steps", "3",
               "--warmup", "1", "--pmc-child"]
        try:
            subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600, check=True)
        except Exception as e:  # profiler unavailable or refused: report null
            return None, "rocprofv3 --pmc %s failed: %s" % (ctr, type(e).__name__)
        got = []
        for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kernel_substr in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                    got.append(float(row["Counter_Value"]))
        shutil.rmtree(out, ignore_errors=True)
        if not got:
            return None, "no %s samples for %s" % (ctr, kernel_substr)
        vals[ctr] = float(np.median(got))
    fetch = 2.0 * vals["FETCH_SIZE"] * 1024
    write = vals["WRITE_SIZE"] * 1024
    return fetch + write, ("per launch: FETCH_SIZE %.0f KiB (x2 gfx950 correction) + WRITE_SIZE %.0f KiB"
                           % (vals["FETCH_SIZE"], vals["WRITE_SIZE"]))


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
    """The step of a config as (name, call, algorithmic bytes of all ranks) in order.

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


FIRST_OP = {"C1": ((0,), (0,)), "C2": ((0,), (0, 1)), "C3": ((0,), (0,)), "C4": ((0,), (0,)), "C5": "T",
            "target64": ((0,), (0,))}


def exchange_check(torch, cfg, b, ctx, dev, shape=None, dtype=None, split=None):
    """Bit-exact check of the first op of the step (the swap / .T that crosses
    GPUs) after the timed region: this rank's slab of the result against the
    same slab rebuilt from every rank's synthetic shard (regenerated from its
    seed) and permuted by torch on this GPU.  Returns True if every byte agrees."""
    from bolt_amd.mi355x.plan import swap_perm
    if shape is None:
        shape, dtype, split, _ = CONFIGS[cfg]
    world = ctx.world_size
    if FIRST_OP[cfg] == "T":
        perm, res = list(range(len(shape)))[::-1], b.T
    else:
        kax, vax = FIRST_OP[cfg]
        perm, _ = swap_perm(len(shape), split, kax, vax)
        res = b.swap(kax, vax)
    gshape = (shape[0] * world,) + tuple(shape[1:])
    a = perm[0]
    idt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[np.dtype(dtype).itemsize]
    if a == 0:  # no exchange: this rank's own shard
        want = synth_shard(torch, shape, dtype, dev, 1234 + ctx.rank).permute(*perm).contiguous()
    else:
        lo, hi = ctx.bounds(gshape[a])[ctx.rank]
        parts = []
        for r in range(world):
            x = synth_shard(torch, shape, dtype, dev, 1234 + r)
            parts.append(x.narrow(a, lo, hi - lo).contiguous())
            del x
        want = torch.cat(parts, 0).permute(*perm).contiguous()
        del parts
    ok = bool(torch.equal(res._data.view(idt), want.view(idt).reshape(-1)))
    del want, res
    torch.cuda.empty_cache()
    return ok


# leading-axis rows of the per-GPU shard timed by local_numpy_baseline (~0.5-1 GB)
LOCAL_SAMPLE_ROWS = {"C3": 64, "C4": 256, "C5": 8, "target64": 64}


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
    total, parts = 0, []
    t0 = time.perf_counter()
    for name, f in ops:
        u = time.perf_counter()
        r = f()
        parts.append("%s %.2fs" % (name, time.perf_counter() - u))
        total += 2 * N if r.shape == x.shape[::-1] or r.size == x.size else N + r.nbytes
        del r
    el = time.perf_counter() - t0
    return {"value": total / el / 1e9, "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "the reference local mode's numpy calls on %s %s (a leading-axis slab of the "
                      "shard; chunk/unchunk not included): %s" % (np.dtype(dtype).name, str(sample_shape),
                                                                   " + ".join(parts)),
            "host_cpus": os.cpu_count()}


def c1_cpu_baseline(shape, dtype):
    """C1 in full on one host core: the oracle's record-level restatement of
    the reference Spark path (8 partitions) and the reference local mode's
    numpy calls, each repeated to ~10 s."""
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
    for name, f in (("spark", spark), ("local", local)):
        reps, t0 = 0, time.perf_counter()
        while True:
            f()
            reps += 1
            if time.perf_counter() - t0 > (10.0 if name == "spark" else 3.0):
                break
        out[name] = (total * reps / (time.perf_counter() - t0) / 1e9, reps)
    return {"value": out["spark"][0], "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle/bolt_oracle.py record-level Spark path (8 partitions) on the whole C1 input, "
                      "swap + sum/mean/var/std at axis=None and axis=(0,), %d repetitions" % out["spark"][1],
            "host_cpus": os.cpu_count(),
            "local_numpy": {"value": round(out["local"][0], 3), "unit": "GB/s", "cores": 1,
                            "sample": "the reference local mode's numpy calls on the same input, %d repetitions"
                                      % out["local"][1]}}


def cpu_baseline(cfg, shape, dtype, rows):
    """Oracle (record-level restatement of the reference Spark path), 1 core, bounded sample."""
    from oracle import bolt_oracle as O
    if cfg == "C1":
        return c1_cpu_baseline(shape, dtype)
    if cfg != "C2":
        return local_numpy_baseline(cfg, shape, dtype)
    rng = np.random.default_rng(0)
    sample_shape = (rows,) + tuple(shape[1:])
    x = (1000 + 50 * rng.standard_normal(sample_shape)).astype(dtype)
    rs = O.parallelize(x, axis=(0,), npartitions=8)
    t0 = time.perf_counter()
    s = O.swap(rs, (0,), (0, 1))
    t1 = time.perf_counter()
    O.stat(s, 'mean', axis=2)
    t2 = time.perf_counter()
    O.stat(s, 'stdev', axis=2)
    t3 = time.perf_counter()
    N = int(np.prod(sample_shape)) * np.dtype(dtype).itemsize
    out = sample_shape[1] * sample_shape[2] * 4
    total = 2 * N + 2 * (N + out)
    # the reference's local mode (bolt/local/array.py) runs the same three calls
    # as numpy on one host thread: ascontiguousarray(transpose) + mean / std
    u0 = time.perf_counter()
    xs = np.ascontiguousarray(x.transpose(1, 2, 0))
    u1 = time.perf_counter()
    xs.mean(axis=2)
    u2 = time.perf_counter()
    xs.std(axis=2)
    u3 = time.perf_counter()
    out = {"value": total / (t3 - t0) / 1e9, "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": "oracle/bolt_oracle.py record-level Spark path (8 partitions) on float32 %s: "
                     "swap((0,),(0,1)) %.2fs + mean(axis=2) %.2fs + std(axis=2) %.2fs"
                     % (str(sample_shape), t1 - t0, t2 - t1, t3 - t2),
           "host_cpus": os.cpu_count(),
           "local_numpy": {"value": round(total / (u3 - u0) / 1e9, 3), "unit": "GB/s", "cores": 1,
                           "sample": "the reference local mode's numpy calls on the same input: transpose "
                                     "%.2fs + mean %.2fs + std %.2fs" % (u1 - u0, u2 - u1, u3 - u2)}}
    del rs, s, xs
    out["spark_local8"] = spark_local8_baseline(x[:LOCAL8_ROWS], dtype)
    out["openmp"] = openmp_baseline(x)
    return out


def openmp_baseline(x):
    """The local mode's three calls as OpenMP C on the host cores
    (oracle/c/local_step.c, a port: SURVEY 8(d)'s optional multi-core line),
    on the same input; best of two timed runs after one warm-up."""
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
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    xc = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty((P, T), np.float32)
    m = np.empty(P, np.float32)
    sd = np.empty(P, np.float32)
    ptr = lambda a: a.ctypes.data_as(f32p)
    best = None
    for it in range(3):
        t0 = time.perf_counter()
        lib.local_swap(ptr(xc), ptr(y), T, P, threads)
        t1 = time.perf_counter()
        lib.local_mean(ptr(y), ptr(m), T, P, threads)
        t2 = time.perf_counter()
        lib.local_std(ptr(y), ptr(sd), T, P, threads)
        t3 = time.perf_counter()
        if it and (best is None or t3 - t0 < best[3] - best[0]):
            best = (t0, t1, t2, t3)
    t0, t1, t2, t3 = best
    N = xc.nbytes
    total = 2 * N + 2 * (N + P * 4)
    return {"value": round(total / (t3 - t0) / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": "oracle/c/local_step.c (OpenMP, the local mode's ascontiguousarray(transpose) + mean + "
                      "std) on float32 %s: swap %.3fs + mean %.3fs + std %.3fs, best of 2"
                      % (str(x.shape), t1 - t0, t2 - t1, t3 - t2)}


LOCAL8_ROWS = 1000  # time points of the local[8] analogue's sample (~1 GB)


def spark_local8_baseline(x, dtype, workers=8):
    """The Spark local[8] analogue (oracle/spark_local.py): the oracle's record-level
    C2 step with Spark's stage structure on 8 host processes -- 8 map tasks, one
    reduce task per chunk group, and the statistics' single task (their _align
    shuffle has one group) -- shuffles pickled through the parent."""
    from oracle import spark_local as SL
    x = np.ascontiguousarray(x)
    _, _, t, tasks = SL.c2_step(x, workers=workers)
    N = x.nbytes
    out = x.shape[1] * x.shape[2] * 4
    total = 2 * N + 2 * (N + out)
    return {"value": round(total / t["total"] / 1e9, 4), "unit": "GB/s", "cores": workers,
            "kind": "port, local[%d] analogue" % workers, "host_cpus": os.cpu_count(),
            "sample": "oracle/spark_local.py on float32 %s: stage 1 (%d map tasks: chunk + relabel) %.2fs, "
                      "stage 2 (%d reduce tasks: rebuild + values_to_keys + unchunk) %.2fs, mean(axis=2) %.2fs "
                      "+ std(axis=2) %.2fs (one task each: _align's shuffle has a single group, as in the "
                      "reference)" % (str(x.shape), tasks["stage1"], t["stage1"], tasks["stage2"], t["stage2"],
                                      t["mean"], t["std"])}


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


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not the measured configuration): several ranks on one
    # GPU over gloo, exchanges staged through the host by the test executor
    # of tests/cpu_backend.py (RCCL refuses two ranks on one GPU)
    backend = os.environ.get("BOLT_AMD_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("BOLT_AMD_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            # gloo for the host-side barrier / timing max / metadata, nccl only
            # as the group's device backend: no device_id, no eager torch RCCL
            # communicator -- the one RCCL communicator per rank is the
            # library's (MI355XContext, bm_comm_init through the group's store)
            _stdout_to_stderr(lambda: dist.init_process_group("cpu:gloo,cuda:nccl"))
        else:
            _stdout_to_stderr(lambda: dist.init_process_group(backend))
            sys.path.insert(0, os.path.join(HERE, "tests"))
            import cpu_backend
            cpu_backend.install_host_staged_gpu()

    import bolt_amd as bolt
    from bolt_amd import MI355XContext
    ctx = _stdout_to_stderr(lambda: MI355XContext(device=dev))
    assert ctx.world_size == world
    if world > 1:
        _stdout_to_stderr(dist.barrier)  # (a lazily connecting transport talks here)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()  # over gloo (host)
        torch.cuda.synchronize()

    def measure(cfg, steps, warmup):
        """One config's timed run -> its JSON line (without PMC traffic / CPU baseline)."""
        shape, dtype, split, desc = CONFIGS[cfg]
        gshape = (shape[0] * world,) + tuple(shape[1:])
        shard = synth_shard(torch, shape, dtype, dev, 1234 + rank)
        b = bolt.ConstructMI355X.fromshards(shard, gshape, context=ctx, split=split, dtype=dtype)
        del shard

        ops = steps_of(cfg, b, world)
        if args.pmc_child:  # profiled child of pmc_traffic(): the roofline op only, no output
            for _ in range(warmup + steps):
                r = ops[0][1]()
                del r
            torch.cuda.synchronize()
            return None

        for _ in range(warmup):
            for _, call, _ in ops:
                r = call()
                del r
        barrier()

        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        # hipEvents bracketing the permute kernel's own launch, on the stream it runs on
        from bolt_amd.mi355x._ops import backend_for
        be = backend_for(dev)
        kev = []
        # event pairs made before the timed region (one permute launch per swap on
        # one GPU; the pipelined multi-GPU swap launches more and draws extra pairs)
        kpool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in range(steps)]
        permute0 = be.permute
        timing = {"on": False}

        def timed_permute(*a, **k):
            if not timing["on"]:
                return permute0(*a, **k)
            if len(kev) < len(kpool):
                e0, e1 = kpool[len(kev)]
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            permute0(*a, **k)
            e1.record(stream)
            kev.append((e0, e1))
        be.permute = timed_permute
        from bolt_amd.mi355x import dist as bdist
        if world > 1:
            bdist.PROFILE = {}  # hipEvent pairs around pack / all_to_all / unpack
        barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            for k, (_, call, _) in enumerate(ops):
                if k == 0:
                    if world > 1:
                        ev[i][0].record(stream)
                    timing["on"] = True
                r = call()
                if k == 0:
                    timing["on"] = False
                    if world > 1:
                        ev[i][1].record(stream)
                del r
        barrier()
        elapsed = time.perf_counter() - t0
        be.permute = permute0
        phases = {}
        rccl_ms = None
        if bdist.PROFILE is not None:
            for k, evs in bdist.PROFILE.items():
                phases[k] = float(np.mean([a.elapsed_time(z) for a, z in evs]))
            if bdist.PROFILE.get("rccl"):
                # the RCCL groups alone (all pipeline stages of a swap), per swap
                rccl_ms = float(np.sum([a.elapsed_time(z) for a, z in bdist.PROFILE["rccl"]])) / steps
            bdist.PROFILE = None
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64)  # host tensor: over gloo
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())

        check = None
        if world > 1:
            # the multi-GPU exchange, bit for bit, outside the timed region
            ok = exchange_check(torch, cfg, b, ctx, dev)
            flag = torch.tensor([0.0 if ok else 1.0])
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            check = ("bit-exact on every rank (%s of the global array rebuilt from each rank's seed)" % ops[0][0]
                     if float(flag.item()) == 0.0 else "MISMATCH on at least one rank")

        # On one GPU the swap call is the one permute launch, so only the kernel's
        # own event pair is recorded (each extra stream event adds a few us between
        # the kernels); across GPUs the call's pair brackets the whole exchange.
        kern_ms = float(np.mean([a.elapsed_time(z) for a, z in kev])) if kev else None
        swap_ms = float(np.mean([a.elapsed_time(z) for a, z in ev])) if world > 1 else kern_ms
        if kern_ms is None:  # (no permute launch in the op: the step's wall time bounds it)
            kern_ms = swap_ms if swap_ms is not None else elapsed / steps * 1e3
            swap_ms = kern_ms
        per = {name: nb * world for name, _, nb in ops}
        total = sum(per.values()) * steps
        value = total / elapsed / 1e9
        swap_bytes_rank = ops[0][2]
        achieved = swap_bytes_rank / (kern_ms / 1e3) / 1e9

        line = {
            "metric": "swap/transpose GB/s + stat-reduce GB/s, % of HBM/xGMI roofline, 1-8 GPUs",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"float32": "f32", "float64": "f64", "uint16": "u16"}[np.dtype(dtype).name],
            "data": "synthetic (generated in HBM: 1000+50*N(0,1) float32 / N(0,1) float64 / uniform uint16)",
            "config": {"workload": desc, "global_shape": list(gshape), "split": split,
                       "parallelism": "dp%d (records sharded on the leading key axis)" % world,
                       "collectives": ("none (single GPU)" if world == 1 else
                                       "RCCL via libbolt_mi355x (bm_alltoallv / bm_allgatherv)" if ctx.comm
                                       else "%s, host-staged (one-GPU rehearsal, not a measurement)" % backend),
                       "bytes_per_step": {k: int(v) for k, v in per.items()}},
            "roofline": {
                "bound": "hbm",
                "kernel": "%s (bm_permute) for the %s" % (ROOFLINE_KERNEL[cfg], ops[0][0]) if world == 1 else
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
        if world > 1:
            line["exchange_check"] = check
            G = world
            xport = "RCCL" if backend == "nccl" else "%s (host-staged rehearsal)" % backend
            n_rank = ops[0][2] / 2                        # bytes held per rank
            payload = n_rank * (G - 1) / G                # bytes each rank sends to its peers
            ex = phases.get("exchange")
            if ex:  # the swap across GPUs: pipelined pack -> RCCL all-to-all -> unpack
                line["roofline"].update({"kernel": "swap exchange per rank (k_transpose pack + %s "
                                                   "all_to_all + k_rowcopy unpack, pipelined)" % xport,
                                         "achieved": round(2 * n_rank / (ex / 1e3) / 1e9, 1),
                                         "avg_ms": round(ex, 4), "bytes_per_launch": int(2 * n_rank)})
                line["roofline"]["frac"] = round(line["roofline"]["achieved"] / HBM_PEAK_GBPS, 4)
            a2a = phases.get("exchange")
            peak = (G - 1) * XGMI_LINK_GBPS
            line["xgmi"] = {"op": ("RCCL send/recv group (bm_alltoallv)" if backend == "nccl" else
                                   "%s all_to_all" % xport) + " inside the pipelined swap exchange "
                                  "(achieved = peer payload / whole exchange time: a lower bound)",
                            "payload_bytes_per_rank": int(payload),
                            "avg_ms": round(a2a, 4) if a2a else None,
                            "achieved": round(payload / (a2a / 1e3) / 1e9, 1) if a2a else None,
                            "peak": peak, "unit": "GB/s per rank (egress)",
                            "frac": round(payload / (a2a / 1e3) / 1e9 / peak, 4) if a2a else None,
                            "phases_ms": {k: round(v, 4) for k, v in phases.items()}}
            if rccl_ms:
                # isolated: hipEvents around each bm_alltoallv on the RCCL stream
                # (stages overlap pack / unpack, so this is the links' own time)
                line["xgmi"]["rccl_ms_per_swap"] = round(rccl_ms, 4)
                line["xgmi"]["rccl_achieved"] = round(payload / (rccl_ms / 1e3) / 1e9, 1)
                line["xgmi"]["rccl_frac"] = round(payload / (rccl_ms / 1e3) / 1e9 / peak, 4)
        try:  # the placement-adaptive transpose order's decisions
            import ctypes
            from bolt_amd.mi355x import _lib
            summ = (ctypes.c_int64 * 3)()
            if _lib.load().bm_tune_summary(summ) == 0:
                line["roofline"]["order_tuner"] = {"entries": int(summ[0]), "decided": int(summ[1]),
                                                   "staggered": int(summ[2])}
        except Exception:
            pass
        line["roofline"]["frac_of_measured_copy"] = round(line["roofline"]["achieved"] / HBM_COPY_GBPS, 4)
        line["roofline"]["measured_copy_peak"] = HBM_COPY_GBPS
        return line

    line = measure(args.config, args.steps, args.warmup)
    if line is None:
        return
    shape, dtype, split, desc = CONFIGS[args.config]
    if rank == 0 and world == 1 and not args.no_pmc:
        traffic, note = pmc_traffic(args.config)
        line["roofline"]["traffic"] = int(traffic) if traffic else None
        line["roofline"]["traffic_note"] = note
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rows = args.cpu_sample_rows or 2000
        line["cpu_baseline"] = cpu_baseline(args.config, shape, dtype, rows)
    if world == 1 and args.config == "C2" and not args.no_target64:
        # BASELINE.json's target sentence: swap and statistics of a 64 GiB
        # float32 4-D array on one GPU at >= 60% of the HBM roofline
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        t = measure("target64", args.target_steps, 1)
        sub = {"workload": CONFIGS["target64"][3], "value": t["value"], "unit": "GB/s",
               "ms_per_step": t["ms_per_step"], "steps": t["steps"], "warmup": t["warmup"],
               "global_shape": t["config"]["global_shape"], "bytes_per_step": t["config"]["bytes_per_step"],
               "frac_of_hbm_peak": round(t["value"] / HBM_PEAK_GBPS, 4),
               "target": "swap + mean/std of 64 GiB on 1 GPU at >= 0.60 of HBM (swap <= 28.6 ms)",
               "roofline": t["roofline"]}
        if not args.no_pmc:
            traffic, note = pmc_traffic("target64")
            sub["roofline"]["traffic"] = int(traffic) if traffic else None
            sub["roofline"]["traffic_note"] = note
        line["target64"] = sub
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        barrier()
        ctx.close()  # the library's RCCL communicator, before the process group
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
