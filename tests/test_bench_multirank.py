"""The bench's weak-scaling step (bench.steps_of) at world sizes 4 and 8 over
gloo on the CPU test executor: each rank builds its own shard with
ConstructMI355X.fromshards, as bench.py does under torch.distributed.run, runs
every op of every config, and checks the results against numpy on the global
array.  A rehearsal of the driver's N-GPU scaling run (there over RCCL)."""
import json
import os
import socket
import subprocess
import sys
import traceback

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

# per-rank shard shapes (leading axis grows with the world, as in bench.py)
SHARDS = {
    "C1": ((3, 4, 5), np.float64, 1),
    "C2": ((3, 4, 5), np.float32, 1),
    "C3": ((2, 3, 4, 8), np.float32, 2),
    "C4": ((3, 6, 8), np.uint16, 1),
    "C5": ((2, 2, 2, 20, 20), np.float64, 3),
    "target64": ((2, 3, 4, 8), np.float32, 2),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(cfg, rank):
    shape, dt, _ = SHARDS[cfg]
    rng = np.random.default_rng(100 + rank)
    if np.dtype(dt).kind == "f":
        return (1000 + 50 * rng.standard_normal(shape)).astype(dt)
    return rng.integers(0, 65536, size=shape).astype(dt)


def _body(rank, world):
    sys.path[:0] = [HERE, ROOT]
    import torch
    import cpu_backend
    cpu_backend.install()
    import bench
    from bolt_amd import ConstructMI355X, MI355XContext
    ctx = MI355XContext(device="cpu")
    for cfg, (shape, dt, split) in SHARDS.items():
        full = np.concatenate([_shard(cfg, r) for r in range(world)], axis=0)
        gshape = (shape[0] * world,) + tuple(shape[1:])
        mine = torch.from_numpy(np.ascontiguousarray(_shard(cfg, rank)).reshape(-1).view(np.uint8).copy())
        b = ConstructMI355X.fromshards(mine, gshape, context=ctx, split=split, dtype=dt)
        assert np.asarray(b.toarray()).tobytes() == full.tobytes(), cfg
        ops = bench.steps_of(cfg, b, world)
        results = {name: call() for name, call, _ in ops}
        # every op moves bytes, except a chunk / unchunk whose packed layout is
        # the dense one (C4's chunk('150'): a relabelling)
        assert all(nb > 0 for name, _, nb in ops if name not in ("chunk", "unchunk"))
        x = full.astype(np.float64)
        if cfg == "C1":
            y = x.transpose(1, 0, 2)
            for name in ("sum", "mean", "var", "std"):
                assert np.allclose(results[name + "_all"], getattr(y, name)(), rtol=1e-12), name
                assert np.allclose(results[name + "_0"], getattr(y, name)(axis=0), rtol=1e-12), name
        elif cfg == "C2":
            s = b.swap((0,), (0, 1))
            assert np.asarray(s.toarray()).tobytes() == np.ascontiguousarray(full.transpose(1, 2, 0)).tobytes()
            assert np.allclose(results["mean"], x.mean(0), rtol=1e-6)
            assert np.allclose(results["std"], x.std(0), rtol=1e-6)
        elif cfg == "target64":
            assert np.allclose(results["mean"], x.mean(0), rtol=1e-6)
            assert np.allclose(results["std"], x.std(0), rtol=1e-6)
            assert np.asarray(results["swap"].toarray()).tobytes() == \
                np.ascontiguousarray(full.transpose(1, 2, 0, 3)).tobytes()
        elif cfg == "C3":
            assert np.asarray(results["swap"].toarray()).tobytes() == \
                np.ascontiguousarray(full.transpose(1, 2, 0, 3)).tobytes()
            assert np.asarray(results["T"].toarray()).tobytes() == np.ascontiguousarray(full.T).tobytes()
        elif cfg == "C4":
            assert np.asarray(results["unchunk"].toarray()).tobytes() == full.tobytes()
            assert np.allclose(results["var"], x.var(0), rtol=1e-12)
            assert np.asarray(results["swap"].toarray()).tobytes() == \
                np.ascontiguousarray(full.transpose(1, 0, 2)).tobytes()
        else:  # C5
            assert np.asarray(results["T"].toarray()).tobytes() == np.ascontiguousarray(full.T).tobytes()
            assert np.asarray(results["transpose"].toarray()).tobytes() == \
                np.ascontiguousarray(full.transpose(2, 0, 4, 1, 3)).tobytes()
            assert np.asarray(results["unchunk"].toarray()).tobytes() == full.tobytes()
            # both re-chunkings keep the axis order of this config
            k2v, v2k = results["keys_to_values"], results["values_to_keys"]
            assert k2v.split == 2 and v2k.split == 4
            assert np.asarray(k2v.unchunk().toarray()).tobytes() == full.tobytes()
            assert np.asarray(v2k.unchunk().toarray()).tobytes() == full.tobytes()
        # bench.py's post-timing checks, on shards made the bench's way: the
        # exchange (first op) and every permute bit for bit, every statistic
        # over the sharded axis (C1's, C4's var, target64's mean / std) against
        # the float64 truth of the global array
        t = bench.synth_shard(torch, shape, dt, torch.device("cpu"), 1234 + rank)
        tb = ConstructMI355X.fromshards(t.reshape(-1).view(torch.uint8), gshape, context=ctx, split=split, dtype=dt)
        assert bench.exchange_check(torch, cfg, tb, ctx, torch.device("cpu"), gshape, dt), cfg
        det, ok = bench.run_checks(torch, cfg, tb, ctx, torch.device("cpu"), gshape, dt, world)
        assert ok, (cfg, det)
        names = [n for n, _, _ in bench.checks_of(cfg, tb)]
        assert sorted(det) == sorted(names), (cfg, det)
        # every op of the step is checked
        assert sorted(names) == sorted(n for n, _, _ in bench.steps_of(cfg, tb, world)), cfg
        stats = [n for n, _, spec in bench.checks_of(cfg, tb) if spec[0] == "stat"]
        assert all(det[n].startswith("ok ") for n in stats), det
        assert all(det[n] == "exact" for n in names if n not in stats), det
        if cfg in ("C4", "target64", "C1", "C2"):
            assert stats, cfg  # the statistics are checked
        if cfg in ("C4", "C5"):
            assert [n for n, _, spec in bench.checks_of(cfg, tb) if spec[0] == "packed"], cfg


def _worker(rank, world, port, errq):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _body(rank, world)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("world", [4, 8])
def test_bench_steps_weak_scaling(world):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join("rank %d:\n%s" % e for e in errs)
    assert all(p.exitcode == 0 for p in procs)


def test_stat_checks_catch_a_wrong_result(monkeypatch):
    """The sharded-axis statistic check fails when the result is off by more
    than the stated tolerance (here: one output nudged by 1e-9 relative, over
    the float64 rtol of 1e-12)."""
    sys.path[:0] = [HERE, ROOT]
    import torch
    import bench
    truth = np.linspace(1.0, 2.0, 12)
    ok, _ = bench.stat_within(truth.copy(), truth, truth.max(), "var")
    assert ok
    bad = truth.copy()
    bad[5] *= 1 + 1e-9
    ok, worst = bench.stat_within(bad, truth, truth.max(), "var")
    assert not ok and worst > 1
    ok, _ = bench.stat_within(truth.astype(np.float32), truth, 2.0, "mean")
    assert ok  # float32 output: rtol 1e-6
    del torch


SHAPES = json.dumps({"C1": [5, 6, 4], "C2": [4, 8, 8], "C3": [2, 3, 4, 8], "C4": [6, 16, 16],
                     "C5": [2, 2, 2, 20, 20], "target64": [2, 3, 4, 8]})
STRONG = ("C1", "C3", "C4", "C5")   # BASELINE's global arrays, cut into N slabs


def _bench(args, env_extra, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _every_op_checked(rec):
    assert rec["ops"] and all("ck" in o for o in rec["ops"].values()), rec["ops"]
    assert all(o["ck"] == "exact" or o["ck"].startswith("ok ") for o in rec["ops"].values()), rec["ops"]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_bench_launches_its_ranks(world):
    """`bench.py --gpus N` without WORLD_SIZE starts the N rank processes itself
    and rank 0's JSON line comes back: n_gpus N, the C2 headline weak-scaled,
    C1/C3/C4/C5 strong-scaled on their global shapes (3 ranks: ragged and empty
    slabs), every op of every step checked (the CPU rehearsal: test executor
    over gloo, tiny shapes)."""
    r = _bench(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-pmc", "--no-cpu-baseline",
                "--shapes", SHAPES],
               {"BOLT_AMD_BENCH_BACKEND": "gloo", "BOLT_AMD_BENCH_DEVICE": "cpu"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["launcher"].startswith("bench.py --gpus %d" % world)
    assert d["exchange_check"] == "exact" and d["checks_ok"] is True and d["scaling"] == "weak"
    assert d["config"]["global_shape"][0] == 4 * world
    _every_op_checked(d)
    assert set(d["ops"]) == {"swap", "mean", "std"}
    for cfg in STRONG:
        c = d["configs"][cfg]
        assert c["ok"] is True and c["scaling"] == "strong", (cfg, c)
        assert c["global_shape"] == json.loads(SHAPES)[cfg]
        _every_op_checked(c)
    assert set(d["configs"]["C5"]["ops"]) == {"T", "transpose", "chunk", "unchunk", "keys_to_values",
                                              "values_to_keys"}
    assert d["configs"]["C4"]["ops"]["var"]["ck"].startswith("ok ")
    assert "target64" not in d  # the 64 GiB target is a one-GPU record
    assert "rocprof_marks" not in d and "rocprof" not in d  # no profiler on the CPU rehearsal
    # tuning data of the N-rank run: the swap by pipeline depth, the bare all-to-all by size
    assert set(d["xgmi"]["stages_ms"]) == {"1", "2", "4", "8", "16"}
    assert set(d["a2a"]) == {"4M", "16M", "64M"} and all(len(v) == 3 and v[0] > 0 for v in d["a2a"].values())


def test_bench_refuses_gpu_count_mismatch():
    """More GPUs than visible (none here) without the rehearsal knobs, or a
    --gpus that differs from WORLD_SIZE: exit 2, nothing measured."""
    r = _bench(["--gpus", "2", "--steps", "1"], {}, timeout=120)
    assert r.returncode == 2 and "refusing" in r.stderr and not r.stdout.strip()
    r = _bench(["--gpus", "3", "--steps", "1"], {"WORLD_SIZE": "2"}, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and not r.stdout.strip()


def _find(d, path):
    for k in path.split("."):
        d = d[k]
    return d


def test_bench_one_rank_rehearsal_record():
    """The default run's record on one rank (CPU rehearsal): the driver's
    contract keys, the C2 ops, stats_roofline for mean / std, target64 and the
    C1 / C3 / C4 / C5 sub-records with per-op time, fraction of peak and check;
    and every headline number inside the record's last 7,000 characters (the
    tail the driver keeps), which must parse as JSON from a key on."""
    r = _bench(["--steps", "2", "--warmup", "1", "--no-pmc", "--no-cpu-baseline", "--target-steps", "1",
                "--shapes", SHAPES], {"BOLT_AMD_BENCH_DEVICE": "cpu"})
    assert r.returncode == 0, r.stderr[-3000:]
    text = r.stdout.strip().splitlines()[-1]
    d = json.loads(text)
    # the driver's contract: one JSON line with these keys
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert d["unit"] == "GB/s" and d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "f32"
    assert set(d["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac", "traffic"}
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["peak"] == 8000.0
    assert set(d["ops"]) == {"swap", "mean", "std"} and all(o["B"] > 0 for o in d["ops"].values())
    assert d["n_gpus"] == 1 and set(d["stats_roofline"]) >= {"mean", "std"}
    assert d["stats_roofline"]["mean"]["nl"] == 1.0
    _every_op_checked(d)
    t = d["target64"]
    assert t["ops"]["mean"]["ck"].startswith("ok ") and t["ops"]["swap"]["ck"] == "exact" and t["ok"] is True
    for cfg, ops in (("C3", {"swap", "T"}), ("C4", {"swap", "chunk", "unchunk", "var"}),
                     ("C5", {"T", "transpose", "chunk", "unchunk", "keys_to_values", "values_to_keys"})):
        c = d["configs"][cfg]
        assert set(c["ops"]) == ops and c["dominant"] in ops
        assert all(o["ms"] is None or o["ms"] > 0 for o in c["ops"].values())
        assert c["ok"] is True
        _every_op_checked(c)
    # the prose lives in the detail file the record names
    det = json.load(open(os.path.join(ROOT, d["detail"])))
    assert det["value"] == d["value"] and "C3" in det["prose"]["workloads"]
    # the driver keeps the last 7,000 characters: all of these must be there
    tail = text[-7000:]
    wanted = ["target64.roofline.frac", "stats_roofline.mean.frac", "stats_roofline.std.frac", "roofline.frac"]
    wanted += ["configs.%s.ops.%s.frac" % (c, o) for c, rec in d["configs"].items() for o, v in rec["ops"].items()
               if "frac" in v]
    wanted += ["configs.%s.ops.%s.ck" % (c, o) for c, rec in d["configs"].items() for o in rec["ops"]]
    for path in wanted:
        keys = path.split(".")
        # each key of the path appears in the tail, in order, and the value is the record's
        assert all('"%s":' % k in tail for k in keys), path
    # the tail from the configs on parses by itself
    i = tail.index('"configs":')
    sub = json.loads("{" + tail[i:])
    for c, rec in d["configs"].items():
        for o, v in rec["ops"].items():
            assert sub["configs"][c]["ops"][o] == v
    assert sub["target64"]["roofline"]["frac"] == _find(d, "target64.roofline.frac")
    assert sub["stats_roofline"]["mean"]["frac"] == _find(d, "stats_roofline.mean.frac")


def test_record_length_budget():
    """The stdout record at the full default run's size stays inside the
    7,000 characters the driver keeps: a record with every field the GPU run
    fills (PMC traffic ratios, the CPU baseline, wide numbers) is built from
    the rehearsal's and measured."""
    r = _bench(["--steps", "1", "--warmup", "1", "--no-pmc", "--no-cpu-baseline", "--target-steps", "1",
                "--config-steps", "1", "--shapes", SHAPES], {"BOLT_AMD_BENCH_DEVICE": "cpu"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])

    def widen(o):
        if isinstance(o, dict):
            if "B" in o:
                o.update({"B": 137438953472, "ms": 23.9276, "frac": 0.7181, "tr": 1.0001})
            for v in o.values():
                widen(v)
    widen(d)
    d["roofline"].update({"traffic": 4194738176, "traffic_ratio": 1.0001, "achieved": 5726.3})
    d["target64"]["roofline"]["traffic_ratio"] = 1.0001
    d["value"] = 6084.33
    d["cpu_baseline"] = {"value": 0.4716, "unit": "GB/s", "cores": 1, "kind": "port",
                         "sample": "oracle Spark-path port, f32 (500,512,512), 1 core, best of 3",
                         "local_numpy": {"value": 5.437, "cores": 1,
                                         "sample": "numpy local mode, whole C2 f32 (2000,512,512), 1 core, best of 3"},
                         "spark_local8": {"value": 0.3912, "cores": 8,
                                          "sample": "Spark local[8] analogue, 8 processes, f32 (500,512,512)"},
                         "openmp": {"value": 75.812, "cores": 16,
                                    "sample": "OpenMP local step, 16 threads, f32 (2000,512,512)"}}
    text = json.dumps(d, separators=(",", ":"))
    assert len(text) <= 7000, len(text)


def test_rocprof_windows_on_a_synthetic_trace():
    """bench.rocprof_windows on a committed synthetic rocprofv3 kernel trace
    (tests/fixtures/rocprof_kernel_trace_synth.csv): 2 steps of a swap (4 pack /
    unpack launches, two overlapping RCCL groups on another stream, a runtime
    copy) and a mean (a reduction and a small all-gather), each call between
    two spin-kernel markers; warm-up kernels before the first marker are not
    counted.  Then merge_rocprof puts the swap's numbers into xgmi."""
    sys.path.insert(0, ROOT)
    import bench
    trace = os.path.join(HERE, "fixtures", "rocprof_kernel_trace_synth.csv")
    marks = [["C2", ["swap", "mean"], 2]]
    info = {"C2.swap": [150000000, 400000000]}
    w = bench.rocprof_windows(trace, marks, info, world=4)
    s, m = w["C2.swap"], w["C2.mean"]
    assert s["n"] == 2 and m["n"] == 2
    assert s["span"] == 0.708 and s["rccl"] == 0.5 and s["rccl_n"] == 2 and s["lib"] == 0.4 and s["blit"] == 0.01
    assert s["xgmi_GBs"] == 300.0 and s["xgmi_frac"] == round(300.0 / (3 * 153.0), 4)
    assert s["pu_frac"] == round(1000.0 / 8000.0, 4)
    assert m["span"] == 0.238 and m["rccl"] == 0.02 and m["lib"] == 0.2 and "xgmi_frac" not in m
    with pytest.raises(RuntimeError):
        bench.rocprof_windows(trace, [["C2", ["swap", "mean"], 3]], info, world=4)
    line = {"config": {"name": "C2"}, "ops": {"swap": {}, "mean": {}}, "xgmi": {}}
    bench.merge_rocprof(line, w, "gpurun_out/x.csv")
    assert line["xgmi"]["rocprof_ms"] == 0.5 and line["xgmi"]["rocprof_frac"] == s["xgmi_frac"]
    assert line["xgmi"]["pack_unpack_frac"] == 0.125 and line["rocprof"]["ops"] is w
    assert bench.kernel_class("void k_transpose<unsigned int, 64, 256, 4, 4, false>(X)") == "lib"
    assert bench.kernel_class("ncclDevKernel_Generic_4(x)") == "rccl"
    assert bench.kernel_class("__amd_rocclr_copyBuffer") == "blit"
    assert bench.kernel_class("at::cuda::(anonymous namespace)::spin_kernel(long)") == "marker"
    assert bench.kernel_class("void at::native::vectorized_elementwise_kernel<16, X>(int, X)") == "torch"


def test_rocprof_only_on_gpu_ranks(monkeypatch):
    """rank 0 goes under rocprofv3 only in an N-rank GPU run (never on one
    rank, on the CPU rehearsal, with --no-rocprof or BOLT_AMD_BENCH_ROCPROF=0)."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(bench, "rocprof_path", lambda: "/opt/rocm/bin/rocprofv3")
    a = bench.parse(["--gpus", "2"])
    assert bench.rocprof_wanted(a, 2, "0") and not bench.rocprof_wanted(a, 1, "0")
    assert not bench.rocprof_wanted(a, 2, "cpu")
    assert not bench.rocprof_wanted(bench.parse(["--no-rocprof"]), 2, "0")
    monkeypatch.setenv("BOLT_AMD_BENCH_ROCPROF", "0")
    assert not bench.rocprof_wanted(a, 2, "0")


@pytest.mark.parametrize("cfg,shape,dtype", [
    ("C3", (4, 8, 8, 32), np.float32), ("C4", (6, 16, 16), np.uint16),
    ("C5", (2, 4, 4, 4, 4), np.float64), ("target64", (4, 8, 8, 32), np.float32)])
def test_local_numpy_baseline_fields(cfg, shape, dtype, monkeypatch):
    """bench.py's CPU baseline for the non-default configs: the reference local
    mode's numpy calls on a leading-axis slab, one thread, reported as GB/s."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.setitem(bench.LOCAL_SAMPLE_ROWS, cfg, 2)
    r = bench.cpu_baseline(cfg, shape, dtype, rows=None)
    assert r["unit"] == "GB/s" and r["cores"] == 1 and r["kind"] == "port"
    assert r["value"] > 0 and "(2," in r["sample"] and r["reps"] == 3 and "best of 3" in r["sample"]


def test_c2_cpu_baseline_method(monkeypatch):
    """SURVEY 8(d)'s method on every C2 CPU line: best of 3 after 1 warm-up;
    the OpenMP line states its threads and why they are fewer than the host's."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "2")
    r = bench.cpu_baseline("C2", (6, 8, 8), np.float32, rows=4)
    assert r["reps"] == 3 and r["local_numpy"]["reps"] == 3 and r["spark_local8"]["reps"] == 3
    assert "best of 3 after 1 warm-up" in r["sample"]
    omp = r["openmp"]
    if omp.get("value") is not None:
        assert omp["reps"] == 3 and omp["cores"] == 2 and omp["affinity_cpus"] >= 1
        if (os.cpu_count() or 1) > 2:
            assert "OMP_NUM_THREADS=2" in omp["cores_reason"]
