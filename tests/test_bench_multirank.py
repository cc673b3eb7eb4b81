"""The bench's weak-scaling step (bench.steps_of) at world sizes 4 and 8 over
gloo on the CPU test executor: each rank builds its own shard with
ConstructMI355X.fromshards, as bench.py does under torch.distributed.run, runs
every op of every config, and checks the results against numpy on the global
array.  A rehearsal of the driver's N-GPU scaling run (there over RCCL)."""
import os
import socket
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
        # bench.py's post-timing check of the exchange, on shards made the bench's way
        t = bench.synth_shard(torch, shape, dt, torch.device("cpu"), 1234 + rank)
        tb = ConstructMI355X.fromshards(t.reshape(-1).view(torch.uint8), gshape, context=ctx, split=split, dtype=dt)
        assert bench.exchange_check(torch, cfg, tb, ctx, torch.device("cpu"), shape, dt, split), cfg


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
    assert r["value"] > 0 and "(2," in r["sample"]
