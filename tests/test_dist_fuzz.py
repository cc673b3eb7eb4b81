"""The seeded oracle fuzz (tests/test_fuzz_oracle.py) on several ranks: world
2 and 3 over gloo with the numpy test executor, and 2 ranks sharing cuda:0
with the HIP kernels.  Random shapes give ragged and empty shards, swaps and
transposes that exchange records (pack -> all_to_all -> unpack), chunked
keys_to_values across ranks, and statistics over the sharded axis (per-rank
states -> all_gather -> ordered Chan combine), each compared with the oracle.
"""
import os
import traceback

import pytest
import torch.multiprocessing as mp

from test_dist_gloo import _free_port

SEEDS = range(0, 200, 4)


def _worker(rank, world, port, errq, device):
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bolt_amd import MI355XContext
        import cpu_backend
        if device == "cpu":
            cpu_backend.install()
        else:
            cpu_backend.install_host_staged_gpu()
        ctx = MI355XContext(device=device)
        from test_fuzz_oracle import check_case
        for seed in SEEDS:
            try:
                check_case(ctx, seed)
            except Exception:
                raise AssertionError("seed %d failed" % seed)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


def _run(world, device):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, errq, device)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join("rank %d:\n%s" % e for e in errs)
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("world", [2, 3])
def test_dist_fuzz_gloo(world):
    _run(world, "cpu")


@pytest.mark.gpu
def test_dist_fuzz_gpu_kernels_one_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(2, "cuda:0")


def _padded_worker(rank, world, port, errq, device="cpu"):
    """The four seeded suites on padded inputs across ranks (round 6): every
    array starts as a padded transposition result (tests/test_row_pitch.py's
    padded_inputs), with the pitch thresholds lowered so small arrays pad, so
    the exchanges read and write padded slabs."""
    import sys
    import numpy as np
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bolt_amd
        import bolt_amd.mi355x.array as A
        from bolt_amd import MI355XContext
        import cpu_backend
        if device == "cpu":
            cpu_backend.install()
        else:
            cpu_backend.install_host_staged_gpu()
        A._PITCH_MIN_ROW, A._PITCH_LINE, A._PITCH_ALIGN, A._PITCH_PAD_DIV = 1, 16, 64, 0
        A._PITCH_PLANS.clear()
        orig = bolt_amd.array

        def array(x, context=None, axis=(0,), **kw):
            x = np.asarray(x)
            if x.ndim < 2 or context is None or kw:
                return orig(x, context, axis=axis, **kw)
            y = np.ascontiguousarray(np.moveaxis(x, -1, 0))
            return orig(y, context, axis=axis).transpose(*(tuple(range(1, x.ndim)) + (0,)))
        bolt_amd.array = array
        ctx = MI355XContext(device=device)
        from test_fuzz_oracle import check_case
        from test_api_fuzz import test_api_fuzz
        from test_getitem_fuzz import test_getitem_fuzz
        from test_chunk_fuzz import test_chunk_fuzz
        for seed in range(0, 60, 3):
            for name, f in (("oracle", check_case), ("api", test_api_fuzz), ("getitem", test_getitem_fuzz),
                            ("chunk", test_chunk_fuzz)):
                try:
                    f(ctx, seed)
                except pytest.skip.Exception:
                    continue  # a case the suite itself skips (on every rank alike)
                except Exception:
                    raise AssertionError("%s seed %d failed" % (name, seed))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


def _run_padded(world, device):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_padded_worker, args=(r, world, port, errq, device)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=400)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join("rank %d:\n%s" % e for e in errs)
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("world", [2, 3])
def test_dist_fuzz_padded_gloo(world):
    _run_padded(world, "cpu")


@pytest.mark.gpu
def test_dist_fuzz_padded_gpu_kernels_one_device():
    """The same on the HIP kernels: 2 ranks sharing cuda:0, the exchanges
    staged through the host (RCCL refuses two ranks on one GPU)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_padded(2, "cuda:0")
