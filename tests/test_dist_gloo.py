"""Multi-rank orchestration of the mi355x mode on CPU: world_size 2 (and 3) over
gloo, with the numpy test executor (tests/cpu_backend.py) in place of the HIP
kernels.  Covers the paths that exchange data between ranks: the swap's
pack -> all_to_all -> unpack, statistics over the sharded axis (states,
all_gather, ordered Chan combine), output gathers, re-slabbing, and ragged /
empty shards.  The collectives are the same torch.distributed calls the GPU
path makes over RCCL.
"""
import os
import socket
import traceback
from itertools import permutations

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def _body(rank, world, device="cpu"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here)]
    import bolt_amd as bolt
    from bolt_amd import MI355XContext
    import cpu_backend
    if device == "cpu":
        cpu_backend.install()
    else:
        cpu_backend.install_host_staged_gpu()
    ctx = MI355XContext(device=device)
    assert ctx.world_size == world and ctx.rank == rank

    rng = np.random.default_rng(0)
    # C2-like: key = time, swap to key = voxel, stats over time
    x = (1000 + 50 * rng.standard_normal((7, 6, 5))).astype(np.float32)
    b = bolt.array(x, ctx)
    lo, hi = ctx.local_bounds(7)
    assert b._data.numel() == (hi - lo) * 30 * 4
    s = b.swap((0,), (0, 1))
    assert s.shape == (6, 5, 7) and s.split == 2
    assert _exact(s.toarray(), x.transpose(1, 2, 0))
    m = s.mean(axis=2)
    assert m.dtype == np.float32 and np.allclose(m, x.astype(np.float64).mean(0), rtol=1e-6)
    assert np.allclose(s.std(axis=2), x.astype(np.float64).std(0), rtol=1e-6)
    # statistics over the sharded axis
    for name in ("mean", "var", "std", "sum"):
        got = getattr(b, name)(axis=0)
        want = getattr(x.astype(np.float64), name)(axis=0)
        assert np.allclose(got, want, rtol=1e-6), name
        got = getattr(b, name)()
        assert np.allclose(got, getattr(x.astype(np.float64), name)(), rtol=1e-6), name
        got = getattr(b, name)(axis=(0, 2), keepdims=True)
        assert np.asarray(got).shape == (1, 6, 1)
    u = rng.integers(0, 65536, size=(9, 4, 3)).astype(np.uint16)
    bu = bolt.array(u, ctx)
    assert _exact(np.asarray(bu.sum(axis=0)), np.add.reduce(u, axis=0, dtype=np.uint16))
    assert np.allclose(bu.var(axis=0), u.astype(np.float64).var(0), rtol=1e-12)
    assert bu.var(axis=0).dtype == np.float64

    # every permutation of a 4-d array with split 2 (a2a whenever perm[0] != 0),
    # with the exchange in 1 stage and pipelined over 2 and 3 stages
    from bolt_amd.mi355x import dist as bdist
    a = np.arange(5 * 3 * 4 * 2).reshape(5, 3, 4, 2).astype(np.int16)
    ba = bolt.array(a, ctx, axis=(0, 1))
    for stages in (None, 2, 3):
        bdist.STAGES = stages
        for p in permutations(range(4)):
            assert _exact(ba.transpose(p).toarray(), a.transpose(p)), (p, stages)
        y = (np.arange(11 * 7 * 6) % 251).astype(np.float32).reshape(11, 7, 6)
        assert _exact(bolt.array(y, ctx).swap((0,), (0, 1)).toarray(), y.transpose(1, 2, 0))
    bdist.STAGES = None
    # automatic stage count on an uneven leading axis: ranks hold different
    # slabs, so K must come from global sizes or the collectives mismatch
    # (tiny STAGE_BYTES so several stages are chosen)
    bdist.STAGE_BYTES = 64
    for shp in ((world + 1, 6, 10), (2 * world + 1, 5, 7), (world - 1 or 1, 9, 8)):
        u = (np.arange(int(np.prod(shp))) % 1009).astype(np.float32).reshape(shp)
        bu = bolt.array(u, ctx)
        want = u.transpose(1, 2, 0)
        if want.shape[-1] == 1:  # a lone (1,) value axis: the reference's unchunk squeezes it
            want = want.reshape(want.shape[:-1])
        assert _exact(bu.swap((0,), (0, 1)).toarray(), want), shp
        assert _exact(bu.transpose(2, 0, 1).toarray(), u.transpose(2, 0, 1)), shp
    bdist.STAGE_BYTES = None
    assert _exact(ba.keys.transpose((1, 0)).toarray(), a.transpose(1, 0, 2, 3))
    assert _exact(ba.keys.reshape((15,)).toarray(), a.reshape(15, 4, 2))
    assert _exact(ba.values.reshape((8,)).toarray(), a.reshape(5, 3, 8))

    # chunked records stay on their rank; moving the sharded key axis exchanges
    c = ba.chunk((3, 1), padding=(1, 0))
    assert _exact(c.unchunk().toarray(), a)
    recs = list(c.records())
    assert len(recs) == 15 * 2 * 2
    k2v = c.keys_to_values((0,))
    assert _exact(k2v.unchunk().toarray(), a.transpose(1, 0, 2, 3))
    v2k = c.values_to_keys((1,))
    assert _exact(v2k.unchunk().toarray(), a.transpose(0, 1, 3, 2))

    # ingest with non-leading key axes: each rank uploads only the planes of
    # x.transpose(perm) behind its slab (every golden construct case, plus
    # ragged and tiny leading axes)
    import golden_cases as G
    for case in G.cases("construct"):
        if "raises" in case:
            continue
        xg = G.make_input(case["input"])
        bg = bolt.array(xg, ctx, axis=G.tup(case["axis"]))
        assert _exact(bg.toarray(), G.arr(case, "out")), case["id"]
    for shp, ax in (((5, 7, 3), (1,)), ((5, 7, 3), (2, 0)), ((2, 3, 9), (2,)), ((1, 4, 5), (1, 2)),
                    ((4, 3), (1,))):
        xg = np.arange(int(np.prod(shp)), dtype=np.int32).reshape(shp)
        perm = list(ax) + [i for i in range(len(shp)) if i not in ax]
        want = np.ascontiguousarray(xg.transpose(perm)).reshape(shp)
        assert _exact(bolt.array(xg, ctx, axis=ax).toarray(), want), (shp, ax)

    # a reduction of the sharded axis with no outputs (mean(axis=0) of (4, 0, 3))
    e0 = bolt.array(np.zeros((4, 0, 3)), ctx)
    assert np.asarray(e0.mean(axis=0)).shape == (0, 3)
    assert np.asarray(e0.sum(axis=0)).shape == (0, 3)

    # fewer records than ranks: empty shards
    t = np.arange(2 * 3).reshape(1, 2, 3).astype(np.float64)
    bt = bolt.array(t, ctx)
    assert _exact(bt.toarray(), t)
    assert _exact(bt.swap((0,), (0,)).toarray(), t.transpose(1, 0, 2))
    assert np.allclose(bt.mean(axis=0), t.mean(0)) and np.allclose(bt.std(), t.std())
    assert _exact(bolt.ones((3, 4), ctx, dtype=np.int32).toarray(), np.ones((3, 4), np.int32))

    import golden_cases as G
    # concatenation along the sharded axis re-slabs rows; along others it is local
    for case in G.cases("concatenate"):
        if "raises" in case:
            continue
        xg, yg = G.make_input(case["input"]), G.make_input(case["other"])
        bg = bolt.array(xg, ctx, axis=G.tup(case["axis"]))
        other = bolt.array(yg, ctx, axis=G.tup(case["other_axis"])) if case["other_kind"] == "spark" else yg
        r = bg.concatenate(other, axis=case["cat_axis"])
        assert _exact(r.toarray(), G.arr(case, "out")), case["id"]

    # user functions: map / filter / chunk map everywhere; stacked maps whose
    # result keeps the records (stacks are per-rank, so re-keyed counts differ)
    from funcs import FUNCS
    for case in G.cases("map") + G.cases("filter") + G.cases("chunk_map") + G.cases("stack_map"):
        if "raises" in case:
            continue
        xg = G.make_input(case["input"])
        bg = bolt.array(xg, ctx, axis=G.tup(case["axis"]))
        if case["op"] == "map":
            r = bg.map(FUNCS[case["func"]], axis=G.tup(case["map_axis"]), value_shape=G.tup(case["value_shape"]),
                       dtype=case["dtype"], with_keys=case["with_keys"])
        elif case["op"] == "filter":
            r = bg.filter(FUNCS[case["func"]], axis=G.tup(case["filter_axis"]), sort=case["sort"])
            if case["shape"] == [0]:
                assert r.shape == (0,)
                continue
        elif case["op"] == "chunk_map":
            c = bg.chunk(size=G.size_arg(case["size"]), padding=G.tup(case["padding"]))
            r = c.map(FUNCS[case["func"]], value_shape=G.tup(case["value_shape"])).unchunk()
        else:
            if case["shape"][:1] != case["input"]["shape"][:1]:
                continue
            st = bg.stack(case["size"])
            for name in case["funcs"]:
                st = st.map(FUNCS[name])
            r = st.unstack()
        got, want = r.toarray(), G.arr(case, "out")
        assert got.shape == want.shape and got.dtype == want.dtype, case["id"]
        assert np.allclose(got, want, rtol=1e-5, atol=1e-5 * float(np.max(np.abs(want)))), case["id"]

    # reduce(func): ufunc modes through per-rank states and the ordered
    # combine, user functions through per-rank trees and a tree over ranks;
    # Keys / Values reshape re-slab the records
    from funcs import RFUNCS
    for case in G.cases("reduce")[::3] + G.cases("reshape"):
        if "raises" in case:
            continue
        xg = G.make_input(case["input"])
        bg = bolt.array(xg, ctx, axis=G.tup(case["axis"]))
        if case["op"] == "reshape":
            r = getattr(bg, case["which"]).reshape(tuple(case["new"]))
            assert r.split == case["split"] and _exact(r.toarray(), G.arr(case, "out")), case["id"]
            continue
        ax = tuple(case["reduce_axis"])
        got = bg.reduce(RFUNCS[case["func"]], axis=ax, keepdims=case["keepdims"])
        a = np.asarray(got.toarray() if hasattr(got, "toarray") else got)
        assert G.reduce_close(a, G.arr(case, "out"), xg, case["func"], ax), case["id"]

    # a user function that is not elementwise, over a non-leading axis: every
    # call must see whole records (array.py:268-269 aligns first).
    # Matrix products of 4x4 records in record order (associative, not
    # commutative, exact in float64 for 0/1 entries): the bracketing cannot
    # change it.
    mats = np.random.default_rng(5).integers(0, 2, size=(4, 5, 4)).astype(np.float64)
    bm = bolt.array(mats, ctx)
    got = np.asarray(bm.reduce(lambda p, q: p @ q, axis=(1,)).toarray())
    want = np.linalg.multi_dot([mats[:, k, :] for k in range(5)])
    assert _exact(got, want), (got, want)
    got = np.asarray(bm.reduce(lambda p, q: p + q.sum(), axis=(1,)).toarray())
    assert got.shape == (4, 4) and got.dtype == np.float64

    # indexing: every golden getitem / squeeze case (rows move between ranks
    # for selections on the sharded axis; squeezing it re-slabs)
    for case in G.cases("getitem") + G.cases("squeeze"):
        if "raises" in case or "collect_raises" in case:
            continue
        xg = G.make_input(case["input"])
        bg = bolt.array(xg, ctx, axis=G.tup(case["axis"]))
        if case["op"] == "squeeze":
            r = bg.squeeze(G.tup(case["squeeze"]))
            assert r.split == case["split"] and _exact(r.toarray(), G.arr(case, "out")), case["id"]
            continue
        r = bg[G.index_arg(case["index"])]
        want = G.arr(case, "out_sorted" if case.get("toarray_unsorted") else "out")
        if case["kind"] == "scalar":
            assert np.asarray(r).tobytes() == want.tobytes(), case["id"]
        else:
            assert r.split == case["split"] and _exact(r.toarray(), want), case["id"]


def _worker(rank, world, port, errq, device="cpu"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _body(rank, world, device)
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
def test_multirank_gloo(world):
    _run(world, "cpu")


def _transport_worker(rank, world, port, errq):
    """Production transport ("rccl", the HIP backend's) over a gloo-only group
    must refuse -- no host staging of device bytes -- and the test transports
    must never take device tensors."""
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import cpu_backend
        from bolt_amd import MI355XContext
        from bolt_amd.mi355x import dist as bdist
        from bolt_amd.mi355x._ops import register_backend

        class ProductionLike(cpu_backend.CpuBackend):
            transport = "rccl"   # what HipBackend declares

        register_backend("cpu", ProductionLike())
        try:
            MI355XContext(device="cpu")
        except RuntimeError as e:
            assert "RCCL" in str(e) and "gloo" in str(e), str(e)
        else:
            raise AssertionError("a gloo group was accepted for the RCCL transport")
        cpu_backend.install()
        ctx = MI355XContext(device="cpu")
        assert ctx.transport == "torch" and ctx.comm is None

        class _Dev(object):
            type = "cuda"

        class _FakeCuda(object):
            device = _Dev()

        try:
            bdist._check_test_transport(ctx, _FakeCuda())
        except RuntimeError as e:
            assert "RCCL" in str(e)
        else:
            raise AssertionError("device bytes took the torch.distributed path")
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


def test_production_transport_refuses_gloo_group():
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transport_worker, args=(r, 2, port, errq)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join("rank %d:\n%s" % e for e in errs)
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.gpu
def test_multirank_gpu_kernels_one_device():
    """The same multi-rank flow with the HIP kernels: 2 ranks share cuda:0,
    exchanges over gloo staged through the host (RCCL needs distinct GPUs)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(2, "cuda:0")
