"""Multi-rank egress (toarray / ChunkedArray.records) gathered window by window
(dist.gather_to_host): world 4 over gloo with the numpy test executor, windows
smaller than one rank's slab.  The host result must be bit-exact, and no
collective of the egress may move more than one window -- device memory per
rank stays at its slab plus one window (the reference's collect goes to the
driver, bolt/spark/array.py:1006-1014; it never replicates the array)."""
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _body(rank, world, window):
    sys.path[:0] = [HERE, ROOT]
    import cpu_backend
    import bolt_amd as bolt
    from bolt_amd import MI355XContext
    from bolt_amd.mi355x import dist as bdist
    cpu_backend.install()
    ctx = MI355XContext(device="cpu")
    bdist.EGRESS_WINDOW = window
    moved = []
    orig = bdist.all_gather_bytes

    def spy(ctx_, local, sizes):
        moved.append(sum(int(v) for v in sizes))
        return orig(ctx_, local, sizes)
    bdist.all_gather_bytes = spy
    try:
        rng = np.random.default_rng(7)
        x = rng.standard_normal((13, 6, 10))              # 13 rows: ragged slabs over 4 ranks
        b = bolt.array(x, ctx)
        slab = b._data.numel()
        moved.clear()
        got = b.toarray()
        assert got.dtype == x.dtype and got.tobytes() == x.tobytes()
        assert moved and max(moved) <= window, (moved, window)
        assert window < slab  # the window really is smaller than one slab
        assert len(moved) == -(-x.nbytes // window)
        # a permuted (exchanged) array and an integer one
        s = b.swap((0,), (0,))
        assert s.toarray().tobytes() == np.ascontiguousarray(x.transpose(1, 0, 2)).tobytes()
        u = rng.integers(0, 65536, size=(9, 5, 7)).astype(np.uint16)
        assert bolt.array(u, ctx).toarray().tobytes() == u.tobytes()
        # chunk records
        c = b.chunk((4, 4), padding=1)
        moved.clear()
        recs = list(c.records())
        assert moved and max(moved) <= window
        k, v = recs[0]
        assert k == (0, 0, 0) and v.tobytes() == np.ascontiguousarray(x[0, :5, :5]).tobytes()
        assert len(recs) == 13 * 2 * 3
        # empty and 0-d arrays
        e = bolt.array(np.zeros((0, 3)), ctx)
        assert e.toarray().shape == (0, 3)
    finally:
        bdist.all_gather_bytes = orig
        bdist.EGRESS_WINDOW = None


def _worker(rank, world, port, window, errq):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _body(rank, world, window)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("window", [96, 1000])
def test_windowed_egress_world4(window):
    world = 4
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, window, errq)) for r in range(world)]
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
