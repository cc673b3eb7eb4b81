"""The RCCL layer of libbolt_mi355x (include/bolt_mi355x.h, bm_comm.hip) on one GPU.

A world-1 communicator drives every entry point: the id, init, info, the
all-to-all (the self block is a local device copy; sync and on the context's
RCCL stream with event fences, as the pipelined swap uses it), the
all-gather in both its ncclAllGather form and its point-to-point form, the
error paths (a mismatched self block is refused; a wait that times out
aborts the communicator and every later call fails with BM_E_COMM instead of
hanging), and destroy.  The multi-rank logic around these calls (block sizes, offsets,
stages) is exercised by tests/test_dist_gloo.py over gloo; RCCL cannot put
two ranks on one GPU, so N > 1 over RCCL runs in the driver's 8-GPU bench.
Reference site replaced: bolt/spark/chunk.py:251-261 (shuffle #1).
"""
import ctypes

import numpy as np
import pytest

from bolt_amd.mi355x import _lib
from bolt_amd.mi355x import dist as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    lib = _lib.load()
    uid = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
    _lib.check(lib.bm_comm_unique_id(uid, _lib.COMM_ID_BYTES), "bm_comm_unique_id")
    c = ctypes.c_void_p()
    _lib.check(lib.bm_comm_init(ctypes.byref(c), 1, uid, 0), "bm_comm_init")
    yield c.value
    _lib.check(lib.bm_comm_destroy(c.value), "bm_comm_destroy")


class _Ctx(object):
    """The attributes of MI355XContext the exchange helpers read."""

    def __init__(self, comm):
        import torch
        self.comm = comm
        self.comm_stream = torch.cuda.Stream()
        self.rank, self.world_size = 0, 1
        self.transport = "rccl"
        self.comm_timeout = 60.0


def _new_comm():
    lib = _lib.load()
    uid = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
    _lib.check(lib.bm_comm_unique_id(uid, _lib.COMM_ID_BYTES), "bm_comm_unique_id")
    c = ctypes.c_void_p()
    _lib.check(lib.bm_comm_init(ctypes.byref(c), 1, uid, 0), "bm_comm_init")
    return c.value


def test_mismatched_self_block_is_an_error(comm):
    """send_bytes[rank] != recv_bytes[rank]: refused before anything is queued."""
    import torch
    lib = _lib.load()
    x = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    y = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    rc = lib.bm_alltoallv(comm, x.data_ptr(), _lib.i64_array([4096]), _lib.i64_array([0]), y.data_ptr(),
                          _lib.i64_array([2048]), _lib.i64_array([0]), torch.cuda.current_stream().cuda_stream)
    assert rc == _lib.BM_E_ARG
    assert b"self block mismatch" in lib.bm_last_error()
    assert lib.bm_comm_check(comm) == 0  # the communicator is unharmed


def test_wait_timeout_aborts_instead_of_hanging():
    """A stream that does not drain within the limit (a spin kernel standing in
    for an exchange whose peer never posts): bm_comm_wait returns BM_E_COMM,
    the communicator is aborted, later exchanges fail fast, destroy works."""
    import time
    import torch
    lib = _lib.load()
    c = _new_comm()
    st = torch.cuda.Stream()
    # calibrate torch's spin kernel to ~1 s (bounded: it always ends)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record()
        torch.cuda._sleep(10 ** 7)
        e1.record()
    torch.cuda.synchronize()
    per = max(e0.elapsed_time(e1), 1e-3) / 1e7           # ms per cycle
    cycles = int(min(2e11, 1000.0 / per))
    with torch.cuda.stream(st):
        torch.cuda._sleep(cycles)
    t0 = time.perf_counter()
    rc = lib.bm_comm_wait(c, st.cuda_stream, 0.1)
    waited = time.perf_counter() - t0
    assert rc == _lib.BM_E_COMM, rc
    assert b"not complete" in lib.bm_last_error()
    assert waited < 15.0
    assert lib.bm_comm_check(c) == _lib.BM_E_COMM
    x = torch.zeros(64, dtype=torch.uint8, device="cuda")
    rc = lib.bm_alltoallv(c, x.data_ptr(), _lib.i64_array([64]), _lib.i64_array([0]), x.data_ptr(),
                          _lib.i64_array([64]), _lib.i64_array([0]), st.cuda_stream)
    assert rc == _lib.BM_E_COMM
    with pytest.raises(_lib.BoltCommError):
        _lib.check(rc, "bm_alltoallv")
    torch.cuda.synchronize()   # the spin kernel ends by itself
    assert lib.bm_comm_destroy(c) == 0


def test_wait_ok_and_abort(comm):
    import torch
    lib = _lib.load()
    st = torch.cuda.current_stream()
    assert lib.bm_comm_wait(comm, st.cuda_stream, 5.0) == 0
    c = _new_comm()
    assert lib.bm_comm_abort(c) == 0
    assert lib.bm_comm_check(c) == _lib.BM_E_COMM
    assert lib.bm_comm_destroy(c) == 0


def test_info_and_errors(comm):
    lib = _lib.load()
    rank, world = ctypes.c_int(-1), ctypes.c_int(-1)
    where = ctypes.create_string_buffer(512)
    _lib.check(lib.bm_comm_info(comm, ctypes.byref(rank), ctypes.byref(world), where, 512), "bm_comm_info")
    assert (rank.value, world.value) == (0, 1)
    assert b"rccl" in where.value.lower()
    assert lib.bm_comm_unique_id(ctypes.create_string_buffer(8), 8) == -1  # BM_E_ARG
    bad = _lib.i64_array([-1])
    assert lib.bm_alltoallv(comm, None, bad, _lib.i64_array([0]), None, _lib.i64_array([0]),
                            _lib.i64_array([0]), None) == -1


@pytest.mark.parametrize("nbytes", [1, 4096, 37 << 20])
def test_alltoallv_self(comm, nbytes):
    import torch
    ctx = _Ctx(comm)
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
    got = D._rccl_all_to_all(ctx, src, [nbytes], [nbytes], async_op=False)
    torch.cuda.synchronize()
    assert torch.equal(got, src)
    got2, work = D._rccl_all_to_all(ctx, src, [nbytes], [nbytes], async_op=True)
    work.wait()
    assert torch.equal(got2, src)


def test_allgatherv_both_forms(comm):
    import torch
    lib = _lib.load()
    src = torch.arange(1000, dtype=torch.int32, device="cuda").view(torch.uint8)
    n = src.numel()
    ctx = _Ctx(comm)
    out = D._rccl_all_gather(ctx, src, [n])  # uniform -> ncclAllGather
    torch.cuda.synchronize()
    assert torch.equal(out, src)
    # a non-packed offset takes the point-to-point group
    recv = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    _lib.check(lib.bm_allgatherv(comm, src.data_ptr(), n, recv.data_ptr(), _lib.i64_array([n]),
                                 _lib.i64_array([64]), torch.cuda.current_stream().cuda_stream), "bm_allgatherv")
    torch.cuda.synchronize()
    assert torch.equal(recv[64:], src) and int(recv[:64].sum()) == 0


def test_exchange_helpers_with_a_comm(comm):
    """all_to_all_bytes / all_gather_bytes take the RCCL route when the context
    has a communicator (world 1: the pipelined swap's single peer is itself)."""
    import torch
    ctx = _Ctx(comm)
    x = torch.from_numpy(np.arange(4096, dtype=np.int64)).cuda().view(torch.uint8)
    recv, work = D.all_to_all_bytes(ctx, x, [x.numel()], [x.numel()], 8, async_op=True)
    work.wait()
    assert torch.equal(recv, x)


_CHILD = r"""
import os, sys
sys.path.insert(0, os.environ["BM_ROOT"])
import numpy as np, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["BM_PORT"])
torch.cuda.set_device(0)
dist.init_process_group("cpu:gloo,cuda:nccl", rank=0, world_size=1)  # as bench.py: no eager torch comm
from bolt_amd import MI355XContext
from bolt_amd.mi355x import dist as D
ctx = MI355XContext(device="cuda:0")
assert ctx.comm is None          # world 1: no exchange, no communicator
ctx._init_comm()                 # the rendezvous-store path an N-GPU context takes
ctx.transport = "rccl"
assert ctx.comm is not None and ctx.comm_stream is not None
x = torch.arange(1 << 20, dtype=torch.int32, device="cuda").view(torch.uint8)
recv, work = D._rccl_all_to_all(ctx, x, [x.numel()], [x.numel()], async_op=True)
work.wait()
assert torch.equal(recv, x)
g = D._rccl_all_gather(ctx, x[:4096], [4096])
assert torch.equal(g, x[:4096])
ctx.close()
assert ctx.comm is None
dist.destroy_process_group()
print("child ok")
"""


def test_context_opens_its_communicator_through_the_store():
    """MI355XContext._init_comm on a one-rank nccl group, in a child process:
    rank 0 makes the id, publishes it in the rendezvous store, bm_comm_init,
    an exchange on the context's RCCL stream, close()."""
    import os
    import socket
    import subprocess
    import sys
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, BM_ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), BM_PORT=str(port))
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "child ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("window_kb,total_kb", [(64, 1000), (32 << 10, 80 << 10)])
def test_windowed_egress_over_rccl(comm, monkeypatch, window_kb, total_kb):
    """dist.gather_windows -- the windowed egress toarray() / records() take
    across GPUs -- with the RCCL all-gather (bm_allgatherv on a world-1
    communicator) and the staged D2H, small windows (many all-gathers, no
    staging) and 32-MiB windows (staged through the two page-locked buffers,
    allocated once): the host bytes equal the device bytes."""
    import torch
    monkeypatch.setattr(D, "EGRESS_WINDOW", window_kb << 10)
    ctx = _Ctx(comm)
    n = total_kb << 10
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    calls = []

    def gather(c, piece, part):
        calls.append(sum(part))
        return D._rccl_all_gather(c, piece, part)
    out = D.gather_windows(ctx, x, [n], np.empty(n, np.uint8), gather)
    assert np.array_equal(out, x.cpu().numpy())
    assert len(calls) == -(-n // (window_kb << 10)) and max(calls) <= window_kb << 10
