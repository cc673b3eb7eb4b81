"""Row-padded transposed results (bolt_amd/mi355x/array.py, ROW_PITCH).

A swap / transpose whose output rows are not a whole number of 128-B lines is
stored with padded rows; statistics over the last axis read them in place
(bm_reduce_rows), swaps / transposes and permuted reductions read them with
the pitch as the source row stride, and every other use compacts them first.  Results must be
the dense layout's: statistics against numpy (float64 truth within
golden_cases.reduce_close for float sums, exact otherwise), data movement
bit-exact.  The size thresholds are lowered here (``small_pitch``) so that the
small arrays of the seeded suites take the padded path too; the oracle suites
(tests/test_fuzz_oracle.py, test_api_fuzz.py, test_getitem_fuzz.py,
test_chunk_fuzz.py) then run again over padded swap results.  Runs on the CPU
test executor and (marker ``gpu``) on the HIP kernels.
"""
import os

import numpy as np
import pytest

import bolt_amd as bolt
import bolt_amd.mi355x.array as A
import golden_cases as G


@pytest.fixture
def small_pitch(monkeypatch):
    """Pad every transposed row that is not a multiple of 16 B, to 64 B."""
    monkeypatch.setattr(A, "_PITCH_MIN_ROW", 1)
    monkeypatch.setattr(A, "_PITCH_LINE", 16)
    monkeypatch.setattr(A, "_PITCH_ALIGN", 64)
    monkeypatch.setattr(A, "_PITCH_PAD_DIV", 0)
    monkeypatch.setattr(A, "_PITCH_PLANS", {})


def _padded(b):
    return "_pbuf" in b.__dict__


def _mv(shape, perm):
    return A._move_plan(shape, perm, 1)


def test_pitch_plan_thresholds():
    # C2: swap((0,),(0,1)) of (2000, 512, 512) float32 -> rows of 2000 at 8192 B
    pp = A._pitch_plan(_mv((2000, 512, 512), (1, 2, 0)), (2000, 512, 512), 4)
    assert pp is not None
    P, rows, oshape, sstr, dstr = pp
    assert P == 2048 and rows == 512 * 512 and oshape == [512, 512, 2000]
    assert sstr == [512, 1, 512 * 512] and dstr == [512 * 2048, 2048, 1]
    # float64 rows of 16000 B are whole lines already
    assert A._pitch_plan(_mv((2000, 512, 512), (1, 2, 0)), (2000, 512, 512), 8) is None
    # the last axis stays put: a row copy, rows written whole
    assert A._pitch_plan(_mv((4096, 256, 250), (1, 0, 2)), (4096, 256, 250), 4) is None
    # short rows, rows whose padding would exceed 1/16 and whole-line rows stay dense
    assert A._pitch_plan(_mv((250, 64), (1, 0)), (250, 64), 4) is None        # 1000 B
    assert A._pitch_plan(_mv((1000, 64), (1, 0)), (1000, 64), 2)[0] == 1024   # 2000 -> 2048 B
    assert A._pitch_plan(_mv((400, 64), (1, 0)), (400, 64), 4) is None        # 1600 -> 1792 B: > 1/16
    assert A._pitch_plan(_mv((1024, 64), (1, 0)), (1024, 64), 4) is None      # 4096 B
    assert A._pitch_plan(_mv((1100, 64), (1, 0)), (1100, 64), 4)[0] == 1152   # 4400 -> 4608 B
    assert A._pitch_plan(_mv((1025, 64), (1, 0)), (1025, 64), 4)[0] == 1088   # 4100 -> 4352 B
    assert A._pitch_plan(_mv((8100, 64), (1, 0)), (8100, 64), 4)[0] == 8128   # 32400 -> 32512 B
    assert A._pitch_plan(_mv((10000, 64), (1, 0)), (10000, 64), 2)[0] == 10112  # C4's u16 rows: 20224 B
    # one row: nothing to align
    assert A._pitch_plan(_mv((2000, 1), (1, 0)), (2000, 1), 4) is None


CASES = [((41, 3, 5), (0,), (0, 1), np.float32),
         ((37, 4, 6), (0,), (0, 1), np.float64),
         ((9, 3, 7), (0,), (1,), np.int16),
         ((21, 2, 3, 5), (0, 1), (1,), np.uint8),
         ((13, 6), (0,), (0,), np.int32),
         ((11, 5, 4), (0,), (0, 1), np.uint16)]


def _data(shape, dtype, seed=0):
    rng = np.random.default_rng(seed)
    if np.dtype(dtype).kind == "f":
        return (3 + rng.standard_normal(shape)).astype(dtype)
    return rng.integers(0, 60, size=shape).astype(dtype)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_padded_statistics(bctx, small_pitch, case):
    shape, kax, vax, dtype = CASES[case]
    x = _data(shape, dtype, case)
    b = bolt.array(x, bctx, axis=tuple(range(len(kax))))
    s = b.swap(kax, vax)
    assert _padded(s), "the small-pitch settings pad this swap"
    want = np.ascontiguousarray(bolt.array(x, bctx, axis=tuple(range(len(kax)))).swap(kax, vax).toarray())
    last = s.ndim - 1
    for name in ("mean", "var", "std"):
        got = getattr(s, name)(axis=last)
        truth = getattr(want.astype(np.float64), name)(axis=last)
        assert np.allclose(got, truth, rtol=1e-5, atol=1e-6), name
    for name, uf in (("sum", np.add), ("min", np.minimum), ("max", np.maximum)):
        got = np.asarray(getattr(s, name)(axis=last))
        w = np.asarray(uf.reduce(want, axis=last, dtype=want.dtype))
        assert got.dtype == w.dtype and got.shape == w.shape, name
        if name != "sum" or w.dtype.kind in "iub":
            assert got.tobytes() == w.tobytes(), name
        else:
            assert G.reduce_close(got, w, want, "add", (last,)), name
    assert _padded(s), "last-axis statistics read the padded rows in place"
    if s.ndim >= 3:
        # axes that are not one block: permuted to the front straight from the padded rows
        got = s.var(axis=(0, last))
        assert np.allclose(got, want.astype(np.float64).var(axis=(0, last)), rtol=1e-5, atol=1e-6)
        assert _padded(s)
    # a statistic over the leading axis: the columns run over the padded rows
    assert np.allclose(s.mean(axis=0), want.astype(np.float64).mean(axis=0), rtol=1e-5, atol=1e-6)
    m0 = np.asarray(s.max(axis=0))
    assert m0.tobytes() == np.maximum.reduce(want, axis=0).tobytes()
    assert _padded(s)
    # over every axis: moments of float rows are read in place (per-column states
    # over the padded rows, merged on the host); anything else compacts first
    w64 = want.astype(np.float64)
    for name in ("mean", "var", "std"):
        got = getattr(s, name)()
        assert np.allclose(got, getattr(w64, name)(), rtol=1e-5, atol=1e-6), name
    if np.dtype(dtype).kind == "f":
        assert _padded(s) and "_data" not in s.__dict__
    s.sum()
    assert not _padded(s)
    assert s.toarray().tobytes() == want.tobytes()


def _consumers(kax, vax):
    """(name, f(swapped bolt array) -> ndarray)."""
    back = (tuple(range(len(vax))), tuple(range(len(kax))))
    return [
        ("toarray", lambda s: s.toarray()),
        ("T", lambda s: s.T.toarray()),
        ("swap back", lambda s: s.swap(*back).toarray()),
        ("chunk", lambda s: s.chunk((2,) * len(s.values.shape)).unchunk().toarray()),
        ("map", lambda s: s.map(lambda v: v * 2, axis=tuple(range(s.split))).toarray()),
        ("getitem", lambda s: s[1:, ::2].toarray()),
        ("astype", lambda s: s.astype(np.float64).toarray()),
        ("astype same", lambda s: s.astype(s.dtype).toarray()),
        ("clip", lambda s: s.clip(2, 40).toarray()),
        ("concatenate", lambda s: s.concatenate(np.ascontiguousarray(s.toarray()), axis=0).toarray()),
        ("values.reshape", lambda s: s.values.reshape((int(np.prod(s.values.shape)),)).toarray()),
        ("first", lambda s: np.asarray(s.first())),
        ("sum all", lambda s: np.asarray(s.sum(axis=None))),
        ("var axis 0", lambda s: np.asarray(s.var(axis=0))),
        ("max first and last", lambda s: np.asarray(s.max(axis=(0, s.ndim - 1)))),
    ]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_padded_consumers(bctx, small_pitch, monkeypatch, case):
    """Every other use of a padded result equals the same use of the dense one."""
    shape, kax, vax, dtype = CASES[case]
    x = _data(shape, dtype, 100 + case)
    axis = tuple(range(len(kax)))
    for name, f in _consumers(kax, vax):
        s = bolt.array(x, bctx, axis=axis).swap(kax, vax)
        assert _padded(s)
        got = f(s)
        monkeypatch.setattr(A, "ROW_PITCH", False)
        d = bolt.array(x, bctx, axis=axis).swap(kax, vax)
        assert not _padded(d)
        want = f(d)
        monkeypatch.setattr(A, "ROW_PITCH", True)
        got, want = np.asarray(got), np.asarray(want)
        assert got.shape == want.shape and got.dtype == want.dtype, name
        assert got.tobytes() == want.tobytes(), name


@pytest.mark.parametrize("dtype", [np.float32, np.uint16, np.float64])
def test_map_reads_padded_records(bctx, small_pitch, dtype):
    """One row per record (the time series after C2's swap): map, filter and
    chunk see the padded rows as the records, without compacting the array."""
    x = _data((37, 3, 4), dtype, 9)
    s = bolt.array(x, bctx).swap((0,), (0, 1))
    assert _padded(s) and s.split == 2
    want = np.ascontiguousarray(x.transpose(1, 2, 0))
    got = s.map(lambda v: v * 3 + 1, axis=(0, 1)).toarray()
    assert got.tobytes() == (want * 3 + 1).astype(got.dtype).tobytes()
    assert _padded(s), "map over single-row records reads the padded rows"
    for size, pad in (((10,), None), ((10,), (2,)), ((37,), None)):
        c = s.chunk(size, padding=pad)
        assert c.unchunk().toarray().tobytes() == want.tobytes(), (size, pad)
    assert _padded(s), "chunk of single-row records packs from the padded rows"
    keep = s.filter(lambda v: float(v.double().sum() if hasattr(v, "double") else v.sum()) > 0, axis=(0, 1))
    assert keep.shape == (12, 37) and _padded(keep) and _padded(s), "filter gathers padded records"
    assert keep.toarray().tobytes() == want.reshape(12, 37).tobytes()


def test_indexing_reads_padded_rows(bctx, small_pitch, monkeypatch):
    """Slices, ints, lists and points select straight from the padded rows (no
    compaction); the same results (or errors) as the dense layout's."""
    x = _data((41, 3, 5), np.float32, 4)
    for index in ((slice(1, None), slice(None, None, 2)), (0, slice(None), slice(3, 30, 4)), (2, 4, 7),
                  (slice(2, 0, -1), 1, slice(None, None, 3)), ([2, 0],), (slice(None), [4, 1, 3]),
                  (1, slice(None), [5, 0, 40]), ([0, 2], [1, 3]), ([0, 1, 2], [4, 0, 2], [7, 8, 40]),
                  ([1, 2], slice(1, 4), slice(None, None, 5)), (slice(None), slice(None), [39, 2])):
        out = []
        for pitch in (True, False):
            monkeypatch.setattr(A, "ROW_PITCH", pitch)
            s = bolt.array(x, bctx).swap((0,), (0, 1))
            assert _padded(s) == pitch
            try:
                got = s[index]
                out.append(np.asarray(got.toarray() if hasattr(got, "toarray") else got))
            except Exception as e:  # the reference's restrictions, the same either way
                out.append(type(e).__name__)
            if pitch and not isinstance(out[-1], str):
                assert _padded(s), index
        if isinstance(out[0], str):
            assert out[0] == out[1], index
        else:
            assert out[0].shape == out[1].shape and out[0].tobytes() == out[1].tobytes(), index


def test_elementwise_reads_padded_rows(bctx, small_pitch):
    """astype and clip read the padded rows through a strided view."""
    x = _data((41, 3, 5), np.int16, 6)
    s = bolt.array(x, bctx).swap((0,), (0, 1))
    want = np.ascontiguousarray(x.transpose(1, 2, 0))
    assert s.astype(np.float32).toarray().tobytes() == want.astype(np.float32).tobytes()
    assert s.clip(5, 30).toarray().tobytes() == want.clip(5, 30).tobytes()
    same = s.astype(np.int16)
    assert _padded(same) and same.toarray().tobytes() == want.tobytes()
    assert _padded(s)


def test_reshapes_keep_padded_rows(bctx, small_pitch):
    """Key reshapes, value reshapes that keep the last axis and squeezes
    relabel the padded rows; a value reshape of the last axis compacts."""
    x = _data((41, 4, 6), np.float32, 8)
    s = bolt.array(x, bctx).swap((0,), (0, 1))        # (4, 6, 41), split 2
    want = np.ascontiguousarray(x.transpose(1, 2, 0))
    k = s.keys.reshape((24,))
    assert _padded(k) and k.shape == (24, 41) and k.toarray().tobytes() == want.tobytes()
    t = bolt.array(x, bctx).transpose(1, 2, 0)        # (4, 6, 41), split 1
    v = t.values.reshape((2, 3, 41))
    assert _padded(v) and v.shape == (4, 2, 3, 41) and v.toarray().tobytes() == want.tobytes()
    w = t.values.reshape((246,))
    assert not _padded(w) and w.toarray().tobytes() == want.tobytes()
    u = bolt.array(x.reshape(41, 1, 4, 6), bctx, axis=(0, 1)).transpose(1, 2, 3, 0)  # (1, 4, 6, 41), split 2
    assert _padded(u)
    q = u.squeeze(0)
    assert _padded(q) and q.shape == (4, 6, 41) and q.toarray().tobytes() == want.tobytes()


def test_row_pitch_off_is_dense(bctx, small_pitch, monkeypatch):
    monkeypatch.setattr(A, "ROW_PITCH", False)
    x = _data((41, 3, 5), np.float32)
    s = bolt.array(x, bctx).swap((0,), (0, 1))
    assert not _padded(s)
    assert s.toarray().tobytes() == np.ascontiguousarray(x.transpose(1, 2, 0)).tobytes()


NSEEDS = 60
# a soak run takes other seeds: BOLT_AMD_PITCH_SEEDS=start:stop (default 0:NSEEDS)
_SEEDS = range(*[int(v) for v in os.environ.get("BOLT_AMD_PITCH_SEEDS", "0:%d" % NSEEDS).split(":")])


@pytest.fixture
def padded_inputs(small_pitch, monkeypatch):
    """bolt.array builds its arrays as padded transposition results: the
    records of x.moveaxis(-1, 0), transposed back (same shape, split and
    values as x), so every operation of a suite starts from padded rows."""
    orig = bolt.array

    def array(x, context=None, axis=(0,), **kw):
        x = np.asarray(x)
        if x.ndim < 2 or context is None or kw:
            return orig(x, context, axis=axis, **kw)
        y = np.ascontiguousarray(np.moveaxis(x, -1, 0))
        b = orig(y, context, axis=axis)
        return b.transpose(*(tuple(range(1, x.ndim)) + (0,)))
    monkeypatch.setattr(bolt, "array", array)


@pytest.mark.parametrize("seed", _SEEDS)
def test_oracle_fuzz_padded(bctx, padded_inputs, seed):
    from test_fuzz_oracle import check_case
    check_case(bctx, seed)


@pytest.mark.parametrize("seed", _SEEDS)
def test_api_fuzz_padded(bctx, padded_inputs, seed):
    from test_api_fuzz import test_api_fuzz
    test_api_fuzz(bctx, seed)


@pytest.mark.parametrize("seed", _SEEDS)
def test_getitem_fuzz_padded(bctx, padded_inputs, seed):
    from test_getitem_fuzz import test_getitem_fuzz
    test_getitem_fuzz(bctx, seed)


@pytest.mark.parametrize("seed", _SEEDS)
def test_chunk_fuzz_padded(bctx, padded_inputs, seed):
    from test_chunk_fuzz import test_chunk_fuzz
    test_chunk_fuzz(bctx, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.float16, np.int32, np.uint16, np.uint8, np.int64])
def test_gpu_reduce_rows_abi(gpu_ctx, dtype):
    """bm_reduce_rows through the C-ABI against bm_reduce on the compacted rows
    (identical bytes: the same plan over the same values) and numpy."""
    import torch
    from bolt_amd.mi355x import _lib
    from bolt_amd.mi355x._ops import backend_for, dtype_code
    from bolt_amd.mi355x.transfer import to_device
    be = backend_for(torch.device("cuda:0"))
    rng = np.random.default_rng(5)
    for O, R, P in ((3, 2000, 2048), (257, 1000, 1001), (64, 4097, 4160), (5, 1, 3), (1000, 60, 64)):
        x = (rng.standard_normal((O, P)) * 7 + 20).astype(dtype) if np.dtype(dtype).kind == "f" else \
            rng.integers(0, 90, size=(O, P)).astype(dtype)
        padded = to_device(np.ascontiguousarray(x).reshape(-1).view(np.uint8), torch.device("cuda:0"))
        dense = to_device(np.ascontiguousarray(x[:, :R]).reshape(-1).view(np.uint8), torch.device("cuda:0"))
        stats = [_lib.STAT_SUM, _lib.STAT_MAX, _lib.STAT_MIN]
        if np.dtype(dtype).kind == "f" or np.dtype(dtype).itemsize <= 4:
            stats += [_lib.STAT_MEAN, _lib.STAT_VAR, _lib.STAT_STD]
        for stat in stats:
            keep = stat in (_lib.STAT_SUM, _lib.STAT_MAX, _lib.STAT_MIN)
            odt = np.dtype(dtype) if keep else np.dtype(np.float64)
            a = torch.empty(O * odt.itemsize, dtype=torch.uint8, device="cuda:0")
            c = torch.empty_like(a)
            code, ocode = dtype_code(np.dtype(dtype)), dtype_code(odt)
            be.reduce_rows(stat, padded, code, O, R, P, a, ocode)
            be.reduce(stat, dense, code, O, R, 1, c, ocode)
            torch.cuda.synchronize()
            ga, gc = a.cpu().numpy().view(odt), c.cpu().numpy().view(odt)
            if P % (16 // np.dtype(dtype).itemsize) == 0 or stat in (_lib.STAT_MAX, _lib.STAT_MIN) \
                    or (stat == _lib.STAT_SUM and odt.kind in "iu"):
                # the same plan (vector width) as the dense rows: identical bytes
                assert ga.tobytes() == gc.tobytes(), (O, R, P, stat)
            else:
                # an odd pitch reads element-wise: another summation order
                assert np.allclose(ga, gc, rtol=2e-3 if odt == np.float16 else 1e-5), (O, R, P, stat)
            if stat == _lib.STAT_MAX:
                assert a.cpu().numpy().view(odt).tobytes() == x[:, :R].max(axis=1).tobytes()
    with pytest.raises(_lib.BoltDeviceError, match="row_pitch"):
        be.reduce_rows(_lib.STAT_SUM, padded, dtype_code(np.dtype(dtype)), 4, 10, 9, a, dtype_code(np.dtype(dtype)))


@pytest.mark.parametrize("case", range(len(CASES)))
def test_toarray_reads_padded_rows(bctx, small_pitch, monkeypatch, case):
    """toarray / records of a padded result compact window by window into the
    host result (array.py _padded_to_host): the array stays padded and no dense
    device copy is made."""
    shape, kax, vax, dtype = CASES[case]
    x = _data(shape, dtype, 200 + case)
    axis = tuple(range(len(kax)))
    s = bolt.array(x, bctx, axis=axis).swap(kax, vax)
    assert _padded(s)
    got = s.toarray()
    assert _padded(s) and "_data" not in s.__dict__
    monkeypatch.setattr(A, "ROW_PITCH", False)
    want = bolt.array(x, bctx, axis=axis).swap(kax, vax).toarray()
    assert got.shape == want.shape and got.dtype == want.dtype and got.tobytes() == want.tobytes()
    recs = list(s.records())
    assert _padded(s) and len(recs) == int(np.prod(s.shape[:s.split]))


@pytest.mark.gpu
def test_gpu_padded_toarray_windows(gpu_ctx, monkeypatch):
    """A padded swap result larger than one egress window (transfer.CHUNK, set
    to 8 MiB here: 33 windows) goes to the host window by window, bit-exact,
    with the array still padded afterwards."""
    from bolt_amd.mi355x import transfer
    monkeypatch.setattr(transfer, "CHUNK", 8 << 20)
    x = (np.arange(500 * 256 * 512, dtype=np.int64) % 65521).astype(np.float32).reshape(500, 256, 512)
    s = bolt.array(x, gpu_ctx).swap((0,), (0, 1))
    assert _padded(s) and s.__dict__["_pitch"] == 512      # 2000-B rows at 2048 B
    got = s.toarray()
    assert _padded(s) and "_data" not in s.__dict__
    assert got.shape == (256, 512, 500) and got.tobytes() == np.ascontiguousarray(x.transpose(1, 2, 0)).tobytes()


def _padded_ranks_body(rank, world):
    """Padded rows across ranks (round 6): the exchange's unpack writes the
    swap result at the same pitch rule as one GPU, and every consumer reads it
    or compacts it, on every rank."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here)]
    import cpu_backend
    from bolt_amd import MI355XContext
    cpu_backend.install()
    A._PITCH_MIN_ROW, A._PITCH_LINE, A._PITCH_ALIGN, A._PITCH_PAD_DIV = 1, 16, 64, 0
    A._PITCH_PLANS.clear()
    ctx = MI355XContext(device="cpu")
    assert ctx.world_size == world
    for case, (shape, kax, vax, dtype) in enumerate(CASES):
        x = _data(shape, dtype, 300 + case)
        axis = tuple(range(len(kax)))
        s = bolt.array(x, ctx, axis=axis).swap(kax, vax)
        assert _padded(s), (rank, case)
        A.ROW_PITCH = False
        d = bolt.array(x, ctx, axis=axis).swap(kax, vax)
        A.ROW_PITCH = True
        assert not _padded(d)
        want = d.toarray()
        last = s.ndim - 1
        for name in ("mean", "var", "std"):
            got, ref = np.asarray(getattr(s, name)(axis=last)), np.asarray(getattr(d, name)(axis=last))
            assert got.shape == ref.shape and got.tobytes() == ref.tobytes(), (rank, case, name)
        assert _padded(s), "last-axis statistics read the padded slab in place"
        got = s.toarray()
        assert _padded(s) and "_data" not in s.__dict__, "toarray compacts window by window"
        assert got.tobytes() == want.tobytes(), (rank, case)
        # a padded source across GPUs: the exchange's pack reads it in place
        back = (tuple(range(len(vax))), tuple(range(len(kax))))
        t = s.swap(*back)
        assert _padded(s) and t.toarray().tobytes() == d.swap(*back).toarray().tobytes(), (rank, case)
        for name, f in _consumers(kax, vax):
            s2 = bolt.array(x, ctx, axis=axis).swap(kax, vax)
            g = np.asarray(f(s2))
            A.ROW_PITCH = False
            w = np.asarray(f(bolt.array(x, ctx, axis=axis).swap(kax, vax)))
            A.ROW_PITCH = True
            assert g.shape == w.shape and g.dtype == w.dtype and g.tobytes() == w.tobytes(), (rank, case, name)
    # the egress windows: whole rows, several of them, ragged slabs
    from bolt_amd.mi355x import dist as bdist
    bdist.EGRESS_WINDOW = 100
    x = _data((13, 5, 7), np.float32, 9)
    s = bolt.array(x, ctx).swap((0,), (0, 1))
    assert _padded(s) and s.toarray().tobytes() == np.ascontiguousarray(x.transpose(1, 2, 0)).tobytes()
    bdist.EGRESS_WINDOW = None


def _padded_ranks_worker(rank, world, port, errq):
    import traceback
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        _padded_ranks_body(rank, world)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_padded_rows_across_ranks_gloo(world):
    """World 2 / 3 over gloo (CPU executor): both ranks hold padded rows after
    the swap, statistics and toarray exact, toarray without a dense copy."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    procs = [ctx.Process(target=_padded_ranks_worker, args=(r, world, port, errq)) for r in range(world)]
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
