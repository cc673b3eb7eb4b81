"""GPU parity of the raw kernels through the C ABI (bm_permute, bm_copy_strided,
bm_reduce*) against numpy on the same seeded inputs.

Data movement is checked bit for bit (uint views); reductions against a
float64/longdouble numpy truth with the tolerances stated per test.
"""
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.uint16, np.float32, np.float64, np.complex128]


def _dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x).reshape(-1).view(np.uint8)).cuda()


def _host(t, dtype, shape):
    return t.cpu().numpy().view(dtype).reshape(shape)


def _be():
    import torch
    from bolt_amd.mi355x._ops import backend_for
    return backend_for(torch.device("cuda", 0))


def _rand(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    n = int(np.prod(shape))
    raw = rng.integers(0, 256, size=n * np.dtype(dtype).itemsize, dtype=np.uint8)
    return raw.view(dtype).reshape(shape)


@pytest.mark.parametrize("dtype", DTYPES)
def test_permute_all_perms_4d(dtype):
    import torch
    be = _be()
    x = _rand((3, 5, 7, 66), dtype, 1)
    src = _dev(x)
    for p in itertools.permutations(range(4)):
        out = torch.empty_like(src)
        be.permute(src, x.shape, p, x.dtype.itemsize, out)
        got = _host(out, x.dtype, tuple(x.shape[i] for i in p))
        want = np.ascontiguousarray(x.transpose(p))
        assert got.tobytes() == want.tobytes(), p


@pytest.mark.parametrize("shape,perm", [
    ((2000, 512), (1, 0)),
    ((129, 257, 3), (2, 0, 1)),
    ((64, 64, 64), (2, 1, 0)),
    ((7, 130, 33), (0, 2, 1)),
    ((1, 1000), (1, 0)),
    ((5,), (0,)),
    ((3, 4, 5, 6, 7), (4, 3, 2, 1, 0)),
    ((4, 6, 8, 10, 3), (2, 0, 4, 1, 3)),
    ((2,) * 8, (0, 3, 4, 7, 1, 2, 5, 6)),
    # tile-shape selection (La = source-contiguous extent, Lb = destination-contiguous)
    ((3000, 16), (1, 0)),        # La 16   -> 16 x 256 tiles
    ((16, 3000), (1, 0)),        # Lb 16   -> 256 x 16 tiles
    ((700, 32), (1, 0)),         # La 32   -> 32 x 128 tiles
    ((40, 300, 32), (2, 1, 0)),  # C3 .T shape family
    ((33, 130, 9), (2, 1, 0)),
    ((2, 8, 300), (2, 0, 1)),
    # kept innermost run of 32-256 B with the two axes around it swapped (runs transpose)
    ((300, 70, 32), (1, 0, 2)),
    ((50, 33, 8), (1, 0, 2)),
    ((17, 40, 4), (1, 0, 2)),
    ((9, 70, 64), (1, 0, 2)),
    ((6, 40, 30, 16), (0, 2, 1, 3)),
    ((40, 7, 30, 16), (2, 1, 0, 3)),
    ((130, 3, 129, 32), (2, 1, 0, 3)),
    # 1-/2-byte transposes on 16-B aligned rows: packed-word tiles, ragged edges
    ((1000, 40), (1, 0)),
    ((528, 2, 144), (2, 1, 0)),
    ((1040, 3, 96), (2, 1, 0)),
    ((48, 1600), (1, 0)),
    # short 16-B aligned axes fused with their continuation (TransDesc Lb1/La1)
    ((100, 24, 16), (2, 1, 0)),
    ((8, 64, 64, 64), (3, 2, 1, 0)),
    ((32, 16, 48, 8), (3, 2, 1, 0)),
    ((12, 20, 36), (2, 0, 1)),
    ((4, 8, 12, 16, 20), (4, 3, 2, 1, 0)),
    ((16, 16, 16, 16), (2, 3, 0, 1)),
    # float64 with 512-B destination rows read from nearby source rows: fused
    # with the continuation, 32 x 128 tiles, a ragged last tile (BM_T8_FUSE512)
    ((5, 3, 7, 64, 64), (2, 0, 4, 1, 3)),
    # fused float32 .T with >= 64 a-tiles: a-tiles spread 32 ways (BM_TR_ASPREAD),
    # a ragged destination axis, and 32 a-tiles (in order)
    ((6, 4, 256, 32), (3, 2, 1, 0)),
    ((7, 3, 128, 32), (3, 2, 1, 0)),
    ((5, 3, 64, 32), (3, 2, 1, 0)),
    ((6, 64, 5, 64), (2, 0, 3, 1)),
    # short rows whose fastest row dim strides the source by >= 64 KiB: the
    # rowcopy walks 16x16 diagonal tiles (Diag16), with and without outer dims,
    # and a row dim that is not a multiple of 16 (row order)
    ((64, 32, 64, 8), (1, 2, 0, 3)),
    ((32, 4, 16, 32, 16), (1, 2, 3, 0, 4)),
    ((48, 20, 40, 8), (1, 2, 0, 3)),
    # round 3: diagonal tiles by row size -- 8x8 up to 1-KiB rows, 16x16 for
    # 1-4-KiB rows (C4's 2-KiB rows), row order beyond 4 KiB or when an
    # extent is not a multiple of the tile side
    ((64, 128, 256), (1, 0, 2)),
    ((40, 24, 8, 512), (1, 2, 0, 3)),
    ((24, 16, 1024), (1, 0, 2)),
])
@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.float32, np.float64, np.complex128])
def test_permute_shapes(shape, perm, dtype):
    import torch
    be = _be()
    x = _rand(shape, dtype, 2)
    src = _dev(x)
    out = torch.empty_like(src)
    be.permute(src, shape, perm, x.dtype.itemsize, out)
    want = np.ascontiguousarray(x.transpose(perm))
    assert _host(out, x.dtype, want.shape).tobytes() == want.tobytes()


def test_copy_strided_subbox_and_broadcast():
    import torch
    be = _be()
    x = _rand((9, 10, 11), np.float32, 3)
    src = _dev(x)
    # sub-box [2:7, 1:9:2, 3:10] into a dense buffer (generic: non-unit inner? no: inner unit)
    want = np.ascontiguousarray(x[2:7, 1:9:2, 3:10])
    out = torch.empty(want.nbytes, dtype=torch.uint8, device="cuda")
    off = (2 * 110 + 1 * 11 + 3) * 4
    be.copy_strided(src, off, out, 0, want.shape, [110, 22, 1], [28, 7, 1], 4)
    assert _host(out, np.float32, want.shape).tobytes() == want.tobytes()
    # strided inner on both sides (generic kernel)
    want2 = np.ascontiguousarray(x[:, :, ::2])
    out2 = torch.zeros(want2.nbytes * 2, dtype=torch.uint8, device="cuda")
    be.copy_strided(src, 0, out2, 0, want2.shape, [110, 11, 2], [120, 12, 2], 4)
    got2 = _host(out2, np.float32, (9, 10, 12))[:, :, ::2]
    assert got2.tobytes() == want2.tobytes()
    # broadcast one element (ones/zeros fill)
    unit = _dev(np.array([1.5], np.float64))
    out3 = torch.empty(8 * 1000, dtype=torch.uint8, device="cuda")
    be.copy_strided(unit, 0, out3, 0, [1000], [0], [1], 8)
    assert np.all(_host(out3, np.float64, (1000,)) == 1.5)


@pytest.mark.parametrize("shape,es", [((1, 5, 1), 8), ((3, 10, 7), 1), ((3, 10, 7), 2), ((4, 9, 33), 4),
                                      ((2, 64, 1024), 16), ((1, 1 << 20, 1), 4), ((600, 37, 4), 4),
                                      ((1, 1000, 3), 2), ((5, 17, 24), 8)])
def test_gather_rows(shape, es):
    """bm_gather_rows: x.take(idx, axis=1) on an (outer, rows, row) byte view,
    unsorted and repeated indices, vector widths 1..16 B, unaligned offsets."""
    import torch
    be = _be()
    n_outer, rows, row = shape
    x = _rand((n_outer, rows, row * es), np.uint8, 7)
    rng = np.random.default_rng(8)
    for n_idx in (1, rows, 3 * rows + 1):
        idx = rng.integers(0, rows, size=n_idx)
        want = np.ascontiguousarray(x[:, idx, :])
        for soff, doff in ((0, 0), (es, 0), (0, 2 * es), (1, 3)):
            src = torch.zeros(x.nbytes + soff, dtype=torch.uint8, device="cuda")
            src[soff:] = _dev(x)
            out = torch.zeros(want.nbytes + doff + 64, dtype=torch.uint8, device="cuda")
            be.gather_rows(src, soff, out, doff, n_outer, rows, row * es, idx)
            got = out.cpu().numpy()
            assert got[doff:doff + want.nbytes].tobytes() == want.tobytes(), (n_idx, soff, doff)
            assert not got[:doff].any() and not got[doff + want.nbytes:].any()
    with pytest.raises(IndexError):
        be.gather_rows(src, 0, out, 0, n_outer, rows, row * es, [rows])


def _ref_stats(x, O, R, I):
    v = x.reshape(O, R, I).astype(np.longdouble)
    mean = v.mean(axis=1)
    var = ((v - mean[:, None, :]) ** 2).mean(axis=1)
    return mean.reshape(-1), var.reshape(-1)


@pytest.mark.parametrize("O,R,I", [(1, 2000, 4096), (1, 100000, 3), (3, 17, 1000), (512, 2000, 1),
                                   (1, 1 << 20, 1), (7, 5, 1), (2, 1, 9), (1, 3, 1)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.uint16, np.int32])
def test_reduce_moments(O, R, I, dtype):
    import torch
    from bolt_amd.mi355x import _lib
    from bolt_amd.mi355x._ops import dtype_code
    be = _be()
    rng = np.random.default_rng(O * 7 + R + I)
    if np.dtype(dtype).kind == 'f':
        x = (1000 + 50 * rng.standard_normal((O, R, I))).astype(dtype)
    else:
        x = rng.integers(0, 60000, size=(O, R, I)).astype(dtype)
    src = _dev(x)
    mean, var = _ref_stats(x, O, R, I)
    out_dt = (np.zeros(1, dtype) - 0.0).dtype
    tol = 1e-6 if out_dt == np.float32 else 1e-12
    for stat, truth in ((_lib.STAT_MEAN, mean), (_lib.STAT_VAR, var), (_lib.STAT_STD, np.sqrt(var))):
        out = torch.empty(O * I * out_dt.itemsize, dtype=torch.uint8, device="cuda")
        be.reduce(stat, src, dtype_code(dtype), O, R, I, out, dtype_code(out_dt))
        got = _host(out, out_dt, (O * I,)).astype(np.longdouble)
        scale = np.abs(truth).max() + (np.sqrt(var).max() if stat == _lib.STAT_MEAN else 0)
        err = np.abs(got - truth).max()
        assert err <= tol * max(scale, 1e-30) + 2 * np.finfo(out_dt).eps * np.abs(truth).max(), (stat, err)


@pytest.mark.parametrize("dtype", [np.uint8, np.int8, np.uint16, np.int16, np.int32, np.uint32,
                                   np.int64, np.uint64, np.bool_, np.float32, np.float64])
@pytest.mark.parametrize("O,R,I", [(1, 3000, 257), (4, 1000, 1), (1, 1 << 18, 1), (5, 3, 6)])
def test_reduce_sum(dtype, O, R, I):
    import torch
    from bolt_amd.mi355x import _lib
    from bolt_amd.mi355x._ops import dtype_code
    be = _be()
    rng = np.random.default_rng(R + I)
    if np.dtype(dtype) == np.bool_:
        x = rng.integers(0, 2, size=(O, R, I)).astype(bool)
        x[:, :, ::3] = False
    elif np.dtype(dtype).kind == 'f':
        x = rng.standard_normal((O, R, I)).astype(dtype)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, info.max, size=(O, R, I), dtype=dtype, endpoint=True)
    src = _dev(x)
    out = torch.empty(O * I * x.dtype.itemsize, dtype=torch.uint8, device="cuda")
    be.reduce(_lib.STAT_SUM, src, dtype_code(dtype), O, R, I, out, dtype_code(dtype))
    got = _host(out, x.dtype, (O, I))
    if x.dtype == np.bool_:
        assert np.array_equal(got, x.any(axis=1))
    elif x.dtype.kind in 'iu':
        want = np.add.reduce(x, axis=1, dtype=x.dtype)  # modular in the input width
        assert got.tobytes() == want.tobytes()
    else:
        truth = x.astype(np.longdouble).sum(axis=1)
        tol = 1e-6 if x.dtype == np.float32 else 1e-12
        assert np.all(np.abs(got - truth) <= tol * np.abs(x).astype(np.longdouble).sum(axis=1) + 1e-300)


@pytest.mark.parametrize("O,R,I", [(1, 1 << 18, 1), (1, 120000, 6)])
@pytest.mark.parametrize("dtype", [np.int32, np.uint16, np.float64, np.float32, np.bool_])
def test_reduce_modes_few_outputs(O, R, I, dtype):
    """Few outputs from hundreds of chunk states (axis=None-like reductions):
    every mode through the block-per-output combine (k_red_combine_blk)."""
    import torch
    from bolt_amd.mi355x import _lib
    from bolt_amd.mi355x._ops import dtype_code
    be = _be()
    rng = np.random.default_rng(R + I)
    dt = np.dtype(dtype)
    if dt == np.bool_:
        x = rng.random((O, R, I)) < 0.9999
        x[0, :, 0] = True  # one all-True column
        stats = {_lib.STAT_LAND: np.logical_and, _lib.STAT_LOR: np.logical_or, _lib.STAT_SUM: np.logical_or,
                 _lib.STAT_MAX: np.maximum, _lib.STAT_MIN: np.minimum, _lib.STAT_PROD: np.logical_and}
    elif dt.kind == 'f':
        x = (1 + 1e-7 * rng.standard_normal((O, R, I))).astype(dt)
        if I > 1:
            x[0, 12345, 1] = np.nan  # NaN wins in maximum/minimum, loses in fmax/fmin
        stats = {_lib.STAT_MAX: np.maximum, _lib.STAT_MIN: np.minimum, _lib.STAT_FMAX: np.fmax,
                 _lib.STAT_FMIN: np.fmin, _lib.STAT_PROD: np.multiply, _lib.STAT_SUM: np.add}
    else:
        info = np.iinfo(dt)
        x = rng.integers(info.min, info.max, size=(O, R, I), dtype=dt, endpoint=True)
        stats = {_lib.STAT_MAX: np.maximum, _lib.STAT_MIN: np.minimum, _lib.STAT_PROD: np.multiply,
                 _lib.STAT_BAND: np.bitwise_and, _lib.STAT_BOR: np.bitwise_or, _lib.STAT_BXOR: np.bitwise_xor,
                 _lib.STAT_LAND: np.logical_and, _lib.STAT_LOR: np.logical_or, _lib.STAT_SUM: np.add}
    src = _dev(x)
    for stat, uf in stats.items():
        out_dt = np.dtype(bool) if stat in (_lib.STAT_LAND, _lib.STAT_LOR) else dt
        out = torch.empty(O * I * out_dt.itemsize, dtype=torch.uint8, device="cuda")
        be.reduce(stat, src, dtype_code(dt), O, R, I, out, dtype_code(out_dt))
        got = _host(out, out_dt, (O, I))
        if dt.kind == 'f' and uf in (np.multiply, np.add):
            truth = uf.reduce(x.astype(np.longdouble), axis=1)
            tol = 1e-6 if dt == np.float32 else 1e-10
            nan = np.isnan(truth)
            assert np.array_equal(np.isnan(got), nan), (stat, got, truth)
            assert np.all(np.abs(got[~nan] - truth[~nan]) <= tol * np.abs(truth[~nan])), (stat, got, truth)
        else:
            want = np.asarray(uf.reduce(x, axis=1, dtype=out_dt) if out_dt != np.bool_ or dt == np.bool_
                              else uf.reduce(x != 0, axis=1), out_dt)
            if dt.kind == 'f':
                assert np.array_equal(got, want, equal_nan=True), (stat, got, want)
            else:
                assert got.tobytes() == want.tobytes(), (stat, got, want)


def test_reduce_state_and_combine_match_single_pass():
    import torch
    from bolt_amd.mi355x import _lib
    from bolt_amd.mi355x._ops import dtype_code
    be = _be()
    rng = np.random.default_rng(5)
    x = (3 + rng.standard_normal((800, 300))).astype(np.float64)
    parts = [x[:100], x[100:450], x[450:]]
    for stat in (_lib.STAT_MEAN, _lib.STAT_VAR, _lib.STAT_STD, _lib.STAT_SUM):
        nb = be.state_bytes(stat, dtype_code(x.dtype), 300)
        states = torch.empty(nb * len(parts), dtype=torch.uint8, device="cuda")
        for i, p in enumerate(parts):
            st = torch.empty(nb, dtype=torch.uint8, device="cuda")
            be.reduce_state(stat, _dev(p), dtype_code(x.dtype), 1, p.shape[0], 300, st)
            states[i * nb:(i + 1) * nb].copy_(st)
        out = torch.empty(300 * 8, dtype=torch.uint8, device="cuda")
        be.reduce_combine(stat, dtype_code(x.dtype), states, [p.shape[0] for p in parts], 300, out,
                          dtype_code(x.dtype))
        got = _host(out, np.float64, (300,))
        ref = {_lib.STAT_MEAN: x.mean(0), _lib.STAT_VAR: x.var(0), _lib.STAT_STD: x.std(0),
               _lib.STAT_SUM: x.sum(0)}[stat]
        assert np.allclose(got, ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("O,R,I", [(70_000_000, 2, 1), (20_000_000, 2, 3)])
def test_reduce_beyond_one_launch(O, R, I):
    """Reductions whose grid exceeds HIP's 2^32-thread launch limit run as
    several launches (rows: 4 outputs per block, > 16.7M blocks; cols: one
    column tile per output row)."""
    import torch
    from bolt_amd.mi355x import _lib
    from bolt_amd.mi355x._ops import dtype_code
    be = _be()
    g = torch.Generator(device="cuda")
    g.manual_seed(O + I)
    x = torch.randint(0, 1000, (O, R, I), generator=g, device="cuda", dtype=torch.int32).float()
    src = x.view(torch.uint8).reshape(-1)
    out = torch.empty(O * I * 4, dtype=torch.uint8, device="cuda")
    be.reduce(_lib.STAT_MEAN, src, dtype_code(np.float32), O, R, I, out, dtype_code(np.float32))
    want = x.double().mean(dim=1).float().reshape(-1)
    assert torch.equal(out.view(torch.float32), want)  # small integers: exact in float64, one rounding
    del x, src, out, want
    torch.cuda.empty_cache()


def test_host_writable_and_zero_copy_statistics(monkeypatch):
    """Small statistics are stored by the kernel into page-locked host memory
    (bm_host_writable); the result equals the device-buffer + copy path."""
    import torch
    import bolt_amd as bolt
    from bolt_amd import MI355XContext
    from bolt_amd.mi355x import transfer
    from bolt_amd.mi355x._ops import backend_for
    dev = torch.device("cuda", 0)
    be = backend_for(dev)
    assert be.host_writable(torch.empty(4096, dtype=torch.uint8, pin_memory=True))
    assert not be.host_writable(torch.empty(4096, dtype=torch.uint8, device=dev))
    assert not be.host_writable(torch.empty(4096, dtype=torch.uint8))  # pageable
    ctx = MI355XContext(device="cuda:0")
    rng = np.random.default_rng(3)
    x = (1000 + 50 * rng.standard_normal((300, 64, 48))).astype(np.float32)
    u = rng.integers(0, 65536, size=(40, 33, 17)).astype(np.uint16)
    b, bu = bolt.array(x, ctx), bolt.array(u, ctx)
    s = b.swap((0,), (0, 1))
    cases = [(s, "mean", 2), (s, "std", 2), (b, "mean", 0), (b, "var", (0, 2)), (bu, "var", 0),
             (bu, "sum", 0), (bu, "max", (1, 2)), (b, "std", None)]
    got = {}
    for zc in (True, False):
        monkeypatch.setattr(transfer, "ZERO_COPY", zc)
        got[zc] = [getattr(a, name)(axis=ax) for a, name, ax in cases]
    for (a, name, ax), z, d in zip(cases, got[True], got[False]):
        z, d = np.asarray(z), np.asarray(d)
        assert z.shape == d.shape and z.dtype == d.dtype and z.tobytes() == d.tobytes(), (name, ax)


@pytest.mark.parametrize("shape,perm,dtype", [
    ((600, 4000), (1, 0), np.float32),      # ragged a- and b-tiles
    ((700, 2048), (1, 0), np.float64),
    ((3, 520, 1024), (0, 2, 1), np.float32),  # with a batch dim
])
def test_transpose_repeated_calls(shape, perm, dtype):
    """Repeated transposes of one source buffer (ragged a- and b-tiles, a batch
    dim) write the same bytes on every call."""
    import torch
    be = _be()
    x = _rand(shape, dtype, 11)
    src = _dev(x)
    want = np.ascontiguousarray(x.transpose(perm))
    for call in range(4):
        out = torch.zeros_like(src)
        be.permute(src, shape, perm, x.dtype.itemsize, out)
        torch.cuda.synchronize()
        assert _host(out, x.dtype, want.shape).tobytes() == want.tobytes(), call


def test_transpose_many_buffers():
    """Many source buffers of one shape, each transposed several times: every
    output is exact (no per-buffer state in the library)."""
    import torch
    be = _be()
    shape, perm = (300, 512), (1, 0)
    xs = [_rand(shape, np.float32, 100 + i) for i in range(70)]
    srcs = [_dev(x) for x in xs]
    for rep in range(3):
        for x, src in zip(xs, srcs):
            out = torch.empty_like(src)
            be.permute(src, shape, perm, 4, out)
            torch.cuda.synchronize()
            assert _host(out, np.float32, (512, 300)).tobytes() == np.ascontiguousarray(x.T).tobytes()
