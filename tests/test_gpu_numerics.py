"""float64 var/std accuracy of the device reductions on ill-conditioned data.

The reference's StatCounter runs Welford per record (statcounter.py:51-59)
and merges partitions by Chan's formula (:85-96).  bm_reduce keeps a Welford
state per lane, built from batches of up to 32 values around a pivot drawn
from the batch and shifted by the row's first element, so neither an outlier
at the start of the reduced axis nor a large common offset costs digits.
These cases size the reduction so that each output is ONE chunk of >= 10,000
values (the case a single first-element pivot handles worst) and check every
output against the float128 truth at the north_star rtol of 1e-12, pure
relative (no absolute slack).  Parity pinned by the golden "numerics" stat
fixtures (tests/golden, make_golden.gen_stats_numerics) at small sizes.
"""
import numpy as np
import pytest

import bolt_amd as bolt

pytestmark = pytest.mark.gpu


def _truth_rows(x):
    v = x.astype(np.longdouble)
    return v.var(axis=-1)


def _check(got, truth, rtol):
    got = np.asarray(got, dtype=np.longdouble)
    err = np.abs(got - truth) / np.abs(truth)
    assert float(err.max()) <= rtol, float(err.max())


@pytest.mark.parametrize("kind", ["outlier", "offset", "outlier1e3"])
def test_rows_single_chunk(gpu_ctx, kind):
    # (8192, 10000): >= 8192 rows -> one chunk per row in the rows kernel
    rng = np.random.default_rng(7)
    x = rng.standard_normal((8192, 10000))
    if kind == "outlier":
        x[:, 0] = 100.0
    elif kind == "outlier1e3":
        x[:, 0] = 1e3
    else:
        x += 1e6
    b = bolt.array(x, gpu_ctx, axis=(0,))
    var = np.asarray(b.var(axis=1))
    std = np.asarray(b.std(axis=1))
    # every row (8192 outputs), truth in float128, in row blocks to bound host memory
    for lo in range(0, x.shape[0], 1024):
        t = _truth_rows(x[lo:lo + 1024])
        _check(var[lo:lo + 1024], t, 1e-12)
        _check(std[lo:lo + 1024], np.sqrt(t), 1e-12)


@pytest.mark.parametrize("kind", ["outlier", "offset"])
def test_cols_single_chunk(gpu_ctx, kind):
    # (2048, 10000, 2) reduced over axis 1: 2048 column tiles -> one chunk of
    # 10,000 rows, 256 row phases per tile merged in LDS
    rng = np.random.default_rng(8)
    x = rng.standard_normal((2048, 10000, 2))
    if kind == "outlier":
        x[:, 0, :] = 100.0
    else:
        x += 1e6
    b = bolt.array(x, gpu_ctx, axis=(0,))
    var = np.asarray(b.var(axis=1))
    # every column (2048 x 2 outputs) against the float128 truth
    for lo in range(0, x.shape[0], 256):
        t = x[lo:lo + 256].astype(np.longdouble).var(axis=1)
        _check(var[lo:lo + 256], t, 1e-12)


@pytest.mark.parametrize("kind", ["outlier", "offset"])
def test_key_axis_chunked(gpu_ctx, kind):
    # variance over the key axis with few outputs: R split into chunks whose
    # states are merged by the combine kernel around the shared pivot
    rng = np.random.default_rng(9)
    x = rng.standard_normal((200000, 8))
    if kind == "outlier":
        x[0, :] = 100.0
    else:
        x += 1e6
    b = bolt.array(x, gpu_ctx, axis=(0,))
    t = x.astype(np.longdouble).var(axis=0)
    _check(b.var(axis=0), t, 1e-12)
    _check(b.std(axis=0), np.sqrt(t), 1e-12)
    tall = x.astype(np.longdouble).var()
    _check(np.asarray(b.var()), tall, 1e-12)


def test_float32_offset(gpu_ctx):
    # float32 input, float64 accumulation, one rounding to float32
    rng = np.random.default_rng(10)
    x = (1e3 + rng.standard_normal((4096, 4000))).astype(np.float32)
    b = bolt.array(x, gpu_ctx, axis=(0,))
    v = np.asarray(b.var(axis=1))
    assert v.dtype == np.float32
    t = x.astype(np.longdouble).var(axis=1)
    err = np.abs(v.astype(np.longdouble) - t) / t
    assert float(err.max()) <= 1e-6


@pytest.mark.parametrize("dtype", [np.uint16, np.int16, np.uint8, np.int8, np.bool_])
@pytest.mark.parametrize("axis", [0, 1])
def test_small_int_var_is_exact(gpu_ctx, dtype, axis):
    """1- and 2-byte integer var / std come from exact integer sums: every
    output within 2 ulp of the exact rational variance (Python integers)."""
    rng = np.random.default_rng(11)
    shape = (3000, 257)
    if dtype == np.bool_:
        x = rng.integers(0, 2, size=shape).astype(bool)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.max - 40, info.max, size=shape, endpoint=True).astype(dtype)
        x[::7] = info.min  # extreme spread
    b = bolt.array(x, gpu_ctx, axis=(0,))
    v = np.asarray(b.var(axis=axis))
    xi = x.astype(np.int64)
    n = x.shape[axis]
    s1 = xi.sum(axis=axis)
    s2 = (xi * xi).sum(axis=axis)
    for k in range(v.size):  # every output
        num = int(n) * int(s2.reshape(-1)[k]) - int(s1.reshape(-1)[k]) ** 2
        exact = num / (n * n)   # Python int / int: correctly rounded
        assert abs(v.reshape(-1)[k] - exact) <= 2 * np.spacing(exact) + 1e-300, (k, v.reshape(-1)[k], exact)


def test_small_int_var_s2_beyond_64_bits(gpu_ctx):
    """the exact-integer var adds every chunk's S2 = sum x^2.  An
    8.6 GB uint16 array of 65535s (one 0) reduced over all axes has
    S2 = (n-1) 65535^2 ~ 2^64: the sum over chunks must not wrap (128-bit
    combine).  Exact value from Python integers: var = (n-1) 65535^2 / n^2."""
    import torch
    from fractions import Fraction
    shape = (4097, 1 << 20)
    n = shape[0] * shape[1]
    raw = torch.full((n,), -1, dtype=torch.int16, device="cuda")   # 0xFFFF = 65535
    raw[0] = 0
    b = bolt.ConstructMI355X.fromshards(raw.view(torch.uint8), shape, context=gpu_ctx, split=1, dtype=np.uint16)
    s1, s2 = (n - 1) * 65535, (n - 1) * 65535 ** 2
    assert s2 >= 2 ** 64
    exact = float(Fraction(n * s2 - s1 * s1, n * n))
    v = float(b.var())
    assert abs(v - exact) <= 2 * np.spacing(exact), (v, exact)
    sd = float(b.std())
    assert abs(sd - np.sqrt(exact)) <= 2 * np.spacing(np.sqrt(exact)), (sd, np.sqrt(exact))
    del b, raw
    torch.cuda.empty_cache()
