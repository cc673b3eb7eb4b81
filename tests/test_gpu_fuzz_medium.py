"""Seeded medium-size cases of the HIP kernels (up to 4M elements, every dtype
width): the sizes where tiles are partial, transposes fuse or pack sub-word
elements, rowcopies and runs transposes take over, record maps split into
parts and reductions split rows over blocks.  Data movement is compared
bit-exactly with numpy's transpose of the same array (the permutation the
reference's swap / transpose / keys_to_values / values_to_keys compute,
spark/array.py:716-833, chunk.py:202-347); the record-level oracle covers the
same operations at small sizes (tests/test_fuzz_oracle.py).  Statistics are
checked against a longdouble computation with the bar of test_fuzz_oracle.
"""
import os

import numpy as np
import pytest

import bolt_amd as bolt

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.uint16, np.float32, np.float64, np.int64, np.int16]


def _shape(rng):
    ndim = int(rng.integers(2, 6))
    cap = 1 << 22
    while True:
        shape = tuple(int(rng.choice([1, 2, 3, 5, 7, 16, 31, 64, 100, 129, 256, 1000, 2048])) for _ in range(ndim))
        n = int(np.prod(shape))
        if 1024 <= n <= cap:
            return shape


def _exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


# a soak run takes other seeds: BOLT_AMD_FUZZ_SEEDS=start:stop (default 0:240)
_SEEDS = range(*[int(v) for v in os.environ.get("BOLT_AMD_FUZZ_SEEDS", "0:240").split(":")])


@pytest.mark.parametrize("seed", _SEEDS)
def test_medium_fuzz(gpu_ctx, seed):
    gctx = gpu_ctx
    rng = np.random.default_rng(5000 + seed)
    shape = _shape(rng)
    ndim = len(shape)
    split = int(rng.integers(1, ndim))
    dtype = DTYPES[int(rng.integers(0, len(DTYPES)))]
    if np.dtype(dtype).kind == "f":
        x = (100 + 7 * rng.standard_normal(shape)).astype(dtype)
    else:
        x = rng.integers(0, 120, size=shape).astype(dtype)
    b = bolt.array(x, gctx, axis=tuple(range(split)))
    assert _exact(b.toarray(), x)

    perm = tuple(rng.permutation(ndim).tolist())
    assert _exact(b.transpose(perm).toarray(), x.transpose(perm)), perm

    nk = int(rng.integers(1, split + 1))
    nv = int(rng.integers(0, ndim - split + 1))
    kax = sorted(rng.choice(split, nk, replace=False).tolist())
    vax = sorted(rng.choice(ndim - split, nv, replace=False).tolist())
    if not (nk == split and nv == 0):
        P = ([k for k in range(split) if k not in kax] + [split + v for v in vax] + kax +
             [split + v for v in range(ndim - split) if v not in vax])
        s = b.swap(tuple(kax), tuple(vax))
        want = x.transpose(P)
        assert s.split == split - nk + nv
        assert _exact(s.toarray().reshape(want.shape), want), (kax, vax)

    vshape = shape[split:]
    size = tuple(int(rng.integers(1, d + 1)) for d in vshape)
    pad = tuple(int(rng.integers(0, min(s_, d - s_) + 1)) for s_, d in zip(size, vshape))
    c = b.chunk(size, padding=pad)
    xu = x.reshape(shape[:-1]) if vshape == (1,) else x  # the trailing (1,) squeeze again
    assert _exact(c.unchunk().toarray(), xu), (size, pad)
    k = int(rng.integers(0, split))
    order = [i for i in range(split) if i != k] + [k] + list(range(split, ndim))
    want = x.transpose(order)
    if vshape == (1,):
        want = want.reshape(want.shape[:-1])  # the all-keys singleton is squeezed (chunk.py:284-287)
        if want.shape[split - 1:] == (1,):
            # a moved key of extent 1 leaves the values (1,) again: unchunk
            # squeezes once more (chunk.py:193-197; the reference itself gives
            # (4, 1, 3, 2, 1) split 4 -> k2v((1,)) -> unchunk -> (4, 3, 2))
            want = want.reshape(want.shape[:-1])
    assert _exact(c.keys_to_values((k,)).unchunk().toarray(), want), k
    if ndim - split > 1:
        v = int(rng.integers(0, ndim - split))
        order = list(range(split)) + [split + v] + [split + i for i in range(ndim - split) if i != v]
        want = x.transpose(order)
        if want.shape[split + 1:] == (1,):
            want = want.reshape(want.shape[:-1])  # unchunk squeezes a trailing (1,) (chunk.py:193-197)
        assert _exact(c.values_to_keys((v,)).unchunk().toarray(), want), v

    na = int(rng.integers(1, ndim + 1))
    ax = tuple(sorted(rng.choice(ndim, na, replace=False).tolist()))
    for name in ("mean", "std"):
        got = np.asarray(getattr(b, name)(axis=ax))
        truth = getattr(x.astype(np.longdouble), name)(axis=ax)
        rtol = 1e-6 if got.dtype == np.float32 else 1e-12
        scale = float(np.abs(x.astype(np.float64)).max()) or 1.0
        err = np.abs(got.astype(np.longdouble) - truth)
        assert np.all(err <= rtol * scale + 4 * np.finfo(got.dtype).eps * scale), (name, ax)
    if np.dtype(dtype).kind in "iu":
        want = np.add.reduce(x, axis=ax, dtype=x.dtype)
        if want.shape == (1,):
            want = want.reshape(())  # shape-(1,) reductions come back as scalars (array.py:275-280)
        assert _exact(np.asarray(b.sum(axis=ax)), want)
