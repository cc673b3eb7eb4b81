"""Seeded random cases of the rest of the array API against the oracle
(oracle/bolt_oracle.py, pinned by the reference's own fixtures): key and value
reshapes, squeeze, concatenate, sum / min / max and reduce with numpy ufuncs
over random axes, map over random key axes, filter (sorted and in record
order), stack -> map -> unstack.  Random shapes (all-key arrays too), random
splits, integer and float dtypes.  Extents are >= 2 except in the squeeze
case, as in tests/test_fuzz_oracle.py: the reference mishandles length-1
axes around its swaps in ways this backend does not reproduce
(docs/HISTORY.md §4, reference bugs not kept, item 6).  Data movement and
integer / min / max results must be bit-exact; float sums and products within
the bar of tests/golden_cases.reduce_close (float128 truth).  Runs on the CPU
test executor and (marker `gpu`) on the HIP kernels.
"""
import os

import numpy as np
import torch
import pytest

import bolt_amd as bolt
import golden_cases as G
from oracle import bolt_oracle as O

NCASES = 200
# a soak run takes other seeds: BOLT_AMD_FUZZ_SEEDS=start:stop (default 0:NCASES)
_SEEDS = range(*[int(v) for v in os.environ.get("BOLT_AMD_FUZZ_SEEDS", "0:%d" % NCASES).split(":")])
DTYPES = [np.float32, np.float64, np.int32, np.uint8, np.int16, np.uint16, np.uint32]


def _factor(rng, n, parts):
    """A random shape of ``parts`` extents whose product is n."""
    dims = [1] * parts
    k = n
    for p in range(2, n + 1):
        while k % p == 0:
            dims[int(rng.integers(0, parts))] *= p
            k //= p
    return tuple(dims)


def _same(got, want):
    a, b = np.asarray(got), np.asarray(want)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def _check_array(got, want):
    assert got.shape == tuple(want.shape) and got.split == want.split, (got.shape, want.shape, got.split, want.split)
    assert _same(got.toarray(), O.toarray(want))


def _check_swapped(got, want):
    """A result built through the reference's swap (map / filter align their
    axes with one): its shape and split (unit-axis squeezes included), dtype
    and bytes."""
    assert got.shape == tuple(want.shape) and got.split == want.split, (got.shape, want.shape, got.split, want.split)
    assert _same(got.toarray(), O.toarray(want))


def _mask_bug(e):
    """The reference's swap of an array with a length-1 axis can index with a
    boolean mask shorter than the array (numpy < 1.13 padded it; numpy >= 1.13
    raises): a reference failure this backend does not reproduce (DESIGN.md
    §4, reference bugs not kept)."""
    return isinstance(e, IndexError) and "boolean index did not match" in str(e)


def _raises_like(f, g, fallback=None):
    """Run oracle f and ours g: the same exception type, or both results.  If
    the oracle hits the reference's short-mask bug, ``fallback()`` (numpy's
    result of the intended operation) is the expectation, or the case is not
    compared (None, None)."""
    try:
        want = f()
    except Exception as e:
        if _mask_bug(e):
            return (fallback(), g()) if fallback is not None else (None, None)
        with pytest.raises(Exception) as got:
            g()
        assert type(got.value).__name__ == type(e).__name__, (e, got.value)
        return None, None
    return want, g()


def _np_reduce(uf, x, ax, keep):
    """numpy's reduction of ``uf`` over ``ax`` in the input dtype, shaped as bolt's result."""
    r = uf.reduce(x, axis=ax, keepdims=keep, dtype=None if uf is np.logical_or else x.dtype)
    return r[()] if np.ndim(r) == 0 else (r[0] if r.shape == (1,) else r)


@pytest.mark.parametrize("seed", _SEEDS)
def test_api_fuzz(bctx, seed):
    rng = np.random.default_rng(7000 + seed)
    nd = int(rng.integers(2, 5))
    shape = tuple(int(rng.integers(2, 6)) for _ in range(nd))
    split = int(rng.integers(1, nd + 1))
    dtype = DTYPES[int(rng.integers(0, len(DTYPES)))]
    if np.dtype(dtype).kind == "f":
        x = (3 + rng.standard_normal(shape)).astype(dtype)
    else:
        x = rng.integers(0, 50, size=shape).astype(dtype)
    axis = tuple(range(split))
    rs = O.parallelize(x, axis=axis, npartitions=int(rng.integers(1, 4)))
    b = bolt.array(x, bctx, axis=axis)

    # key / value reshapes (shapes.py:40-64, :111-134)
    ksh, vsh = shape[:split], shape[split:]
    newk = _factor(rng, int(np.prod(ksh)), int(rng.integers(1, 4)))
    want, got = _raises_like(lambda: O.keys_reshape(rs, newk), lambda: b.keys.reshape(newk))
    if want is not None:
        _check_array(got, want)
    if vsh:
        newv = _factor(rng, int(np.prod(vsh)), int(rng.integers(1, 4)))
        want, got = _raises_like(lambda: O.values_reshape(rs, newv), lambda: b.values.reshape(newv))
        if want is not None:
            _check_array(got, want)

    # squeeze of every / one unit axis (array.py:879-918), on a copy of the
    # array with unit axes inserted
    ushape = list(shape)
    for _ in range(int(rng.integers(1, 3))):
        ushape.insert(int(rng.integers(0, len(ushape) + 1)), 1)
    usplit = int(rng.integers(1, len(ushape) + 1))
    xu = x.reshape(ushape)
    rsu = O.parallelize(xu, axis=tuple(range(usplit)), npartitions=2)
    bu = bolt.array(xu, bctx, axis=tuple(range(usplit)))
    units = [i for i, d in enumerate(ushape) if d == 1]
    q = None if rng.random() < 0.4 else (units[int(rng.integers(0, len(units)))] if rng.random() < 0.7 else
                                         tuple(units))
    want, got = _raises_like(lambda: O.squeeze(rsu, q), lambda: bu.squeeze(q))
    if want is not None and len(want.shape):
        _check_array(got, want)

    # concatenate with an ndarray along a random axis (array.py:429-478)
    cat = int(rng.integers(0, nd))
    oshape = list(shape)
    oshape[cat] = int(rng.integers(1, 4))
    other = (np.arange(int(np.prod(oshape))) % 7).astype(dtype).reshape(oshape)
    want, got = _raises_like(lambda: O.concatenate(rs, other, axis=cat), lambda: b.concatenate(other, axis=cat))
    if want is not None:
        _check_array(got, want)

    # sum / min / max / reduce(ufunc) over random axes (array.py:243-427)
    na = int(rng.integers(1, nd + 1))
    ax = tuple(sorted(rng.choice(nd, na, replace=False).tolist()))
    keep = bool(rng.random() < 0.3)
    for name, f, g, uf in (("sum", O.sum_, b.sum, np.add), ("min", O.min_, b.min, np.minimum),
                           ("max", O.max_, b.max, np.maximum)):
        want, got = _raises_like(lambda: f(rs, ax, keep), lambda: g(axis=ax, keepdims=keep),
                                 lambda: _np_reduce(uf, x, ax, keep))
        if want is None:
            continue
        a = np.asarray(got.toarray() if hasattr(got, "toarray") else got)
        w = np.asarray(want)
        assert a.shape == w.shape and a.dtype == w.dtype, (name, a.shape, w.shape, a.dtype, w.dtype)
        if name != "sum" or a.dtype.kind in "iub":
            assert a.tobytes() == w.tobytes(), name
        else:
            assert G.reduce_close(a, w, x, "add", ax), name
    if np.dtype(dtype).kind in "iu":
        uf = [np.multiply, np.bitwise_xor, np.logical_or][int(rng.integers(0, 3))]
        want, got = _raises_like(lambda: O.reduce_(rs, uf, ax, keep), lambda: b.reduce(uf, axis=ax, keepdims=keep),
                                 lambda: _np_reduce(uf, x, ax, keep))
        if want is not None:
            a = np.asarray(got.toarray() if hasattr(got, "toarray") else got)
            assert _same(a, np.asarray(want)), uf

    # map over random key axes (array.py:125-191): an elementwise function
    nk = int(rng.integers(1, nd + 1))
    max_ax = tuple(sorted(rng.choice(nd, nk, replace=False).tolist()))
    fn = (lambda v: v * 2 + 1)
    want, got = _raises_like(lambda: O.map_(rs, fn, axis=max_ax), lambda: b.map(fn, axis=max_ax))
    if want is not None:
        _check_swapped(got, want)
    if np.dtype(dtype) in (np.dtype(np.uint16), np.dtype(np.uint32)):
        # records torch has no arithmetic for (functional.user_fn): a record sum
        # is numpy's uint64 and exact past 2**32, an explicit cast is kept
        big = x.astype(np.uint64) * 0 + (np.iinfo(dtype).max - int(rng.integers(0, 5)))
        bb, rb = bolt.array(big.astype(dtype), bctx, axis=axis), O.parallelize(big.astype(dtype), axis=axis)
        for f in (lambda v: v.sum(),
                  lambda v: v.to(torch.int64) if hasattr(v, "to") else v.astype(np.int64),
                  lambda v: (v.to(torch.int64) if hasattr(v, "to") else v.astype(np.int64)) * 3):
            want, got = _raises_like(lambda: O.map_(rb, f, axis=max_ax), lambda: bb.map(f, axis=max_ax))
            if want is not None:
                _check_swapped(got, want)

    # filter (array.py:193-241): keep records whose sum is above the median
    fax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
    thr = float(np.median(x))
    srt = bool(rng.random() < 0.5)

    def keep_rec(v):  # a numpy record (the oracle) or a device tensor (bolt_amd on a GPU)
        tot = v.double().sum() if hasattr(v, "double") else v.astype(np.float64).sum()
        return float(tot) > thr * max(1, v.reshape(-1).shape[0])
    want, got = _raises_like(lambda: O.filter_(rs, keep_rec, axis=fax, sort=srt),
                             lambda: b.filter(keep_rec, axis=fax, sort=srt))
    if want is not None:
        if want.shape == (0,):
            assert got.shape == (0,)
        else:
            _check_swapped(got, want)

    # stack -> map -> unstack (stack.py)
    size = int(rng.integers(1, 5))
    want = O.unstack(O.stack_map(O.stack(rs, size), lambda v: v + 1))
    got = b.stack(size).map(lambda v: v + 1).unstack()
    assert got.shape == tuple(want.shape) and got.split == want.split
    assert _same(got.toarray(), O.toarray(want).astype(got.dtype))
