"""Seeded random cases of the hot path against the oracle (oracle/bolt_oracle.py,
the record-level restatement of the reference's Spark path pinned to its
golden outputs): random ndim / shapes / split / dtype, then swap, transpose,
chunk (string and tuple sizes, padding) with its records, keys_to_values /
values_to_keys, unchunk and the statistics over random axes.

Runs on the CPU test executor and (marker `gpu`) on the HIP kernels, so odd
shapes reach every kernel family (tile / packed / fused transposes, runs,
rowcopy, record-map gathers with parts, row and column reductions).
Data movement must be bit-exact; statistics use the bar of
tests/test_golden_api.py (rtol 1e-6 float32 / 1e-12 float64, scaled).
"""
import os

import numpy as np
import pytest

import bolt_amd as bolt
from oracle import bolt_oracle as O

DTYPES = [np.float32, np.float64, np.uint8, np.int16, np.uint16, np.int32]
NCASES = 200
# a soak run takes other seeds: BOLT_AMD_FUZZ_SEEDS=start:stop (default 0:NCASES)
_SEEDS = range(*[int(v) for v in os.environ.get("BOLT_AMD_FUZZ_SEEDS", "0:%d" % NCASES).split(":")])


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    ndim = int(rng.integers(2, 6))
    # axes of length >= 2: the reference mishandles length-1 value axes around
    # swaps ("not kept" 6; test_swap_length1_value_axis)
    shape = tuple(int(rng.integers(2, 7 if ndim > 3 else 13)) for _ in range(ndim))
    split = int(rng.integers(1, ndim))
    dtype = DTYPES[int(rng.integers(0, len(DTYPES)))]
    if np.dtype(dtype).kind == "f":
        x = (10 + 3 * rng.standard_normal(shape)).astype(dtype)
    else:
        x = rng.integers(0, 200, size=shape).astype(dtype)
    return rng, x, split


def _exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def _records_equal(got, want):
    want = sorted(want, key=lambda kv: kv[0])
    assert len(got) == len(want)
    for (gk, gv), (wk, wv) in zip(got, want):
        assert gk == tuple(wk), (gk, wk)
        assert _exact(gv, np.ascontiguousarray(wv) if np.ndim(wv) else np.asarray(wv)), gk


@pytest.mark.parametrize("seed", _SEEDS)
def test_fuzz_against_oracle(bctx, seed):
    check_case(bctx, seed)


def check_case(bctx, seed):
    """One seeded case on context ``bctx`` (also run per rank by
    tests/test_dist_fuzz.py, where every collective path is exercised)."""
    rng, x, split = _case(seed)
    ndim = x.ndim
    axis = tuple(range(split))
    b = bolt.array(x, bctx, axis=axis)
    rs = O.parallelize(x, axis=axis, npartitions=2)
    assert _exact(b.toarray(), O.toarray(rs))

    # swap: random non-trivial key / value subsets
    nk = int(rng.integers(0, split + 1))
    nv = int(rng.integers(0, ndim - split + 1))
    kax = tuple(sorted(rng.choice(split, nk, replace=False).tolist()))
    vax = tuple(sorted(rng.choice(ndim - split, nv, replace=False).tolist()))
    if not (len(kax) == split and len(vax) == 0) and (kax or vax):
        s = b.swap(kax, vax)
        ws = O.swap(rs, kax, vax)
        assert s.shape == ws.shape and s.split == ws.split
        assert _exact(s.toarray(), O.toarray(ws))

    # transpose: a random permutation, split unchanged
    perm = tuple(rng.permutation(ndim).tolist())
    t = b.transpose(perm)
    wt = O.transpose(rs, perm)
    assert t.shape == wt.shape and t.split == wt.split
    assert _exact(t.toarray(), O.toarray(wt))

    # chunk: a tuple size (with padding when it fits) or a string size
    vshape = x.shape[split:]
    if rng.random() < 0.5:
        size = tuple(int(rng.integers(1, d + 1)) for d in vshape)
        pad = tuple(int(rng.integers(0, min(s, d - s) + 1)) for s, d in zip(size, vshape))
        # 0 < d % s < p is the reference's removepad over-trim (not kept 2)
        pad = tuple(0 if 0 < d % s < q else q for s, d, q in zip(size, vshape, pad))
        c, wc = b.chunk(size, padding=pad), O.chunk(rs, size, padding=pad)
    else:
        size = "%.3f" % (rng.random() * 0.2 + 0.01)
        c, wc = b.chunk(size), O.chunk(rs, size)
    assert np.array_equal(c.plan, wc.plan) and np.array_equal(c.padding, wc.padding)
    _records_equal(list(c.records()), wc.records())
    assert _exact(c.unchunk().toarray(), O.toarray(O.unchunk(wc)))
    # keys_to_values / values_to_keys on the chunked array
    if split > 1:
        k = int(rng.integers(0, split))
        kc, wkc = c.keys_to_values((k,)), O.keys_to_values(wc, (k,))
        assert kc.shape == wkc.shape and np.array_equal(kc.plan, wkc.plan)
        _records_equal(list(kc.records()), wkc.records())
    if ndim - split > 1:
        v = int(rng.integers(0, ndim - split))
        vc, wvc = c.values_to_keys((v,)), O.values_to_keys(wc, (v,))
        assert vc.shape == wvc.shape and np.array_equal(vc.plan, wvc.plan)
        _records_equal(list(vc.records()), wvc.records())

    # statistics over a random axis subset
    na = int(rng.integers(1, ndim + 1))
    ax = tuple(sorted(rng.choice(ndim, na, replace=False).tolist()))
    for name, oname in (("mean", "mean"), ("var", "variance"), ("std", "stdev")):
        got = getattr(b, name)(axis=ax)
        want = O.stat(rs, oname, axis=ax)
        got_a, want_a = np.asarray(got), np.asarray(want)
        assert got_a.shape == want_a.shape and got_a.dtype == want_a.dtype, name
        rtol = 1e-6 if got_a.dtype == np.float32 else 1e-12
        truth = getattr(x.astype(np.longdouble), name)(axis=ax)
        scale = float(np.abs(x.astype(np.float64)).max()) or 1.0
        err = np.abs(got_a.astype(np.longdouble) - truth)
        ref_err = np.abs(want_a.astype(np.longdouble) - truth)
        assert np.all(err <= rtol * scale + ref_err + np.finfo(got_a.dtype).eps * scale), name
    if np.dtype(x.dtype).kind in "iu":
        assert _exact(np.asarray(b.sum(axis=ax)), np.asarray(O.sum_(rs, axis=ax)))


def test_swap_length1_value_axis(bctx):
    """A swap whose result has exactly one value axis of length 1: the reference's
    unchunk squeezes it (chunk.py:193-197), so its (5, 3, 1) swap((), (0,)) is
    (5, 3) with split 2 and its (1, 5) swap((0,), (0,)) is (5,) -- bolt_amd
    returns the same shapes (plan.swap_shape); the bytes are numpy's transpose.
    A transpose through such shapes raises in the reference and is numpy's
    here (docs/HISTORY.md §4 item 6)."""
    x = np.arange(15, dtype=np.float32).reshape(5, 3, 1)
    b = bolt.array(x, bctx)
    s = b.swap((), (0,))
    ws = O.swap(O.parallelize(x), (), (0,))
    assert ws.shape == (5, 3) and ws.split == 2          # the reference (oracle pinned to it)
    assert s.shape == (5, 3) and s.split == 2
    assert _exact(s.toarray(), O.toarray(ws))
    y = np.arange(5.).reshape(1, 5)
    s = bolt.array(y, bctx).swap((0,), (0,))
    assert s.shape == (5,) and s.split == 1 and _exact(s.toarray(), y.reshape(5))
    assert _exact(bolt.array(np.zeros((3, 1)), bctx).T.toarray(), np.zeros((1, 3)))


def _raises(f):
    try:
        return f(), None
    except Exception as e:  # noqa: BLE001 -- the oracle's refusal, whatever its type
        return None, e


@pytest.mark.parametrize("seed", range(150))
def test_unit_axes_against_oracle(bctx, seed):
    """Arrays with length-1 axes through swap and the statistics: wherever the
    oracle (the reference's chain restated) answers, bolt_amd's shape, split and
    values are its; where it raises, bolt_amd is numpy's (not checked here)."""
    rng = np.random.default_rng(7000 + seed)
    ndim = int(rng.integers(2, 5))
    shape = tuple(int(rng.choice([1, 1, 2, 3, 4])) for _ in range(ndim))
    split = int(rng.integers(1, ndim + 1))
    x = (3 + rng.standard_normal(shape)).astype([np.float32, np.float64][seed % 2])
    axis = tuple(range(split))
    b = bolt.array(x, bctx, axis=axis)
    rs = O.parallelize(x, axis=axis, npartitions=2)
    for _ in range(3):
        kax = tuple(sorted(rng.choice(split, int(rng.integers(0, split + 1)), replace=False).tolist()))
        vax = tuple(sorted(rng.choice(ndim - split, int(rng.integers(0, ndim - split + 1)),
                                      replace=False).tolist()))
        if (len(kax) == split and not vax) or not (kax or vax):
            continue
        ws, err = _raises(lambda: O.swap(rs, kax, vax))
        if err is None:
            ws_arr, err = _raises(lambda: O.toarray(ws))
        if err is not None:
            continue
        s = b.swap(kax, vax)
        assert s.shape == ws.shape and s.split == ws.split, (kax, vax, s.shape, ws.shape)
        assert _exact(s.toarray(), ws_arr)
    for name, oname in (("mean", "mean"), ("var", "variance"), ("std", "stdev")):
        ax = tuple(sorted(rng.choice(ndim, int(rng.integers(1, ndim + 1)), replace=False).tolist()))
        keep = bool(rng.random() < 0.5)
        want, err = _raises(lambda: O.stat(rs, oname, axis=ax, keepdims=keep))
        if err is not None:
            continue
        got = getattr(b, name)(axis=ax, keepdims=keep)
        ga, wa = np.asarray(got), np.asarray(want)
        assert ga.shape == wa.shape and ga.dtype == wa.dtype, (name, ax, keep, ga.shape, wa.shape)
        tol = 1e-5 if ga.dtype == np.float32 else 1e-12
        assert np.allclose(ga, wa, rtol=tol, atol=tol, equal_nan=True), (name, ax)


def test_transpose_all_key_array(bctx):
    """An array whose every axis is a key (split = ndim): the reference's
    transpose raises ValueError (Values.transpose(()) takes max() of an empty
    sequence, bolt/utils.py:171); bolt_amd transposes the keys, as numpy
    would (docs/HISTORY.md §4, reference bugs not kept, item 7)."""
    x = np.arange(24, dtype=np.int16).reshape(2, 3, 4)
    b = bolt.array(x, bctx, axis=(0, 1, 2))
    for perm in ((2, 0, 1), (1, 0, 2), (2, 1, 0)):
        t = b.transpose(perm)
        assert t.split == 3 and _exact(t.toarray(), x.transpose(perm))
    assert _exact(b.T.toarray(), x.T)
