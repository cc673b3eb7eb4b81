"""Seeded random chains of chunked-array operations against the oracle
(oracle/bolt_oracle.py, pinned by the reference's fixtures): chunk on a
random subset of the value axes (tuple sizes with padding, or string sizes),
then one to three of keys_to_values (random key subsets, with or without new
chunk sizes) / values_to_keys (random value subsets) / an elementwise map,
checking the plan, padding, shape, split and every record after each step,
then unchunk.  Random shapes (extents >= 2, as tests/test_fuzz_oracle.py:
the reference mishandles length-1 axes around its swaps), splits and dtypes.
Runs on the CPU test executor and (marker `gpu`) on the HIP kernels (record
maps, scatters, runs, strided copies).
"""
import os

import numpy as np
import pytest

import bolt_amd as bolt
from oracle import bolt_oracle as O

NCASES = 200
# a soak run takes other seeds: BOLT_AMD_FUZZ_SEEDS=start:stop (default 0:NCASES)
_SEEDS = range(*[int(v) for v in os.environ.get("BOLT_AMD_FUZZ_SEEDS", "0:%d" % NCASES).split(":")])
DTYPES = [np.float32, np.float64, np.uint8, np.int16, np.int64]


def _exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def _same_chunks(c, w, what):
    assert c.shape == w.shape and c.split == w.split, (what, c.shape, w.shape, c.split, w.split)
    assert np.array_equal(c.plan, w.plan) and np.array_equal(c.padding, w.padding), (what, c.plan, w.plan)
    got = list(c.records())
    want = sorted(w.records(), key=lambda kv: kv[0])
    assert [k for k, _ in got] == [tuple(k) for k, _ in want], what
    for (k, gv), (_, wv) in zip(got, want):
        assert _exact(gv, np.ascontiguousarray(wv)), (what, k)


def _chunk_args(rng, vshape):
    nv = len(vshape)
    if rng.random() < 0.25:
        return "%.3f" % (rng.random() * 0.3 + 0.005), None, None
    axes = tuple(sorted(rng.choice(nv, int(rng.integers(1, nv + 1)), replace=False).tolist()))
    size = tuple(int(rng.integers(1, vshape[a] + 1)) for a in axes)
    pad = None
    if rng.random() < 0.6:
        # 0 < d % s < p is the reference's removepad over-trim (docs/HISTORY.md §4 item 2)
        pad = tuple(0 if 0 < vshape[a] % s < q else q for a, s, q in
                    ((a, s, int(rng.integers(0, min(s, vshape[a] - s) + 1))) for a, s in zip(axes, size)))
    return size, axes, pad


@pytest.mark.parametrize("seed", _SEEDS)
def test_chunk_fuzz(bctx, seed):
    rng = np.random.default_rng(11000 + seed)
    nd = int(rng.integers(2, 6))
    shape = tuple(int(rng.integers(2, 7 if nd > 3 else 11)) for _ in range(nd))
    split = int(rng.integers(1, nd))
    dtype = DTYPES[int(rng.integers(0, len(DTYPES)))]
    x = (np.arange(int(np.prod(shape))) * 13 % 241).astype(dtype).reshape(shape)
    axis = tuple(range(split))
    b = bolt.array(x, bctx, axis=axis)
    rs = O.parallelize(x, axis=axis, npartitions=int(rng.integers(1, 4)))

    size, caxes, pad = _chunk_args(rng, shape[split:])
    c = b.chunk(size, axis=caxes, padding=pad)
    w = O.chunk(rs, size, axis=caxes, padding=pad)
    _same_chunks(c, w, ("chunk", size, caxes, pad))

    for step in range(int(rng.integers(1, 4))):
        r = rng.random()
        if r < 0.4 and c.split > 1:
            n = int(rng.integers(1, c.split))
            ax = tuple(sorted(rng.choice(c.split, n, replace=False).tolist()))
            sz = None
            if rng.random() < 0.5:
                sz = tuple(int(rng.integers(1, c.kshape[a] + 1)) for a in ax)
            c, w = c.keys_to_values(ax, size=sz), O.keys_to_values(w, ax, size=sz)
            what = ("k2v", ax, sz)
        elif r < 0.8 and len(c.vshape) > 1:
            n = int(rng.integers(1, len(c.vshape)))
            ax = tuple(sorted(rng.choice(len(c.vshape), n, replace=False).tolist()))
            c, w = c.values_to_keys(ax), O.values_to_keys(w, ax)
            what = ("v2k", ax)
        else:
            c = c.map(lambda v: v * 3 + 1)
            w = O.chunk_map(w, lambda v: v * 3 + 1)
            what = ("map",)
        _same_chunks(c, w, what)

    u = c.unchunk()
    wu = O.unchunk(w)
    assert u.shape == wu.shape and u.split == wu.split
    got = u.toarray()
    want = O.toarray(wu)
    assert got.tobytes() == want.astype(got.dtype).tobytes()
