"""Seeded random indexing against the oracle (oracle/bolt_oracle.py getitem,
the restatement of BoltArraySpark.__getitem__, bolt/spark/array.py:480-676,
pinned by the reference's own getitem fixtures in tests/golden).

Random shapes (extents 1-7, so length-1 axes and all-key arrays occur), a
random split, and a random index: ints (negative too), slices with random
start / stop / step (negative steps, out-of-range bounds, empty selections
that the reference refuses), one list mixed with basic indices (on a key or a
value axis, unique entries in random order, negative entries), or lists on
every axis (advanced indexing, distinct key tuples).  The result must match the
oracle's: the same exception type, or the same shape, split and bytes (a
scalar: the same type and bytes).  Runs on the CPU test executor and (marker
`gpu`) on the HIP kernels (bm_gather_rows, strided copies).
"""
import os

import numpy as np
import pytest

import bolt_amd as bolt
from oracle import bolt_oracle as O

NCASES = 300
# a soak run takes other seeds: BOLT_AMD_FUZZ_SEEDS=start:stop (default 0:NCASES)
_SEEDS = range(*[int(v) for v in os.environ.get("BOLT_AMD_FUZZ_SEEDS", "0:%d" % NCASES).split(":")])


def _bound(rng, d):
    return None if rng.random() < 0.25 else int(rng.integers(-d - 2, d + 3))


def _basic(rng, d):
    if rng.random() < 0.35:
        return int(rng.integers(-d, d))
    step = [None, 1, 1, 2, 3, -1, -1, -2][int(rng.integers(0, 8))]
    return slice(_bound(rng, d), _bound(rng, d), step)


def _unique_list(rng, d):
    n = int(rng.integers(1, d + 1))
    vals = rng.permutation(d)[:n]
    return [int(v - d) if rng.random() < 0.3 else int(v) for v in vals]


def _index(rng, shape, split):
    nd = len(shape)
    n = int(rng.integers(1, nd + 1))
    kind = rng.random()
    if kind < 0.15:
        # advanced: lists on the first n axes, one entry per selected position,
        # distinct key tuples (the reference's repeated-key grouping is not kept)
        m = int(rng.integers(1, 5))
        cols = [rng.integers(0, shape[a], size=m) for a in range(n)]
        keys = list(zip(*[c.tolist() for c in cols[:min(n, split)]]))
        if len(set(keys)) != len(keys):
            return None
        return tuple(c.tolist() for c in cols)
    idx = [_basic(rng, shape[a]) for a in range(n)]
    if kind < 0.5:
        loc = int(rng.integers(0, n))
        idx[loc] = _unique_list(rng, shape[loc])
    return tuple(idx) if n > 1 or rng.random() < 0.5 else idx[0]


def _oracle(x, split, index):
    """(result, None) or (None, the exception type name the reference raises).
    An array the reference builds but cannot collect (its records fall short
    of the shape it declares) counts as ValueError: this backend refuses it."""
    try:
        want = O.getitem(O.parallelize(x, axis=tuple(range(split)), npartitions=3), index)
        if isinstance(want, O.RecSet):
            O.toarray(want)
        return want, None
    except Exception as e:  # the reference refuses this index
        return None, type(e).__name__


@pytest.mark.parametrize("seed", _SEEDS)
def test_getitem_fuzz(bctx, seed):
    rng = np.random.default_rng(9000 + seed)
    nd = int(rng.integers(2, 5))
    shape = tuple(int(rng.integers(1, 8)) for _ in range(nd))
    split = int(rng.integers(1, nd + 1))
    dtype = [np.float32, np.int16, np.float64, np.uint8][int(rng.integers(0, 4))]
    x = (np.arange(int(np.prod(shape))) * 7 % 251).astype(dtype).reshape(shape)
    index = _index(rng, shape, split)
    if index is None:
        pytest.skip("repeated key tuples (reference behaviour not kept)")
    want, raised = _oracle(x, split, index)
    b = bolt.array(x, bctx, axis=tuple(range(split)))
    if raised is not None:
        with pytest.raises(Exception) as e:
            r = b[index]
            if hasattr(r, "toarray"):
                r.toarray()
        assert type(e.value).__name__ == raised, (index, e.value)
        return
    got = b[index]
    if not isinstance(want, O.RecSet):
        assert type(got).__name__ == type(want).__name__, index
        assert np.asarray(got).tobytes() == np.asarray(want).tobytes(), index
        return
    assert got.shape == tuple(want.shape) and got.split == want.split, (index, got.shape, want.shape)
    out = O.toarray(want)
    arr = got.toarray()
    assert arr.dtype == out.dtype and arr.tobytes() == out.tobytes(), index
