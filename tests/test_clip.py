"""BoltArray.clip (bolt/spark/array.py:932-945: mapValues(v.clip(min, max)))
against numpy's record.clip, on the GPU and on the CPU test executor: every
unsigned width (torch has no max/min kernels for uint16/32/64),
float bounds on integer records (numpy promotes), per-record array bounds."""
import numpy as np
import pytest

import bolt_amd as bolt

DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int16, np.int64, np.float32, np.float64]


@pytest.mark.parametrize("dt", DTYPES, ids=lambda d: np.dtype(d).name)
def test_clip_matches_numpy(bctx, dt):
    rng = np.random.default_rng(0)
    if np.dtype(dt).kind in "ui":
        info = np.iinfo(dt)
        x = rng.integers(info.min, info.max, size=(6, 5, 3), dtype=dt, endpoint=True)
    else:
        x = rng.standard_normal((6, 5, 3)).astype(dt)
    b = bolt.array(x, bctx)
    bounds = [(None, 7), (3, None), (2, 100), (1.5, None), (None, 2.5),
              (np.array([1, 2, 3], dtype=dt), None)]
    if dt == np.uint64:
        bounds.append((np.uint64(2 ** 63 + 5), np.uint64(2 ** 64 - 9)))
    for lo, hi in bounds:
        got = b.clip(lo, hi)
        want = np.asarray([r.clip(lo, hi) for r in x])
        assert got.dtype == want.dtype, (lo, hi)
        a = got.toarray()
        assert a.dtype == want.dtype and a.tobytes() == want.tobytes(), (lo, hi)
