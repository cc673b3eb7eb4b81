"""The reference's hot-path tests, run against the 'mi355x' mode.

Each test runs twice: on the GPU (marker `gpu`: the HIP kernels) and on the
CPU test executor (tests/cpu_backend.py: the host logic -- plans, copy
descriptors, formatting -- with numpy standing in for the kernels).

Mirrors test/spark/test_spark_shaping.py:148-227 (swap, transpose, T,
swapaxes), test/spark/test_spark_chunking.py:6-112 (chunk contents, unchunk,
keys_to_values, values_to_keys, padding) and test/spark/
test_spark_functional.py:73-125 (mean/std/var/sum).  The expected values are
numpy's (the reference tests' own oracle); tests/test_gpu_golden.py checks
the same paths against outputs of the reference itself.
"""
from itertools import permutations

import numpy as np
import pytest

import bolt_amd as bolt
from bolt_amd.utils import allclose


def exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def test_construct(bctx):
    x = np.arange(2 * 3 * 4).reshape((2, 3, 4))
    for axis in [(0,), 0, (0, 1), (0, 1, 2)]:
        b = bolt.array(x, bctx, axis=axis)
        assert b.mode == 'mi355x'
        assert exact(b.toarray(), x)
    b = bolt.array(x, mode='mi355x')
    assert exact(b.toarray(), x)
    with pytest.raises(ValueError):
        bolt.array(x, bctx, axis=-1)
    with pytest.raises(ValueError):
        bolt.array(x, bctx, axis=(0, 1, 2, 3))
    # non-leading key axes: the reference keeps the old shape (construct.py:48-67)
    b = bolt.array(x, bctx, axis=(1,))
    assert exact(b.toarray(), x.transpose(1, 0, 2).reshape(x.shape))
    assert exact(bolt.ones((2, 3, 4), bctx).toarray(), np.ones((2, 3, 4)))
    assert exact(bolt.zeros(5, bctx, dtype=np.int16).toarray(), np.zeros(5, np.int16))


def test_swap(bctx):
    a = np.arange(2 ** 8).reshape(*(8 * [2]))
    b = bolt.array(a, bctx, axis=(0, 1, 2, 3))
    bs = b.swap((1, 2), (0, 3), size=(2, 2))
    assert exact(bs.toarray(), a.transpose((0, 3, 4, 7, 1, 2, 5, 6)))
    bs = b.swap((1, 2), (0, 3), size="50")
    assert exact(bs.toarray(), a.transpose((0, 3, 4, 7, 1, 2, 5, 6)))
    bs = b.swap((), (0, 1, 2, 3))
    assert exact(bs.toarray(), a)
    assert bs.split == 8
    bs = b.swap(0, 0)
    assert exact(bs.toarray(), a.transpose((1, 2, 3, 4, 0, 5, 6, 7)))
    bs = b.swap([], 0)
    assert exact(bs.toarray(), a) and bs.split == 5
    bs = b.swap(0, [])
    assert exact(bs.toarray(), a.transpose((1, 2, 3, 0, 4, 5, 6, 7))) and bs.split == 3
    b = bolt.array(a, bctx, axis=range(8))
    bs = b.swap([0, 1], [])
    assert exact(bs.toarray(), a.transpose((2, 3, 4, 5, 6, 7, 0, 1))) and bs.split == 6
    a = np.arange(2 * 3 * 4).reshape(2, 3, 4)
    b = bolt.array(a, bctx, axis=(0,))
    bs = b.swap((0,), (0, 1))
    assert exact(bs.toarray(), a.transpose(1, 2, 0))
    with pytest.raises(ValueError):
        b.swap((0,), ())


def test_transpose_all_perms(bctx):
    a = np.arange(2 * 3 * 4 * 5).reshape((2, 3, 4, 5))
    b = bolt.array(a, bctx, axis=(0, 1))
    for p in permutations(range(4), 4):
        t = b.transpose(p)
        assert exact(t.toarray(), a.transpose(p))
        assert t.split == 2
    assert exact(b.transpose().toarray(), a.transpose())
    assert exact(bolt.array(a, bctx, axis=0).T.toarray(), a.T)
    assert exact(b.T.toarray(), a.T)
    for i, j in [(1, 2), (0, 1), (2, 3)]:
        assert exact(b.swapaxes(i, j).toarray(), a.swapaxes(i, j))
    with pytest.raises(ValueError):
        b.transpose((0, 1, 1, 2))


def test_keys_values_transpose(bctx):
    x = np.arange(2 * 3 * 4).reshape((2, 3, 4))
    b = bolt.array(x, bctx, axis=(0, 1))
    c = b.keys.transpose((1, 0))
    assert c.keys.shape == (3, 2)
    assert exact(c.toarray(), x.transpose((1, 0, 2)))
    b = bolt.array(x, bctx, axis=0)
    c = b.values.transpose((1, 0))
    assert c.values.shape == (4, 3)
    assert exact(c.toarray(), x.transpose((0, 2, 1)))
    with pytest.raises(ValueError):
        b.values.transpose((0, 2))
    b = bolt.array(x, bctx, axis=(0, 1))
    assert exact(b.keys.reshape((6,)).toarray(), x.reshape(6, 4))
    assert b.keys.reshape((6,)).split == 1


def test_chunk_records(bctx):
    x = np.arange(4 * 6).reshape(1, 4, 6)
    b = bolt.array(x, bctx)
    k1, v1 = zip(*b.chunk((2, 3))._rdd.sortByKey().collect())
    assert k1 == ((0, 0, 0), (0, 0, 1), (0, 1, 0), (0, 1, 1))
    v2 = [s for m in np.split(x[0], (2,), axis=0) for s in np.split(m, (3,), axis=1)]
    assert all(exact(m1, m2) for m1, m2 in zip(v1, v2))
    k1, v1 = zip(*b.chunk((3, 4))._rdd.sortByKey().collect())
    v2 = [s for m in np.split(x[0], (3,), axis=0) for s in np.split(m, (4,), axis=1)]
    assert all(exact(m1, m2) for m1, m2 in zip(v1, v2))


def test_unchunk(bctx):
    x = np.arange(4 * 6).reshape(1, 4, 6)
    b = bolt.array(x, bctx)
    for s in [(2, 3), (3, 4), (4, 6), '0.1', '150']:
        assert exact(b.chunk(s).unchunk().toarray(), x)
    x = np.arange(4 * 5 * 10).reshape(1, 4, 5, 10)
    b = bolt.array(x, bctx)
    for s in [(4, 5, 10), (1, 1, 1), (3, 3, 3)]:
        assert exact(b.chunk(s).unchunk().toarray(), x)
    x = np.arange(4 * 6).reshape(4, 6)
    assert exact(bolt.array(x, bctx, (0, 1)).chunk(()).unchunk().toarray(), x)
    assert exact(bolt.array(x, bctx, (0,)).chunk((2)).unchunk().toarray(), x)


def test_keys_to_values(bctx):
    x = np.arange(4 * 7 * 9 * 6).reshape(4, 7, 9, 6)
    b = bolt.array(x, bctx, (0, 1))
    c = b.chunk((4, 2))
    assert exact(x, c.keys_to_values((0,)).unchunk().toarray().transpose(1, 0, 2, 3))
    assert exact(x, c.keys_to_values((1,)).unchunk().toarray())
    assert exact(x, c.keys_to_values((1,), size=(3,)).unchunk().toarray())
    assert exact(x, c.keys_to_values((0, 1)).unchunk().toarray())
    assert exact(x, c.keys_to_values((0, 1), size=(2, 3)).unchunk().toarray())
    assert exact(x, c.keys_to_values(()).unchunk().toarray())
    b = bolt.array(x, bctx, range(4))
    c = b.chunk(())
    assert exact(x, c.keys_to_values((3,)).unchunk().toarray())
    assert exact(x, c.keys_to_values((0, 1)).unchunk().toarray().transpose(2, 3, 0, 1))
    b = bolt.array(x, bctx, (0,))
    c = b.chunk((2, 3, 4))
    assert exact(x, c.keys_to_values((0,)).unchunk().toarray())


def test_values_to_keys(bctx):
    x = np.arange(4 * 7 * 9 * 6).reshape(4, 7, 9, 6)
    b = bolt.array(x, bctx, (0, 1))
    c = b.chunk((4, 2))
    assert exact(x, c.values_to_keys((0,)).unchunk().toarray())
    assert exact(x, c.values_to_keys((1,)).unchunk().toarray().transpose(0, 1, 3, 2))
    assert exact(x, c.values_to_keys((0, 1)).unchunk().toarray())
    assert exact(x, c.values_to_keys(()).unchunk().toarray())
    b = bolt.array(x, bctx, (0,))
    c = b.chunk((2, 3, 4))
    assert exact(x, c.values_to_keys((0,)).unchunk().toarray())
    assert exact(x, c.values_to_keys((0, 1)).unchunk().toarray())


def test_padding(bctx):
    x = np.arange(2 * 2 * 5 * 6).reshape(2, 2, 5, 6)
    b = bolt.array(x, bctx, (0, 1))
    c = b.chunk((2, 2), padding=1)
    chunks = c.tordd().sortByKey().values().collect()
    assert exact(chunks[0], np.array([[0, 1, 2], [6, 7, 8], [12, 13, 14]]))
    assert exact(chunks[1], np.array([[1, 2, 3, 4], [7, 8, 9, 10], [13, 14, 15, 16]]))
    assert exact(chunks[4], np.array([[7, 8, 9, 10], [13, 14, 15, 16], [19, 20, 21, 22], [25, 26, 27, 28]]))
    assert exact(chunks[6], np.array([[18, 19, 20], [24, 25, 26]]))
    c = b.chunk((3, 3), padding=(1, 2))
    chunks = c.tordd().sortByKey().values().collect()
    assert exact(chunks[0], np.array([[0, 1, 2, 3, 4], [6, 7, 8, 9, 10], [12, 13, 14, 15, 16], [18, 19, 20, 21, 22]]))
    c = b.chunk((2, 2), padding=1)
    assert exact(x, c.unchunk().toarray())
    assert exact(x, c.keys_to_values((1,)).unchunk().toarray())
    assert exact(x, c.values_to_keys((0,)).unchunk().toarray())
    with pytest.raises(ValueError):
        b.chunk((2, 2), padding=(3, 1))
    with pytest.raises(ValueError):
        b.chunk((4, 4), padding=(2, 2))


def test_chunk_properties(bctx):
    x = np.arange(4 * 6).reshape(1, 4, 6)
    b = bolt.array(x, bctx)
    assert b.chunk(size=(2, 3)).uniform is True
    assert b.chunk(size=(2, 4)).uniform is False
    with pytest.raises(ValueError):
        b.chunk(size=(5, 6))


@pytest.mark.parametrize("name", ["mean", "std", "var", "sum"])
def test_stats(bctx, name):
    x = np.arange(2 * 3 * 4).reshape(2, 3, 4)
    b = bolt.array(x, bctx, axis=(0,))
    f = getattr(b, name)
    g = getattr(x, name)
    assert allclose(f(), g())
    assert allclose(f(axis=0), g(axis=0))
    assert allclose(f(axis=(0, 1)), g(axis=(0, 1)))
    assert f(axis=(0, 1, 2)) == g(axis=(0, 1, 2))
    for axis in [1, 2, (1, 2), (0, 2)]:
        assert allclose(f(axis=axis), g(axis=axis))
    assert f(axis=1, keepdims=True).shape == (2, 1, 4)


def test_stats_dtypes(bctx):
    rng = np.random.default_rng(0)
    x = (1000 + 50 * rng.standard_normal((200, 16, 8))).astype(np.float32)
    b = bolt.array(x, bctx)
    m = b.mean(axis=0)
    assert m.dtype == np.float32 and m.shape == (16, 8)
    assert np.allclose(m, x.astype(np.float64).mean(0), rtol=1e-6)
    s = b.std(axis=0)
    assert np.allclose(s, x.astype(np.float64).std(0), rtol=1e-6)
    u = rng.integers(0, 65536, size=(50, 8, 8)).astype(np.uint16)
    bu = bolt.array(u, bctx)
    v = bu.var(axis=0)
    assert v.dtype == np.float64
    assert np.allclose(v, u.astype(np.float64).var(0), rtol=1e-12)
    sm = bu.sum(axis=0)
    assert sm.dtype == np.uint16
    assert exact(np.asarray(sm), np.add.reduce(u, axis=0, dtype=np.uint16))


def test_empty_reductions(bctx):
    """Reductions over zero records follow the reference's StatCounter / treeReduce
    (statcounter.py:28-130, array.py:243-334): an empty StatCounter gives mean
    0.0 and variance / stdev nan; reduce() of no records raises ValueError.
    Axes with records but empty values give empty results of the kept shape."""
    import math
    b = bolt.array(np.zeros((0, 3, 4), np.float32), bctx)
    assert b.mean(axis=0) == 0.0
    assert math.isnan(b.var(axis=0)) and math.isnan(b.std(axis=0))
    with pytest.raises(ValueError):
        b.sum(axis=0)
    with pytest.raises(ValueError):
        b.max(axis=0)
    assert b.mean(axis=1).shape == (0, 4) and b.sum(axis=(1,)).shape == (0, 4)
    c = bolt.array(np.zeros((3, 0, 4), np.float32), bctx)
    assert c.mean(axis=0).shape == (0, 4) and c.std(axis=0).shape == (0, 4)
    assert c.swap((0,), (0,)).shape == (0, 3, 4)
    assert exact(c.T.toarray(), np.zeros((4, 0, 3), np.float32))


def test_display(bctx, capsys):
    """display() prints rdd.take(10): the first 10 (key, value) records in key
    order (spark/array.py:1022-1027)."""
    x = np.arange(4 * 5 * 3).reshape((4, 5, 3)).astype(np.float32)
    b = bolt.array(x, bctx, axis=(0, 1))
    b.display()
    want = []
    for i, key in enumerate(np.ndindex(4, 5)):
        if i == 10:
            break
        want.append(str((key, x[key])))
    assert capsys.readouterr().out.splitlines() == "\n".join(want).splitlines()
    small = bolt.array(x[:1, :3], bctx, axis=(0, 1))
    small.display()
    assert len(capsys.readouterr().out.strip().splitlines()) == 3


def test_permute_of_unit_axes_shares_bytes(bctx):
    """A permutation that moves only extent-1 axes is a relabelling: same
    bytes, new shape (swap / transpose results as the reference's)."""
    x = np.arange(1 * 4 * 1 * 5, dtype=np.float32).reshape(1, 4, 1, 5)
    b = bolt.array(x, bctx, axis=(0, 1))
    t = b.transpose(2, 1, 0, 3)
    assert t._data.data_ptr() == b._data.data_ptr()
    assert exact(t.toarray(), x.transpose(2, 1, 0, 3))
    s = b.swap((0,), (0,))
    assert exact(s.toarray(), x.transpose(1, 2, 0, 3)) and s.split == 2
    moved = b.transpose(0, 3, 2, 1)
    assert moved._data.data_ptr() != b._data.data_ptr()
    assert exact(moved.toarray(), x.transpose(0, 3, 2, 1))
