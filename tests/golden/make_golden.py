"""Generate the golden fixtures from the REFERENCE bolt (Spark mode).

Run in the build container only (it imports /root/reference, which is not on
the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's Spark path runs over fakespark/ (an in-process RDD, see
fakerdd.py) with two shims for behaviour the reference relied on from old
numpy:
  * ChunkedArray.removepad indexes with tuple(slices) (chunk.py:550 passes a
    list, which numpy >= 1.23 rejects);
  * _getbasic / _getmixed index a value with tuple(slices) (array.py:508,
    :584 pass lists);
  * after keys_to_values squeezes the all-keys singleton value axis
    (chunk.py:284-287) the padding and the stale trailing chunk id are
    trimmed, as numpy < 1.13's short boolean masks did.
Writes tests/golden/golden.json (case specs + scalar results) and
tests/golden/golden.npz (output arrays).  Inputs are regenerated from specs
(tests/golden/inputs.py).
"""
import collections
import collections.abc
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("BOLT_REFERENCE", "/root/reference")
sys.path[:0] = [REF, os.path.join(HERE, "fakespark"), HERE]
collections.Iterable = collections.abc.Iterable  # bolt/utils.py:3 on Python >= 3.10

import numpy as np  # noqa: E402

import bolt  # noqa: E402
from bolt.spark.array import BoltArraySpark  # noqa: E402
from bolt.spark.chunk import ChunkedArray  # noqa: E402
from fakerdd import FakeContext  # noqa: E402
from inputs import make_input  # noqa: E402


# ---------------------------------------------------------------- shims
def _removepad(idx, value, number, padding, axes=None):
    if axes is None:
        axes = range(len(number))
    mask = len(number) * [False, ]
    for i in range(len(mask)):
        if i in axes and padding[i] != 0:
            mask[i] = True
    starts = [0 if (i == 0 or not m) else p for (i, m, p) in zip(idx, mask, padding)]
    stops = [None if (i == n - 1 or not m) else -p for (i, m, p, n) in zip(idx, mask, padding, number)]
    slices = [slice(i1, i2) for (i1, i2) in zip(starts, stops)]
    return value[tuple(slices)]


ChunkedArray.removepad = staticmethod(_removepad)
_k2v = ChunkedArray.keys_to_values


def _keys_to_values(self, axes, size=None):
    res = _k2v(self, axes, size)
    if res is not self and len(res._padding) > len(res._plan):
        res._padding = res._padding[:len(res._plan)]
        res._rdd = res._rdd.map(lambda kv: (kv[0][:-1], kv[1]))
    return res


ChunkedArray.keys_to_values = _keys_to_values


# BoltArraySpark._getbasic / _getmixed index a record's value with a LIST of
# slices (array.py:508, :584), which numpy < 1.23 read as a tuple; numpy 2
# raises IndexError.  Same logic, the value index passed as a tuple.
def _getbasic(self, index):
    ksl, vsl = index[:self.split], index[self.split:]

    def keep(key):
        for k, s in zip(key, ksl):
            inside = (s.start <= k < s.stop) if s.step > 0 else (s.stop < k <= s.start)
            if not (inside and np.mod(k - s.start, s.step) == 0):
                return False
        return True

    def rekey(key):
        return tuple([(k - s.start) / s.step for k, s in zip(key, ksl)])

    picked = self._rdd.filter(lambda kv: keep(kv[0]))
    if self._split == self.ndim:
        rdd = picked.map(lambda kv: (rekey(kv[0]), kv[1]))
    else:
        vt = tuple(s if s.stop != -1 else slice(s.start, None, s.step) for s in vsl)
        rdd = picked.map(lambda kv: (rekey(kv[0]), kv[1][vt]))
    shape = tuple([int(np.ceil((s.stop - s.start) / float(s.step))) for s in index])
    return rdd, shape, self.split


def _getmixed(self, index):
    loc = np.where([isinstance(i, (tuple, list, np.ndarray)) for i in index])[0][0]
    idx = list(index[loc])
    if isinstance(idx[0], (tuple, list, np.ndarray)):
        raise ValueError("When mixing basic and advanced indexing, "
                         "advanced index must be one-dimensional")
    if loc < self.split:
        def rekey(key):
            key = list(key)
            key[loc] = idx.index(key[loc])
            return tuple(key)
        rdd = self._rdd.filter(lambda kv: kv[0][loc] in idx).map(lambda kv: (rekey(kv[0]), kv[1]))
    else:
        vt = [slice(0, None, None) for _ in self.values.shape]
        vt[loc - self.split] = idx
        vt = tuple(vt)
        rdd = self._rdd.map(lambda kv: (kv[0], kv[1][vt]))
    newshape = list(self.shape)
    newshape[loc] = len(idx)
    b = self._constructor(rdd, shape=tuple(newshape)).__finalize__(self)
    rest = index[:]
    rest[loc] = slice(0, None, None)
    b = b[tuple(rest)]
    return b._rdd, b.shape, b.split


BoltArraySpark._getbasic = _getbasic
BoltArraySpark._getmixed = _getmixed


# ---------------------------------------------------------------- cases
CASES = []
ARRAYS = {}


def add(case, **arrays):
    i = len(CASES)
    case["id"] = i
    for k, v in arrays.items():
        ARRAYS["c%d_%s" % (i, k)] = np.asarray(v)
    case["arrays"] = sorted(arrays)
    CASES.append(case)


def spec(shape, dtype="int64", kind="arange", seed=0, **kw):
    d = {"shape": list(shape), "dtype": str(np.dtype(dtype)), "kind": kind, "seed": seed}
    d.update(kw)
    return d


def run(fn, case):
    try:
        return fn()
    except Exception as e:  # record the exception type as the golden result
        case["raises"] = type(e).__name__
        return None


def gen_construct():
    for sh, axis, npart in [((2, 3, 4), (0,), None), ((2, 3, 4), (0, 1), 5), ((2, 3, 4), (0, 1, 2), None),
                            ((2, 3, 4), (1,), None), ((2, 3, 4), (2, 0), None), ((4, 5, 6), (1, 2), 3),
                            ((2, 3, 4), (-1,), None), ((2, 3, 4), (0, 1, 2, 3), None)]:
        s = spec(sh)
        x = make_input(s)
        case = {"op": "construct", "input": s, "axis": list(axis), "npartitions": npart}
        b = run(lambda: bolt.array(x, sc, axis=axis, npartitions=npart), case)
        if b is None:
            add(case)
            continue
        case.update(shape=list(b.shape), split=b.split)
        add(case, out=b.toarray())


def gen_swap():
    items = [
        (spec([2] * 8), (0, 1, 2, 3), (1, 2), (0, 3), (2, 2)),
        (spec([2] * 8), (0, 1, 2, 3), (1, 2), (0, 3), "50"),
        (spec([2] * 8), (0, 1, 2, 3), (1, 2), (0, 3), "150"),
        (spec([2] * 8), (0, 1, 2, 3), (), (0, 1, 2, 3), "150"),
        (spec([2] * 8), (0, 1, 2, 3), (0,), (0,), "150"),
        (spec([2] * 8), (0, 1, 2, 3), (), (0,), "150"),
        (spec([2] * 8), (0, 1, 2, 3), (0,), (), "150"),
        (spec([2] * 8), tuple(range(8)), (0, 1), (), "150"),
        (spec((2, 3, 4)), (0,), (0,), (0, 1), "150"),
        (spec((2, 3, 4)), (0,), (0,), (), "150"),
        (spec((2, 3, 4)), (0,), (), (), "150"),
        (spec((50, 32, 32), "float64", "normal", 0), (0,), (0,), (0,), "150"),         # C1 scaled
        (spec((20, 16, 16), "float32", "imaging", 1), (0,), (0,), (0, 1), "150"),     # C2 scaled
        (spec((16, 8, 8, 4), "float32", "bits", 2), (0, 1), (0,), (0,), "150"),       # C3 scaled
        (spec((16, 8, 8, 4), "float32", "bits", 2), (0, 1), (0,), (0,), "150000"),
        (spec((16, 8, 8, 4), "float32", "bits", 2), (0, 1), (1,), (0,), "150"),
        (spec((30, 40, 24), "uint16", "ints", 3), (0,), (0,), (0,), "0.5"),           # C4 scaled
        (spec((4, 4, 4, 6, 6), "float64", "normal", 4), (0, 1, 2), (0, 2), (1,), "0.1"),  # C5 scaled
        (spec((4, 4, 4, 6, 6), "float64", "normal", 4), (0, 1, 2), (1,), (0, 1), (2, 3)),
        (spec((3, 5, 7), "bool", "bool", 5), (0,), (0,), (1,), "150"),
        (spec((6, 10), "int8", "ints", 6), (0,), (0,), (0,), (4,)),
        (spec((2, 3, 4)), (0, 1), (0, 1), (), "150"),    # all keys, no values: error
        (spec((2, 3, 4)), (0,), (0,), (0,), (5, 5)),     # plan > vshape: error
    ]
    for s, axis, kax, vax, size in items:
        x = make_input(s)
        b = bolt.array(x, sc, axis=axis)
        case = {"op": "swap", "input": s, "axis": list(axis), "kaxes": list(kax), "vaxes": list(vax),
                "size": size if isinstance(size, str) else list(size)}
        r = run(lambda: b.swap(kax, vax, size=size), case)
        if r is None:
            add(case)
            continue
        case.update(shape=list(r.shape), split=r.split)
        out, srt = r.toarray(), _sorted_array(r)
        if out.tobytes() != srt.tobytes():
            # records are right but toarray() collects them unsorted: the
            # result of values_to_keys inherits ordered=True from
            # keys_to_values (chunk.py:236, :302-303) although _extract emits
            # records chunk by chunk, and toarray only sorts when unordered
            # (array.py:1012)
            case["toarray_unsorted"] = True
            add(case, out=out, out_sorted=srt)
        else:
            add(case, out=out)


def _sorted_array(r):
    recs = sorted(r._rdd.collect(), key=lambda kv: tuple(int(k) for k in kv[0]))
    return np.asarray([v for _, v in recs]).reshape(r.shape)


def gen_transpose():
    from itertools import permutations
    s = spec((2, 3, 4, 5))
    x = make_input(s)
    for axis in [(0, 1), (0,), (0, 1, 2)]:
        b = bolt.array(x, sc, axis=axis)
        for p in permutations(range(4)):
            case = {"op": "transpose", "input": s, "axis": list(axis), "perm": list(p)}
            r = b.transpose(p)
            case.update(shape=list(r.shape), split=r.split)
            out, srt = r.toarray(), _sorted_array(r)
            if out.tobytes() != srt.tobytes():
                case["toarray_unsorted"] = True
                add(case, out=out, out_sorted=srt)
            else:
                add(case, out=out)
    for s2, axis in [(spec((4, 4, 4, 6, 6), "float64", "normal", 4), (0, 1, 2)),
                     (spec((16, 8, 8, 4), "float32", "bits", 2), (0, 1))]:
        x2 = make_input(s2)
        b = bolt.array(x2, sc, axis=axis)
        for name, f in [("T", lambda b: b.T), ("perm20413", lambda b: b.transpose(2, 0, 4, 1, 3) if b.ndim == 5 else b.transpose(3, 1, 0, 2)),
                        ("swapaxes", lambda b: b.swapaxes(0, b.ndim - 1))]:
            case = {"op": "transpose_named", "input": s2, "axis": list(axis), "name": name}
            r = f(b)
            case.update(shape=list(r.shape), split=r.split)
            out, srt = r.toarray(), _sorted_array(r)
            if out.tobytes() != srt.tobytes():
                case["toarray_unsorted"] = True
                add(case, out=out, out_sorted=srt)
            else:
                add(case, out=out)
    b = bolt.array(x, sc, axis=(0, 1))
    for bad in [(0, 1, 1, 2), (0, 1, 2), (0, 1, 2, 4)]:
        case = {"op": "transpose", "input": s, "axis": [0, 1], "perm": list(bad)}
        run(lambda: b.transpose(bad), case)
        add(case)


def _records(chunked):
    recs = chunked.tordd().sortByKey().collect()
    keys = [[int(k) for k in kk] for kk, _ in recs]
    shapes = [list(v.shape) for _, v in recs]
    flat = np.concatenate([np.asarray(v).reshape(-1) for _, v in recs]) if recs else np.zeros(0)
    return keys, shapes, flat


def gen_chunk():
    items = [
        (spec((1, 4, 6)), (0,), (2, 3), None, None),
        (spec((1, 4, 6)), (0,), (3, 4), None, None),
        (spec((1, 4, 6)), (0,), (4, 6), None, None),
        (spec((1, 4, 6)), (0,), "0.1", None, None),
        (spec((1, 4, 6)), (0,), "150", None, None),
        (spec((1, 4, 5, 10)), (0,), (3, 3, 3), None, None),
        (spec((1, 4, 5, 10)), (0,), (1, 1, 1), None, None),
        (spec((4, 6)), (0, 1), (), None, None),
        (spec((4, 6)), (0,), 2, None, None),
        (spec((2, 2, 5, 6)), (0, 1), (2, 2), None, 1),
        (spec((2, 2, 5, 6)), (0, 1), (3, 3), None, (1, 2)),
        (spec((2, 2, 5, 6)), (0, 1), (2, 2), None, (3, 1)),   # error
        (spec((2, 2, 5, 6)), (0, 1), (4, 4), None, (2, 2)),   # error
        (spec((1, 4, 6)), (0,), (5, 6), None, None),          # error
        (spec((3, 12, 12), "float64", "normal", 7), (0,), (4, 4), None, 2),    # C5-like padded
        (spec((3, 10, 9), "float64", "normal", 7), (0,), (4, 4), None, (1, 2)),
        (spec((3, 10, 9), "uint16", "ints", 8), (0,), (3,), (1,), None),       # axis subset (tuple size)
        (spec((5, 20, 30), "uint16", "ints", 9), (0,), "0.5", None, None),     # C4-like ragged plan
        (spec((2, 3, 64, 64), "float64", "normal", 10), (0, 1), (16, 16), None, 2),
    ]
    for s, axis, size, caxis, pad in items:
        x = make_input(s)
        b = bolt.array(x, sc, axis=axis)
        case = {"op": "chunk", "input": s, "axis": list(axis),
                "size": size if isinstance(size, str) else (list(size) if isinstance(size, tuple) else size),
                "chunk_axis": caxis if caxis is None else list(caxis),
                "padding": pad if not isinstance(pad, tuple) else list(pad)}
        c = run(lambda: b.chunk(size, axis=caxis, padding=pad), case)
        if c is None:
            add(case)
            continue
        keys, shapes, flat = _records(c)
        case.update(keys=keys, shapes=shapes, plan=[int(p) for p in c.plan],
                    padding_out=[int(p) for p in c.padding], uniform=bool(c.uniform),
                    chunk_shape=list(c.shape), split=c.split)
        u = c.unchunk()
        case.update(unchunk_shape=list(u.shape), unchunk_split=u.split)
        sub = {}
        arr = run(lambda: u.toarray(), sub)
        if arr is None:
            # the reference's removepad trims a full p from a clipped chunk
            # when 0 < d % s < p (chunk.py:546-547 vs getslices' clipping)
            case["unchunk_raises"] = sub["raises"]
            add(case, flat=flat)
            continue
        add(case, flat=flat, unchunk=arr)


def gen_moves():
    """keys_to_values / values_to_keys chains (test_spark_chunking.py:51-112 and more)."""
    items = [
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("k2v", (0,), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("k2v", (1,), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("k2v", (1,), (3,))]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("k2v", (0, 1), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("k2v", (0, 1), (2, 3))]),
        (spec((4, 7, 9, 6)), (0, 1, 2, 3), (), None, [("k2v", (3,), None)]),
        (spec((4, 7, 9, 6)), (0, 1, 2, 3), (), None, [("k2v", (0, 1), None)]),
        (spec((4, 7, 9, 6)), (0,), (2, 3, 4), None, [("k2v", (0,), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("v2k", (0,), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("v2k", (1,), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("v2k", (0, 1), None)]),
        (spec((4, 7, 9, 6)), (0, 1), (4, 2), None, [("v2k", (), None)]),
        (spec((4, 7, 9, 6)), (0,), (2, 3, 4), None, [("v2k", (0,), None)]),
        (spec((4, 7, 9, 6)), (0,), (2, 3, 4), None, [("v2k", (0, 1), None)]),
        (spec((2, 2, 5, 6)), (0, 1), (2, 2), 1, [("k2v", (1,), None)]),
        (spec((2, 2, 5, 6)), (0, 1), (2, 2), 1, [("v2k", (0,), None)]),
        (spec((3, 4, 9, 10), "float64", "normal", 11), (0, 1), (4, 4), (1, 2), [("k2v", (0,), None), ("v2k", (1,), None)]),
        (spec((3, 4, 9, 10), "float64", "normal", 11), (0, 1), (4, 4), 2, [("v2k", (0, 1), None), ("k2v", (1, 2), (2, 3))]),
        # a moved key of extent 1 when the values are (1,): keys_to_values
        # squeezes the old (1,) and the values are (1,) again, so unchunk
        # squeezes once more (chunk.py:284-287, :193-197)
        (spec((4, 1, 3, 2, 1)), (0, 1, 2, 3), (1,), None, [("k2v", (1,), None)]),
        (spec((4, 1, 3, 1)), (0, 1, 2), (1,), None, [("k2v", (1,), None)]),
        (spec((4, 1, 3, 2)), (0, 1, 2), (2,), None, [("k2v", (1,), None)]),
    ]
    for s, axis, size, pad, steps in items:
        x = make_input(s)
        b = bolt.array(x, sc, axis=axis)
        c = b.chunk(size, padding=pad)
        case = {"op": "moves", "input": s, "axis": list(axis),
                "size": list(size) if isinstance(size, tuple) else size,
                "padding": list(pad) if isinstance(pad, tuple) else pad,
                "steps": [[n, list(a), (list(z) if z is not None else None)] for n, a, z in steps]}
        def apply(c):
            for n, a, z in steps:
                c = c.keys_to_values(a, size=z) if n == "k2v" else c.values_to_keys(a)
            return c, _records(c)
        res = run(lambda: apply(c), case)
        if res is None:
            add(case)
            continue
        c, (keys, shapes, flat) = res
        case.update(keys=keys, shapes=shapes, plan=[int(p) for p in c.plan],
                    padding_out=[int(p) for p in c.padding], chunk_shape=[int(q) for q in c.shape],
                    split=c.split)
        u = c.unchunk()
        case.update(unchunk_shape=list(u.shape), unchunk_split=u.split)
        add(case, flat=flat, unchunk=u.toarray())


def gen_getplan():
    cfg = [((512, 512), "float32", "150"), ((256, 256, 32), "float32", "150"), ((256, 32), "float32", "150"),
           ((256, 32), "float32", "150000"), ((1024, 1024), "uint16", "150"), ((64, 64), "float64", "150"),
           ((64, 64), "float64", "150000"), ((5, 6), "int64", "0.1"), ((5, 6), "int64", "0.001"),
           ((7, 9, 11), "float64", "1"), ((3, 4, 5), "uint8", "0.02")]
    for vs, dt, size in cfg:
        x = np.zeros((1,) + vs, dtype=dt)
        b = bolt.array(x, sc)
        c = b.chunk(size)
        add({"op": "getplan", "vshape": list(vs), "dtype": dt, "size": size,
             "plan": [int(p) for p in c.plan], "padding_out": [int(p) for p in c.padding]})


def gen_stats():
    inputs = [
        (spec((2, 3, 4)), (0,)),
        (spec((2, 3, 4), "float64", "normal", 12), (0,)),
        (spec((2, 3, 4), "float64", "normal", 12), (0, 1)),
        (spec((6, 5, 7), "float32", "imaging", 13), (0,)),
        (spec((6, 5, 7), "float32", "normal", 13), (0, 1)),
        (spec((9, 4, 3), "uint16", "ints", 14), (0,)),
        (spec((9, 4, 3), "int32", "ints", 15, small=1), (0,)),
        (spec((5, 4), "bool", "bool", 16), (0,)),
        (spec((100, 64, 64), "float64", "normal", 0), (0,)),   # C1
    ]
    axes_list = [None, 0, 1, 2, (0, 1), (0, 2), (1, 2), (0, 1, 2)]
    for s, kaxis in inputs:
        x = make_input(s)
        for npart in ((8,) if s["shape"] == [100, 64, 64] else (1, 2, 8)):
            b = bolt.array(x, sc, axis=kaxis, npartitions=npart)
            for name in ("mean", "var", "std", "sum", "min", "max"):
                for ax in axes_list:
                    if ax is not None and max(np.atleast_1d(ax)) >= x.ndim:
                        continue
                    for keep in (False, True):
                        if keep and ax not in (None, 1, (0, 2)):
                            continue
                        if npart != 2 and s["shape"] != [100, 64, 64] and (ax not in (None, 0, (0, 1))):
                            continue
                        case = {"op": "stat", "input": s, "axis": list(kaxis), "npartitions": npart,
                                "name": name, "reduce_axis": ax if not isinstance(ax, tuple) else list(ax),
                                "keepdims": keep}
                        r = run(lambda: getattr(b, name)(axis=ax, keepdims=keep), case)
                        if r is None and "raises" in case:
                            add(case)
                            continue
                        case["result_type"] = type(r).__name__
                        case["result_dtype"] = str(np.asarray(r).dtype)
                        add(case, out=np.asarray(r))


def gen_stat_errors():
    s = spec((2, 3, 4))
    x = make_input(s)
    b = bolt.array(x, sc, axis=(0,))
    for ax in [3, (0, 3), -1]:
        case = {"op": "stat", "input": s, "axis": [0], "npartitions": None, "name": "mean",
                "reduce_axis": ax if not isinstance(ax, tuple) else list(ax), "keepdims": False}
        run(lambda: b.mean(axis=ax), case)
        add(case)


def enc_item(i):
    if isinstance(i, slice):
        return {"slice": [i.start, i.stop, i.step]}
    if isinstance(i, np.ndarray):
        return {"array": i.tolist()}
    return i  # int or (nested) list


def gen_getitem():
    S = slice
    x66 = spec((6, 6))
    basic = [(S(0, 1), S(0, 1)), (S(0, 2), S(0, 2)), (S(0, 2), S(0, 3)), (S(0, 2), S(0, 3, 2)),
             (S(None, 2), S(None, 2)), (S(1, None), S(1, None)), (S(5, 1, -1), S(5, 1, -1)),
             (S(10, -10, -2), S(10, -10, -2)), (S(-5, -1), S(-5, -1)), (S(-1, -5, -2), S(-1, -5, -2)),
             (S(None, None, -1), S(None, None, -1)), (S(None, None, -2), 3), (-1, S(None, None, -3)),
             (S(2, 3),), S(1, 4), 2]
    items = [(x66, ax, idx) for ax in ((0,), (0, 1)) for idx in basic]
    x1010 = spec((10, 10, 3))
    items += [(x1010, (0, 1), idx) for idx in [(S(0, 5, 2), S(0, 2)), (S(0, 5, 3), S(0, 2)), (S(0, 9, 3), S(0, 2)),
                                               (S(9, None, -4), S(None, None, -2), S(2, 0, -1))]]
    x23 = spec((2, 3))
    ints = [(0, 0), (0, 1), (0, S(0, 1)), (1, 2), 0, [0], ([1], [2]), ([1], 2), (-1, -2), (1,), [-1],
            ([1, 0], [0, 2]), ([0, 1, 1], [2, 0, 1])]
    items += [(x23, ax, idx) for ax in ((0,), (0, 1)) for idx in ints]
    x334 = spec((3, 3, 4))
    lists = [([0, 1], [0, 1], [0, 2]), ([0, 1], [0, 2], [0, 3]), ([0, 1, 2], [0, 2, 1], [0, 3, 1]),
             ([[0, 0], [1, 1]], [[0, 2], [0, 2]], [[0, 3], [0, 3]]),
             ([2, 0, 1], [0, 1, 2], [1, 1, 1]), ([0, 0, 1], [2, 1, 0], [0, 1, 2]), ([0, 1, 0], [2, 1, 0], [0, 1, 2]),
             ([-1, 0], [1, -3], [-4, 3]), (np.array([1, 2]), np.array([0, 0]), np.array([3, 2])),
             ([0, 1], [0, 1]), ([0, 3], [0, 1], [0, 1]), ([0, 1], [0, 1, 2], [0, 1])]
    items += [(x334, ax, idx) for ax in ((0,), (0, 1), (0, 1, 2)) for idx in lists]
    x4 = spec((4, 4, 4, 4), "float32", "normal", 21)
    i, s2 = [0, 1], S(1, 3)
    mixed = [(i, S(None), S(None), S(None)), (i, s2, s2, s2), (S(None), S(None), i, S(None)), (s2, s2, i, s2),
             ([1], S(None), S(None), S(None)), (S(None), S(None), [1], S(None)),
             ([[0, 1], [1, 0]], S(None), S(None), S(None)), ([2, 0], S(None), S(None), S(None)),
             (S(None), [3, 1, 1], S(None), S(None)), (S(None), S(None), [3, 1, 1], S(None)),
             (S(None), S(None), S(None), [2, 0, 3]), ([0, 1], S(None, None, -1)), ([3, 1], 2, S(None), 1),
             (1, [2, 0], S(0, 4, 2)), (S(None), S(None), [-1, 0], -1)]
    items += [(x4, ax, idx) for ax in ((0,), (0, 1), (0, 1, 2)) for idx in mixed]
    x5 = spec((5,))
    items += [(x5, (0,), idx) for idx in [5, -6, [1, 5], S(3, 2), S(5, None), S(-6, 0), S(0, 5, -1),
                                          (0, 0), 4, -5, [4, 0, 0], S(None, None, -1)]]
    xb = spec((7, 5, 6), "uint16", "ints", 22)
    for ax, npart in [((0,), 3), ((0, 1), 4), ((1,), 2)]:
        for idx in [(S(6, 0, -2), S(None, None, -1), S(1, 5, 3)), (S(1, 6, 2), 4), (3, S(None), [5, 0, 2]),
                    ([6, 2, 3], S(4, None, -2)), ([0, 6], [4, 1], [5, 0]), (-2,), (S(None), S(None), 0)]:
            items.append((xb, ax, idx, npart))
    for it in items:
        s, ax, idx = it[:3]
        npart = it[3] if len(it) > 3 else None
        x = make_input(s)
        b = bolt.array(x, sc, axis=ax, npartitions=npart)
        enc = {"tuple": [enc_item(j) for j in idx]} if isinstance(idx, tuple) else {"item": enc_item(idx)}
        case = {"op": "getitem", "input": s, "axis": list(ax), "npartitions": npart, "index": enc}
        r = run(lambda: b[idx], case)
        if r is None and "raises" in case:
            add(case)
            continue
        if isinstance(r, BoltArraySpark):
            arr = run(lambda: r.toarray(), case)
            if arr is None:
                case["collect_raises"] = case.pop("raises")
                case.update(shape=list(r.shape), split=r.split)
                add(case)
                continue
            case.update(kind="array", shape=list(r.shape), split=r.split)
            srt = _sorted_array(r)
            if srt.tobytes() != arr.tobytes():  # toarray skips the sort
                case["toarray_unsorted"] = True
                add(case, out=arr, out_sorted=srt)
            else:
                add(case, out=arr)
        else:
            case.update(kind="scalar", result_type=type(r).__name__)
            add(case, out=np.asarray(r))
    for shp, ax, sq in [((1, 2, 1, 4), (0,), [None, (0, 2), 0, 2]), ((1, 2, 1, 4), (0, 1), [None, (0, 2), 0, 2]),
                        ((1, 1, 1, 1), (0, 1), [None, (1, 3)]), ((3, 1, 2), (0, 1), [1, None, 0, (1,)]),
                        ((2, 1, 1), (0, 1, 2), [None, 2])]:
        s = spec(shp, "float64", "normal", 23)
        x = make_input(s)
        b = bolt.array(x, sc, axis=ax)
        for q in sq:
            case = {"op": "squeeze", "input": s, "axis": list(ax), "npartitions": None,
                    "squeeze": list(q) if isinstance(q, tuple) else q}
            r = run(lambda: b.squeeze(q), case)
            if r is None and "raises" in case:
                add(case)
                continue
            case.update(shape=list(r.shape), split=r.split)
            add(case, out=r.toarray())


def gen_concatenate():
    items = [((2, 3), (0,), (2, 3), (0,), 0), ((2, 3), (0,), (5, 3), (0,), 0), ((2, 3), (0,), (2, 4), (0,), 1),
             ((4, 3, 5), (0, 1), (2, 3, 5), (0, 1), 0), ((4, 3, 5), (0, 1), (4, 6, 5), (0, 1), 1),
             ((4, 3, 5), (0, 1), (4, 3, 2), (0, 1), 2), ((4, 3, 5), (0,), (4, 1, 5), (0,), 1),
             ((4, 3, 5), (0,), (4, 3, 7), (0,), 2), ((3, 2, 2, 3), (0, 1, 2), (3, 2, 1, 3), (0, 1, 2), 2),
             ((4, 3, 5), (0,), (4, 3, 6), (0,), 1), ((4, 3, 5), (0,), (4, 3, 5), (0, 1), 0),
             ((7, 3), (0,), (9, 3), (0,), 0)]
    for n, (sa, aa, sb, ab, axis) in enumerate(items):
        specA = spec(sa, "float32", "normal", 30 + n)
        specB = spec(sb, "float32", "normal", 60 + n)
        x, y = make_input(specA), make_input(specB)
        for kind in ("ndarray", "local", "spark"):
            if kind != "spark" and ab != aa[:1] and ab != aa:
                continue
            for npart in (None, 3):
                b = bolt.array(x, sc, axis=aa, npartitions=npart)
                other = {"ndarray": lambda: y, "local": lambda: bolt.array(y),
                         "spark": lambda: bolt.array(y, sc, axis=ab, npartitions=npart)}[kind]()
                case = {"op": "concatenate", "input": specA, "axis": list(aa), "npartitions": npart,
                        "other": specB, "other_axis": list(ab), "other_kind": kind, "cat_axis": axis}
                r = run(lambda: b.concatenate(other, axis=axis), case)
                if r is None:
                    add(case)
                    continue
                case.update(shape=list(r.shape), split=r.split)
                add(case, out=r.toarray())
    x = make_input(spec((2, 3)))
    case = {"op": "concatenate", "input": spec((2, 3)), "axis": [0], "npartitions": None, "other": None,
            "other_axis": [0], "other_kind": "list", "cat_axis": 0}
    run(lambda: bolt.array(x, sc).concatenate([[1, 2, 3]]), case)
    add(case)


def gen_chunk_map():
    from funcs import FUNCS
    items = [
        (spec((4, 8, 8)), (0,), (4, 8), None, ["double", "crop_last", "dup_last", "flip_last", "shrink0",
                                                 "first_row", "to_f64"]),
        (spec((3, 10, 7), "float32", "normal", 40), (0,), (4, 7), (1, 0), ["affine", "square", "center0",
                                                                          "dup_last", "to_f64"]),
        (spec((2, 3, 6, 9, 5), "float64", "normal", 41), (0, 1), (3, 9, 5), (1, 0, 0), ["double", "norm_rows",
                                                                                         "crop_last"]),
        (spec((5, 12, 10), "float32", "normal", 42), (0,), (5, 4), (2, 1), ["affine", "flip_last"]),
        (spec((4, 6), "int32", "ints", 43, small=1), (0,), (6,), None, ["double", "crop_last", "dup_last"]),
    ]
    for s, ax, size, pad, names in items:
        x = make_input(s)
        b = bolt.array(x, sc, axis=ax)
        c = b.chunk(size=size, padding=pad)
        for name in names:
            for vs in (None, "given"):
                value_shape = None
                if vs == "given":
                    try:
                        value_shape = FUNCS[name](np.zeros(tuple(c.plan), dtype=x.dtype)).shape
                    except Exception:
                        continue
                case = {"op": "chunk_map", "input": s, "axis": list(ax), "npartitions": None,
                        "size": list(size), "padding": list(pad) if pad else None, "func": name,
                        "value_shape": list(value_shape) if value_shape is not None else None}
                r = run(lambda: c.map(FUNCS[name], value_shape=value_shape), case)
                if r is None:
                    add(case)
                    continue
                u = run(lambda: r.unchunk().toarray(), case)
                if u is None:
                    case["unchunk_raises"] = case.pop("raises")
                    add(case)
                    continue
                case.update(shape=list(r.shape), plan=[int(p) for p in r.plan], dtype=str(u.dtype))
                add(case, out=u)
    for s, size in [(spec((2, 8, 8)), (8, 5)), (spec((3, 4, 6)), (2, 3))]:
        x = make_input(s)
        c = bolt.array(x, sc).chunk(size=size)
        d = c.map_generic(lambda v: [int(v.sum()), v.shape]).toarray()
        flat = [list(o) for o in d.reshape(-1)]
        add({"op": "chunk_map_generic", "input": s, "axis": [0], "npartitions": None, "size": list(size),
             "shape": list(d.shape), "objects": [[o[0], list(o[1])] for o in flat]})


def gen_functional():
    from funcs import FUNCS
    x10 = spec((10, 10))
    x3 = spec((10, 10, 10), "float32", "normal", 50)
    o2 = spec((100, 2), "float64", "normal", 51)
    # stack / unstack
    for s, ax, npart in [(x10, (0,), 2), (x10, (0,), 3), (x3, (0,), 2), (x3, (0, 1), 4), (o2, (0,), 2),
                         (o2, (0,), 1)]:
        x = make_input(s)
        b = bolt.array(x, sc, axis=ax, npartitions=npart)
        for size in (None, 0, 2, 3, -1, 7):
            st = b.stack(size)
            recs = st._rdd.collect()
            add({"op": "stack", "input": s, "axis": list(ax), "npartitions": npart, "size": size,
                 "stack_shapes": [list(v.shape) for _, v in recs], "stack_keys": [[[int(q) for q in k] for k in ks]
                                                                                for ks, _ in recs],
                 "shape": list(st.shape), "split": st.split}, out=st.unstack().toarray())
    # stacked map
    chains = [["double"], ["sum1"], ["tile12"], ["ones22"], ["sum0"], ["arr1"], ["arr0"], ["double", "double"],
              ["double", "ones22"], ["ones22", "double"], ["scalar2"], ["none"], ["zerodiv"], ["sum0", "double"],
              ["square", "sum1"]]
    for s, ax, npart, size in [(o2, (0,), 2, 5), (x3, (0,), 2, None), (x3, (0, 1), 3, 4), (x10, (0,), 1, 3)]:
        x = make_input(s)
        b = bolt.array(x, sc, axis=ax, npartitions=npart)
        for chain in chains:
            case = {"op": "stack_map", "input": s, "axis": list(ax), "npartitions": npart, "size": size,
                    "funcs": chain}

            def go():
                st = b.stack(size)
                for name in chain:
                    st = st.map(FUNCS[name])
                return st.unstack()
            r = run(go, case)
            if r is None:
                add(case)
                continue
            arr = r.toarray()
            case.update(shape=list(r.shape), split=r.split, dtype=str(arr.dtype))
            add(case, out=arr)
    # BoltArraySpark.map / filter
    y = spec((4, 5, 6), "float32", "normal", 52)
    for s in (y, spec((4, 5, 6), "int64", "ints", 53, small=1)):
        x = make_input(s)
        for kax in ((0,), (0, 1)):
            b = bolt.array(x, sc, axis=kax, npartitions=2)
            for name, axis, vs, dt in [("double", (0,), None, None), ("sum0", (0,), None, None),
                                       ("sum0", (0, 1), None, None), ("sum1", (2,), None, None),
                                       ("double", (1, 2), None, None), ("to_f64", (0,), None, None),
                                       ("double", (0,), "given", "given"), ("crop_last", (0, 2), None, None),
                                       ("keyed", (0,), None, None), ("keyed", (1, 2), None, None)]:
                with_keys = name == "keyed"
                value_shape = dtype = None
                if vs == "given":
                    value_shape = tuple(x.shape[i] for i in range(x.ndim) if i not in axis)
                    dtype = x.dtype
                case = {"op": "map", "input": s, "axis": list(kax), "npartitions": 2, "func": name,
                        "map_axis": list(axis), "value_shape": list(value_shape) if value_shape else None,
                        "dtype": str(dtype) if dtype is not None else None, "with_keys": with_keys}
                r = run(lambda: b.map(FUNCS[name], axis=axis, value_shape=value_shape, dtype=dtype,
                                      with_keys=with_keys), case)
                if r is None:
                    add(case)
                    continue
                arr = r.toarray()
                case.update(shape=list(r.shape), split=r.split, out_dtype=str(arr.dtype))
                add(case, out=arr)
            for name, axis, srt in [("gt_mean", (0,), False), ("gt_mean", (0, 1), True), ("gt_big", (2,), False),
                                    ("never", (0,), False), ("gt_mean", (1, 2), False), ("gt_mean", (0, 1), False)]:
                case = {"op": "filter", "input": s, "axis": list(kax), "npartitions": 2, "func": name,
                        "filter_axis": list(axis), "sort": srt}
                r = run(lambda: b.filter(FUNCS[name], axis=axis, sort=srt), case)
                if r is None:
                    add(case)
                    continue
                if r.shape == (0,):
                    case.update(shape=[0], split=r.split)
                    add(case)
                    continue
                case.update(shape=list(r.shape), split=r.split)
                add(case, out=r.toarray())


def gen_stats_numerics():
    """float64 statistics where a pivot-shifted sum loses digits: an outlier at
    index 0 of the reduced axis, and data offset far from zero (1e6 + N(0,1)),
    reduced over a value axis (device rows kernel) and over the key axis
    (device column kernel); float32 at a 1e3 offset.  n = 10,000."""
    inputs = [
        (spec((4, 10000), "float64", "normal", 70, outlier=[1, 100.0]), (0,), 1),
        (spec((10000, 4), "float64", "normal", 71, outlier=[0, 100.0]), (0,), 0),
        (spec((4, 10000), "float64", "normal", 72, shift=1e6), (0,), 1),
        (spec((10000, 4), "float64", "normal", 73, shift=1e6), (0,), 0),
        (spec((4, 10000), "float32", "normal", 74, shift=1e3), (0,), 1),
        (spec((10000, 4), "float32", "normal", 75, outlier=[0, 100.0]), (0,), 0),
        (spec((20, 500, 3), "float64", "normal", 76, shift=1e6), (0, 1), (0, 1)),
    ]
    for s, kaxis, red in inputs:
        x = make_input(s)
        for npart in (2, 8):
            b = bolt.array(x, sc, axis=kaxis, npartitions=npart)
            for name in ("mean", "var", "std"):
                for ax in (red, None):
                    case = {"op": "stat", "input": s, "axis": list(kaxis), "npartitions": npart,
                            "name": name, "reduce_axis": list(ax) if isinstance(ax, tuple) else ax,
                            "keepdims": False, "numerics": True}
                    r = getattr(b, name)(axis=ax)
                    case["result_type"] = type(r).__name__
                    case["result_dtype"] = str(np.asarray(r).dtype)
                    add(case, out=np.asarray(r))


def gen_reshape():
    """Keys.reshape / Values.reshape (shapes.py:40-64, :111-134), mirroring
    test_spark_shaping.py:27-84 plus larger and multi-partition cases."""
    x = spec((2, 3, 4))
    y = spec((6, 4, 5), "float32", "normal", 80)
    z = spec((8, 3, 2, 5), "uint16", "ints", 81)
    items = [
        (x, (0, 1), "keys", (3, 2), None), (x, (0,), "keys", (2, 1), None), (x, (0,), "keys", (2,), None),
        (x, (0, 1), "keys", (2, 3), None), (x, (0, 1), "keys", (2, 3, 4), None),
        (x, (0,), "values", (4, 3), None), (x, (0, 1), "values", (1, 4), None), (x, (0, 1), "values", (4,), None),
        (x, (0,), "values", (3, 4), None), (x, (0, 1), "values", (2, 3, 4), None),
        (y, (0, 1), "keys", (24,), 3), (y, (0, 1), "keys", (4, 6), 5), (y, (0, 1), "keys", (2, 2, 6), None),
        (y, (0,), "keys", (3, 2), 2), (y, (0,), "values", (5, 4), 2), (y, (0,), "values", (20,), 4),
        (y, (0,), "values", (2, 10), None), (y, (0, 1), "values", (5, 1), 3), (y, (0,), "values", (3, 7), None),
        (z, (0, 1), "keys", (4, 6), 4), (z, (0, 1, 2), "keys", (48,), 3), (z, (0,), "values", (6, 5), 3),
        (z, (0, 1), "values", (10,), 2), (z, (0, 1), "keys", (25,), None),
    ]
    for s, ax, which, new, npart in items:
        xx = make_input(s)
        b = bolt.array(xx, sc, axis=ax, npartitions=npart)
        case = {"op": "reshape", "input": s, "axis": list(ax), "npartitions": npart, "which": which,
                "new": list(new)}
        r = run(lambda: getattr(b, which).reshape(new), case)
        if r is None:
            add(case)
            continue
        case.update(shape=list(r.shape), split=r.split)
        add(case, out=r.toarray())
    # varargs spelling: b.keys.reshape(3, 2)
    xx = make_input(x)
    b = bolt.array(xx, sc, axis=(0, 1))
    r = b.keys.reshape(3, 2)
    add({"op": "reshape", "input": x, "axis": [0, 1], "npartitions": None, "which": "keys", "new": [3, 2],
         "varargs": True, "shape": list(r.shape), "split": r.split}, out=r.toarray())


def gen_reduce():
    """reduce(func, axis, keepdims) with numpy ufuncs, operator functions and
    plain lambdas (array.py:243-282; test_spark_functional.py:31-48)."""
    from funcs import RFUNCS
    ia = spec((4, 3, 5))
    f32 = spec((6, 4, 5), "float32", "normal", 90)
    fnan = spec((5, 4, 3), "float64", "normal", 91, nan_every=7)
    u8 = spec((7, 3, 4), "uint8", "ints", 92)
    i16 = spec((6, 5), "int16", "ints", 93)
    bb = spec((6, 5), "bool", "bool", 94)
    one = spec((1, 4, 5), "float32", "normal", 95)
    rep = spec((10, 10, 10))  # test_spark_functional.py:34-36 style (arange)
    table = [
        (ia, ["add", "np_add", "multiply", "mul", "maximum", "minimum", "fmax", "logical_and", "logical_or",
              "bitwise_and", "bitwise_or", "bitwise_xor", "and_", "or_", "xor", "lam_add", "lam_absadd", "lam_mul"]),
        (f32, ["add", "multiply", "maximum", "fmin", "logical_and", "logical_or", "bitwise_and", "lam_add",
               "lam_absadd"]),
        (fnan, ["maximum", "minimum", "fmax", "fmin", "add", "logical_and"]),
        (u8, ["add", "multiply", "bitwise_and", "bitwise_or", "bitwise_xor", "maximum", "logical_or", "lam_mul"]),
        (i16, ["multiply", "bitwise_xor", "fmin", "lam_add"]),
        (bb, ["add", "multiply", "logical_and", "logical_or", "bitwise_xor", "maximum", "lam_add"]),
        (one, ["add", "logical_and", "bitwise_and", "lam_absadd"]),
        (rep, ["add", "maximum", "lam_add"]),
    ]
    for s, names in table:
        x = make_input(s)
        nd = len(s["shape"])
        axes_list = [(0,), (1,), (0, 1)] + ([(0, 2), (0, 1, 2)] if nd == 3 else [])
        for kax in ((0,), (0, 1)):
            for npart in (None, 3):
                b = bolt.array(x, sc, axis=kax, npartitions=npart)
                for name in names:
                    for ax in axes_list:
                        for keep in ((False, True) if ax == (0,) else (False,)):
                            case = {"op": "reduce", "input": s, "axis": list(kax), "npartitions": npart,
                                    "func": name, "reduce_axis": list(ax), "keepdims": keep}
                            r = run(lambda: b.reduce(RFUNCS[name], axis=ax, keepdims=keep), case)
                            if r is None:
                                add(case)
                                continue
                            case["result_type"] = type(r).__name__
                            a = np.asarray(r.toarray() if hasattr(r, "toarray") else r)
                            case["result_dtype"] = str(a.dtype)
                            add(case, out=a)


def gen_unit_axes():
    """Swaps and statistics around length-1 axes (round 6): the reference's swap
    chain squeezes unit value axes (chunk.py:193-197, :284-287, :342-345), so a
    (1, 5) swap((0,), (0,)) is (5,) and statistics whose _align swaps end on
    (1,) values are scalars (array.py:85-115, :316-329).  Only cases the
    reference answers are kept (a chain that raises in the reference keeps
    numpy's answer in bolt_amd, docs/HISTORY.md §4 item 6), and only those
    whose result is not numpy's shape."""
    swaps = [((1, 5), (0,), (0,), (0,)), ((5, 3, 1), (0,), (), (0,)), ((2, 3, 1), (0, 1), (1,), ()),
             ((2, 2, 5, 1), (0, 1, 2), (1, 2), ()), ((5, 1), (0,), (0,), (0,)), ((3, 4, 1, 1), (0,), (), (0, 1)),
             ((6, 1, 1), (0,), (0,), (1,)), ((1, 1), (0,), (0,), (0,)), ((4, 6, 1), (0,), (0,), (1,)),
             ((3, 2, 4, 1), (0, 1), (0,), (1,)), ((2, 3, 4, 1), (0, 1, 2), (0, 2), ())]
    for i, (sh, axis, kax, vax) in enumerate(swaps):
        s = spec(sh, ("float32", "float64", "int16", "uint8")[i % 4], "normal" if i % 4 < 2 else "ints", 30 + i)
        x = make_input(s)
        b = bolt.array(x, sc, axis=axis)
        case = {"op": "swap", "input": s, "axis": list(axis), "kaxes": list(kax), "vaxes": list(vax), "size": "150"}
        r = run(lambda: b.swap(kax, vax), case)
        if r is None:
            continue
        case.update(shape=list(r.shape), split=r.split)
        add(case, out=_sorted_array(r))
    shapes = [((3, 4, 1), (0, 1)), ((4, 1), (0,)), ((1, 5), (0,)), ((2, 3, 1, 1), (0, 1)), ((5, 2, 1), (0,)),
              ((1, 3, 1, 2, 1), (0, 1)), ((3, 1, 4), (0, 1, 2)), ((2, 1, 1, 3), (0,))]
    for i, (sh, kaxis) in enumerate(shapes):
        s = spec(sh, ("float64", "float32", "int32", "uint16")[i % 4], "normal" if i % 4 < 2 else "ints", 50 + i)
        x = make_input(s)
        b = bolt.array(x, sc, axis=kaxis, npartitions=2)
        nd = x.ndim
        axes = [(a,) for a in range(nd)] + [(a, c) for a in range(nd) for c in range(a + 1, nd)]
        for ax in axes:
            for name in ("mean", "var", "std", "sum", "max"):
                for keep in (False, True):
                    case = {"op": "stat", "input": s, "axis": list(kaxis), "npartitions": 2,
                            "name": name, "reduce_axis": list(ax), "keepdims": keep}
                    r = run(lambda: getattr(b, name)(axis=ax, keepdims=keep), case)
                    if r is None:
                        continue
                    a = np.asarray(r.toarray() if hasattr(r, "toarray") else r)
                    kept = tuple(d for j, d in enumerate(sh) if j not in ax)
                    plain = tuple(1 if j in ax else d for j, d in enumerate(sh)) if keep else kept
                    if a.shape == plain or (plain == (1,) and a.shape == ()):
                        continue  # numpy's shape: covered elsewhere
                    case["result_type"] = type(r).__name__
                    case["result_dtype"] = str(a.dtype)
                    add(case, out=a)


if __name__ == "__main__":
    sc = FakeContext(2)
    for g in (gen_construct, gen_swap, gen_transpose, gen_chunk, gen_moves, gen_getplan, gen_stats,
              gen_stat_errors, gen_getitem, gen_concatenate, gen_chunk_map,
              gen_functional, gen_stats_numerics, gen_reshape, gen_reduce, gen_unit_axes):
        try:
            g()
        except Exception:
            traceback.print_exc()
            raise
    meta = {"generator": "tests/golden/make_golden.py", "reference": "beautifulNow1992/bolt v%s" % bolt.__version__,
            "numpy": np.__version__, "python": sys.version.split()[0], "cases": CASES}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=0, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **ARRAYS)
    print("wrote %d cases, %d arrays" % (len(CASES), len(ARRAYS)))
