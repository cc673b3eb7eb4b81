"""Differential fuzz against the REFERENCE itself (build container only: it
imports /root/reference through tests/golden/make_golden.py's fake Spark
context and its old-numpy shims; nothing of it reaches the GPU box).

Random arrays (extents 2-6, random splits and dtypes) go through the same
random operation on the reference's Spark mode and on bolt_amd (the numpy
test executor of the kernel contracts; the HIP kernels are held to that
executor's bytes by the GPU suites): swap, transpose, chunk -> records ->
unchunk, keys_to_values / values_to_keys, indexing, mean / var / std, sum /
min / max (also with keepdims), reduce with numpy ufuncs, key / value reshape
and transpose, swapaxes, concatenate, map, filter, first, astype, clip,
stack -> map -> unstack, ChunkedArray.map.  Data movement must
be bit-exact, statistics within tests/golden_cases.stat_close's rule, and an
operation the reference refuses must raise the same exception type here.  The
reference behaviours bolt_amd does not keep (docs/HISTORY.md §4) are routed
around: length-1 axes are not generated, records are compared in key order,
paddings that trigger removepad's over-trim are not drawn, an array the
reference builds but cannot collect must raise ValueError here, a transpose
of an all-key array (which the reference cannot do) must be numpy's, and
filter is compared in key order (the reference's sort=True), and so is a
list index on every axis of an array a shuffle left out of key order (the
reference applied to the same array in key order).

    PYTHONDONTWRITEBYTECODE=1 python tools/reference_diff_fuzz.py 0 2000
    BOLT_AMD_DIFF_PADDED=1 ... (the same with padded rows for small arrays)
"""
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests", "golden"), os.path.join(HERE, "tests"), HERE]

import make_golden  # noqa: E402,F401  (the reference, its shims, fakespark)
import numpy as np  # noqa: E402

import bolt as ref_bolt  # noqa: E402  (the reference)
from fakerdd import FakeContext  # noqa: E402

import bolt_amd  # noqa: E402
import cpu_backend  # noqa: E402
import golden_cases as G  # noqa: E402
from test_chunk_fuzz import _chunk_args  # noqa: E402
from test_getitem_fuzz import _index  # noqa: E402

DTYPES = [np.float32, np.float64, np.int32, np.uint8, np.int16, np.uint16]
# BOLT_AMD_DIFF_MIN_EXTENT=1 also draws length-1 axes.  Around them the
# reference's swap chain squeezes unit value axes (bolt_amd returns the same
# shapes: plan.swap_shape) and raises IndexError / ValueError / AxisError in
# many chains where numpy has an answer; bolt_amd keeps numpy's answer there
# (docs/HISTORY.md §4 item 6).  Such a refusal is counted, not failed, when the
# array involved has a unit axis; every result the reference does return must
# match, shape and split included.
MIN_EXTENT = int(os.environ.get("BOLT_AMD_DIFF_MIN_EXTENT", "2"))
REF_RAISED = [0]  # unit-axis refusals of the reference where bolt_amd answers
UNIT = [False]    # the chain's current array has a length-1 axis
CATALOGUE = os.environ.get("BOLT_AMD_DIFF_CATALOGUE") == "1"  # list every difference, by message
if os.environ.get("BOLT_AMD_DIFF_PADDED") == "1":
    # every transposed result whose rows are not a multiple of 16 B is stored
    # with padded rows (tests/test_row_pitch.py's small_pitch settings)
    import bolt_amd.mi355x.array as _A
    _A._PITCH_MIN_ROW, _A._PITCH_LINE, _A._PITCH_ALIGN, _A._PITCH_PAD_DIV = 1, 16, 64, 0
    PADDED = [0]
    _plan = _A._pitch_plan

    def _counted(*a):
        r = _plan(*a)
        PADDED[0] += r is not None
        return r
    _A._pitch_plan = _counted
else:
    PADDED = None


class Refused(Exception):
    pass


def ref_records(r):
    return sorted(r._rdd.collect(), key=lambda kv: kv[0])


def ref_array(r):
    """The reference's array in key order (its sortByKey + collect); ValueError
    when its records cannot fill the shape it declares."""
    recs = ref_records(r)
    try:
        return np.asarray([v for _, v in recs]).reshape(r.shape)
    except ValueError as e:
        raise Refused("uncollectable: %s" % e)


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and a.dtype == b.dtype and a.tobytes() == b.tobytes()


def run_both(f_ref, f_ours, unit=None):
    """(ref result, our result) or (exception name, None) when both refuse alike.
    ``unit``: the input has a length-1 axis, where a refusal of the reference
    only is counted (REF_RAISED), not failed (default: the chain's current array)."""
    unit = UNIT[0] if unit is None else unit
    try:
        rv = f_ref()
        if hasattr(rv, "_rdd") and not hasattr(rv, "plan"):
            ref_array(rv)  # an uncollectable array counts as refused (ValueError)
    except Refused:
        try:
            ov = f_ours()
            if hasattr(ov, "toarray"):
                ov.toarray()
        except ValueError:
            return "refused", None
        raise AssertionError("reference array cannot be collected; bolt_amd did not refuse")
    except Exception as e:
        try:
            f_ours()
        except Exception as e2:
            if unit and MIN_EXTENT == 1 and type(e2).__name__ != type(e).__name__:
                REF_RAISED[0] += 1
                return "raised " + type(e).__name__, None
            assert type(e2).__name__ == type(e).__name__, (type(e).__name__, type(e2).__name__, e2)
            return "raised " + type(e).__name__, None
        if unit and MIN_EXTENT == 1:
            REF_RAISED[0] += 1
            return "raised " + type(e).__name__, None
        raise AssertionError("reference raised %s (%s); bolt_amd did not" % (type(e).__name__, e))
    return rv, f_ours()


def check_array(rv, ov, what):
    assert tuple(ov.shape) == tuple(rv.shape) and ov.split == rv.split, (what, ov.shape, rv.shape, ov.split, rv.split)
    assert same(ov.toarray(), ref_array(rv)), what


def check_chunked(rv, ov, what):
    assert tuple(ov.shape) == tuple(rv.shape) and ov.split == rv.split, (what, ov.shape, rv.shape)
    assert np.array_equal(ov.plan, rv.plan) and np.array_equal(ov.padding, rv.padding), (what, ov.plan, rv.plan)
    got = list(ov.records())
    want = ref_records(rv)
    assert [tuple(k) for k, _ in got] == [tuple(k) for k, _ in want], what
    for (k, gv), (_, wv) in zip(got, want):
        assert same(gv, np.ascontiguousarray(wv) if np.ndim(wv) else np.asarray(wv)), (what, k)  # 0-d: a squeezed record


def one_case(seed, sc, ctx):
    rng = np.random.default_rng(20000 + seed)
    nd = int(rng.integers(2, 6))
    shape = tuple(int(rng.integers(MIN_EXTENT, 7 if nd > 3 else 9)) for _ in range(nd))
    split = int(rng.integers(1, nd + 1))
    dtype = DTYPES[int(rng.integers(0, len(DTYPES)))]
    if np.dtype(dtype).kind == "f":
        x = (5 + 2 * rng.standard_normal(shape)).astype(dtype)
    else:
        x = rng.integers(0, 60, size=shape).astype(dtype)
    axis = tuple(range(split))
    npart = int(rng.integers(1, 5))
    r = ref_bolt.array(x, sc, axis=axis, npartitions=npart)
    o = bolt_amd.array(x, ctx, axis=axis)
    check_array(r, o, "construct")
    fam = ["swap", "transpose", "chunk", "getitem", "stat", "reduce", "reshape", "concat", "map", "filter",
           "swapaxes", "kvtranspose", "keepdims", "ufunc", "first", "astype", "clip", "stack", "chunkmap"]
    did = []
    for _ in range(int(rng.integers(1, 4))):
        f = fam[int(rng.integers(0, len(fam)))]
        did.append(f)
        nd, split = len(r.shape), r.split
        UNIT[0] = 1 in r.shape
        if f == "swap":
            kax = tuple(sorted(rng.choice(split, int(rng.integers(0, split + 1)), replace=False).tolist()))
            vax = tuple(sorted(rng.choice(nd - split, int(rng.integers(0, nd - split + 1)), replace=False).tolist()))
            if (len(kax) == split and not vax) or not (kax or vax):
                continue
            rv, ov = run_both(lambda: r.swap(kax, vax), lambda: o.swap(kax, vax))
            if ov is not None:
                check_array(rv, ov, ("swap", kax, vax))
                r, o = rv, ov
        elif f == "transpose":
            perm = tuple(rng.permutation(nd).tolist())
            if split == nd:
                # the reference cannot transpose an all-key array (Values.transpose(())
                # -> max() of an empty sequence, utils.py:171): a bug not kept
                # (docs/HISTORY.md §4 item 7); bolt_amd gives numpy's transpose
                try:
                    r.transpose(perm)
                    raise AssertionError("the reference transposed an all-key array")
                except ValueError:
                    pass
                ot = o.transpose(perm)
                assert ot.split == split and same(ot.toarray(), np.transpose(o.toarray(), perm)), ("T all-key", perm)
                continue
            rv, ov = run_both(lambda: r.transpose(perm), lambda: o.transpose(perm))
            if ov is not None:
                check_array(rv, ov, ("transpose", perm))
                r, o = rv, ov
        elif f == "chunk":
            if split == nd:
                continue
            size, caxes, pad = _chunk_args(rng, r.shape[split:])
            rv, ov = run_both(lambda: r.chunk(size, axis=caxes, padding=pad), lambda: o.chunk(size, axis=caxes, padding=pad))
            if ov is None:
                continue
            check_chunked(rv, ov, ("chunk", size, caxes, pad))
            if rng.random() < 0.5 and rv.split > 1:
                k = (int(rng.integers(0, rv.split)),)
                rv2, ov2 = run_both(lambda: rv.keys_to_values(k), lambda: ov.keys_to_values(k))
                if ov2 is not None:
                    check_chunked(rv2, ov2, ("k2v", k))
                    rv, ov = rv2, ov2
            elif len(rv.vshape) > 1:
                v = (int(rng.integers(0, len(rv.vshape))),)
                rv2, ov2 = run_both(lambda: rv.values_to_keys(v), lambda: ov.values_to_keys(v))
                if ov2 is not None:
                    check_chunked(rv2, ov2, ("v2k", v))
                    rv, ov = rv2, ov2
            ru, ou = rv.unchunk(), ov.unchunk()
            check_array(ru, ou, "unchunk")
        elif f == "getitem":
            index = _index(rng, r.shape, split)
            if index is None:
                continue
            rr = r
            if not getattr(r, "_ordered", True) and (isinstance(index, list) or (
                    isinstance(index, tuple) and all(isinstance(i, list) for i in index))):
                # advanced indexing numbers the selected records in the RDD's
                # current order (array.py:552 zipWithIndex), which after a
                # shuffle is the partitioner's, not key order (docs/HISTORY.md
                # §4 item 9): compared with the reference on the same array in
                # key order
                rr = ref_bolt.array(ref_array(r), sc, axis=tuple(range(r.split)))
            rv, ov = run_both(lambda: rr[index], lambda: o[index])
            if ov is None:
                continue
            if hasattr(rv, "_rdd"):
                check_array(rv, ov, ("getitem", index))
            else:
                assert type(ov).__name__ == type(rv).__name__ and same(ov, rv), ("getitem scalar", index)
        elif f == "stat":
            ax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
            name = ["mean", "var", "std"][int(rng.integers(0, 3))]
            rv, ov = run_both(lambda: getattr(r, name)(axis=ax), lambda: getattr(o, name)(axis=ax))
            if ov is None:
                continue
            a, w = np.asarray(ov), np.asarray(rv)
            assert a.shape == w.shape and a.dtype == w.dtype, (name, a.shape, w.shape, a.dtype, w.dtype)
            xa = o.toarray()
            assert G.stat_close(a, w, G.truth_stat(xa, name, ax), w.dtype, xa, name), (name, ax)
        elif f == "reduce":
            ax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
            name = ["sum", "min", "max"][int(rng.integers(0, 3))]
            rv, ov = run_both(lambda: getattr(r, name)(axis=ax), lambda: getattr(o, name)(axis=ax))
            if ov is None:
                continue
            a = np.asarray(ov.toarray() if hasattr(ov, "toarray") else ov)
            w = np.asarray(rv.toarray() if hasattr(rv, "toarray") else rv)
            assert G.reduce_close(a, w, o.toarray(), "add" if name == "sum" else name, ax), (name, ax)
        elif f == "reshape":
            which = "keys" if rng.random() < 0.5 or split == nd else "values"
            dims = r.shape[:split] if which == "keys" else r.shape[split:]
            n = int(np.prod(dims))
            parts = int(rng.integers(1, 4))
            new = [1] * parts
            k = n
            for p in range(2, n + 1):
                while k % p == 0:
                    new[int(rng.integers(0, parts))] *= p
                    k //= p
            new = tuple(new)
            if 1 in new:
                continue
            rv, ov = run_both(lambda: getattr(r, which).reshape(new), lambda: getattr(o, which).reshape(new))
            if ov is not None:
                check_array(rv, ov, ("reshape", which, new))
                r, o = rv, ov
        elif f == "concat":
            cat = int(rng.integers(0, nd))
            oshape = list(r.shape)
            oshape[cat] = int(rng.integers(2, 4))
            other = (np.arange(int(np.prod(oshape))) % 11).astype(r.dtype).reshape(oshape)
            rv, ov = run_both(lambda: r.concatenate(other, axis=cat), lambda: o.concatenate(other, axis=cat))
            if ov is not None:
                check_array(rv, ov, ("concatenate", cat))
        elif f == "map":
            ax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
            rv, ov = run_both(lambda: r.map(lambda v: v * 2 + 1, axis=ax), lambda: o.map(lambda v: v * 2 + 1, axis=ax))
            if ov is not None:
                assert tuple(ov.shape) == tuple(rv.shape) and ov.split == rv.split, ("map", ax, ov.shape, rv.shape)
                assert np.dtype(ov.dtype) == np.dtype(rv.dtype), ("map dtype", ov.dtype, rv.dtype)
                assert same(ov.toarray(), ref_array(rv)), ("map", ax)
        elif f == "swapaxes":
            if nd < 2:
                continue
            a1, a2 = (int(v) for v in rng.choice(nd, 2, replace=False))
            if split == nd:
                continue  # an all-key array: the reference cannot transpose it (item 7)
            rv, ov = run_both(lambda: r.swapaxes(a1, a2), lambda: o.swapaxes(a1, a2))
            if ov is not None:
                check_array(rv, ov, ("swapaxes", a1, a2))
                r, o = rv, ov
        elif f == "kvtranspose":
            which = "keys" if rng.random() < 0.5 or split == nd else "values"
            n = split if which == "keys" else nd - split
            p = tuple(rng.permutation(n).tolist())
            rv, ov = run_both(lambda: getattr(r, which).transpose(*p), lambda: getattr(o, which).transpose(*p))
            if ov is not None:
                check_array(rv, ov, (which + ".transpose", p))
                r, o = rv, ov
        elif f == "keepdims":
            ax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
            name = ["sum", "mean", "max", "std"][int(rng.integers(0, 4))]
            rv, ov = run_both(lambda: getattr(r, name)(axis=ax, keepdims=True),
                              lambda: getattr(o, name)(axis=ax, keepdims=True))
            if ov is None:
                continue
            a = np.asarray(ov.toarray() if hasattr(ov, "toarray") else ov)
            w = np.asarray(rv.toarray() if hasattr(rv, "toarray") else rv)
            assert a.shape == w.shape and a.dtype == w.dtype, (name, "keepdims", a.shape, w.shape)
            xa = o.toarray()
            if name in ("mean", "std"):
                assert G.stat_close(a, w, G.truth_stat(xa, name, ax).reshape(w.shape), w.dtype, xa, name), name
            else:
                assert G.reduce_close(a, w, xa, "add" if name == "sum" else name, ax), name
        elif f == "ufunc":
            ax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
            kind = np.dtype(r.dtype).kind
            ufs = [np.multiply, np.maximum, np.minimum, np.fmax, np.fmin] + (
                [np.bitwise_and, np.bitwise_or, np.bitwise_xor, np.logical_and, np.logical_or] if kind in "iu" else [])
            uf = ufs[int(rng.integers(0, len(ufs)))]
            rv, ov = run_both(lambda: r.reduce(uf, axis=ax), lambda: o.reduce(uf, axis=ax))
            if ov is None:
                continue
            a = np.asarray(ov.toarray() if hasattr(ov, "toarray") else ov)
            w = np.asarray(rv.toarray() if hasattr(rv, "toarray") else rv)
            fname = {np.multiply: "multiply"}.get(uf, uf.__name__)
            assert G.reduce_close(a, w, o.toarray(), fname, ax), ("reduce", uf.__name__, ax)
        elif f == "first":
            rv, ov = run_both(lambda: r.first(), lambda: o.first())
            if ov is not None:
                assert same(np.asarray(ov), np.asarray(rv)), "first"
        elif f == "astype":
            dt = [np.float64, np.int32, np.uint8, np.float32][int(rng.integers(0, 4))]
            rv, ov = run_both(lambda: r.astype(dt), lambda: o.astype(dt))
            if ov is not None:
                check_array(rv, ov, ("astype", dt))
                r, o = rv, ov
        elif f == "clip":
            lo_, hi_ = sorted(float(v) for v in rng.integers(0, 60, 2))
            rv, ov = run_both(lambda: r.clip(lo_, hi_), lambda: o.clip(lo_, hi_))
            if ov is not None:
                check_array(rv, ov, ("clip", lo_, hi_))
        elif f == "stack":
            size = int(rng.integers(1, 5))
            rv, ov = run_both(lambda: r.stack(size).map(lambda v: v + 1).unstack(),
                              lambda: o.stack(size).map(lambda v: v + 1).unstack())
            if ov is not None:
                assert tuple(ov.shape) == tuple(rv.shape) and ov.split == rv.split, ("stack", ov.shape, rv.shape)
                assert same(ov.toarray(), ref_array(rv)), ("stack", size)
        elif f == "chunkmap":
            if split == nd:
                continue
            size, caxes, pad = _chunk_args(rng, r.shape[split:])
            rv, ov = run_both(lambda: r.chunk(size, axis=caxes, padding=pad).map(lambda v: v * 3 + 2),
                              lambda: o.chunk(size, axis=caxes, padding=pad).map(lambda v: v * 3 + 2))
            if ov is not None:
                check_chunked(rv, ov, ("chunk.map", size, caxes, pad))
                check_array(rv.unchunk(), ov.unchunk(), "chunk.map unchunk")
        elif f == "filter":
            ax = tuple(sorted(rng.choice(nd, int(rng.integers(1, nd + 1)), replace=False).tolist()))
            thr = float(np.median(r.toarray().astype(np.float64)))
            srt = bool(rng.random() < 0.5)

            def keep(v):
                tot = v.double().sum() if hasattr(v, "double") else np.asarray(v).astype(np.float64).sum()
                return float(tot) > thr * max(1, v.reshape(-1).shape[0])
            # bolt_amd renumbers the kept records in key order whatever ``sort`` says;
            # the reference's sort=False keeps its RDD's current order, which after
            # a shuffle (a swap / transpose earlier in the chain) is the shuffle's
            # (docs/HISTORY.md §4 item 8): compared with the reference's sort=True
            rv, ov = run_both(lambda: r.filter(keep, axis=ax, sort=True), lambda: o.filter(keep, axis=ax, sort=srt))
            if ov is not None:
                assert tuple(ov.shape) == tuple(rv.shape) and ov.split == rv.split, ("filter", ax, ov.shape, rv.shape)
                if rv.shape != (0,):
                    assert same(ov.toarray(), ref_array(rv)), ("filter", ax)
    return did


def main(lo, hi):
    cpu_backend.install()
    ctx = bolt_amd.MI355XContext(device="cpu")
    sc = FakeContext(4)
    counts, bad = {}, []
    t0 = time.time()
    for seed in range(lo, hi):
        try:
            for f in one_case(seed, sc, ctx):
                counts[f] = counts.get(f, 0) + 1
        except Exception:
            bad.append((seed, traceback.format_exc()[-1500:]))
            if len(bad) >= 5 and not CATALOGUE:
                break
    if CATALOGUE:
        kinds = {}
        for seed, tb in bad:
            kinds.setdefault(tb.strip().splitlines()[-1][:160], []).append(seed)
        for k, seeds in sorted(kinds.items(), key=lambda kv: -len(kv[1])):
            print("%5d  e.g. seed %d  %s" % (len(seeds), seeds[0], k))
        bad = bad[:3]
    print("seeds %d..%d: %d failed, operations compared %s, %.0f s"
          % (lo, hi - 1, len(bad), dict(sorted(counts.items())), time.time() - t0))
    if MIN_EXTENT == 1:
        print("unit-axis refusals of the reference only (bolt_amd answers as numpy): %d" % REF_RAISED[0])
    if PADDED is not None:
        print("padded rows: %d distinct padded move plans" % PADDED[0])
    for seed, tb in bad:
        print("seed %d:\n%s" % (seed, tb))
    return 1 if bad else 0


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:3]] or [0, 200]
    sys.exit(main(*a))
