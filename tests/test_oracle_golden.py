"""Pin the CPU oracle (oracle/bolt_oracle.py) against the reference's own outputs.

Every fixture in tests/golden was produced by the reference bolt (Spark mode,
tests/golden/make_golden.py).  Data movement must match bit for bit (bytes,
shape, split, chunk keys, plan, padding); statistics by the rule in
golden_cases.stat_close; errors by exception type.
"""
import numpy as np
import pytest

import golden_cases as G
from oracle import bolt_oracle as O


def _rs(case, npart=2):
    x = G.make_input(case["input"])
    return x, O.parallelize(x, axis=G.tup(case["axis"]), npartitions=npart or 2)


@pytest.mark.parametrize("case", G.cases("construct"), ids=G.case_id)
def test_construct(case):
    x = G.make_input(case["input"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.parallelize(x, axis=G.tup(case["axis"]))
        assert type(e.value).__name__ == case["raises"]
        return
    rs = O.parallelize(x, axis=G.tup(case["axis"]), npartitions=case["npartitions"] or 2)
    assert list(rs.shape) == case["shape"] and rs.split == case["split"]
    assert O.toarray(rs).tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("swap"), ids=G.case_id)
def test_swap(case):
    x, rs = _rs(case)
    size = G.size_arg(case["size"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.swap(rs, G.tup(case["kaxes"]), G.tup(case["vaxes"]), size)
        assert type(e.value).__name__ == case["raises"]
        return
    out = O.swap(rs, G.tup(case["kaxes"]), G.tup(case["vaxes"]), size)
    assert list(out.shape) == case["shape"] and out.split == case["split"]
    got = O.toarray(out)
    # key order (the reference's sortByKey order; see make_golden.py on toarray_unsorted)
    want = G.arr(case, "out_sorted" if case.get("toarray_unsorted") else "out")
    assert got.dtype == want.dtype and got.tobytes() == want.tobytes()


@pytest.mark.parametrize("case", [c for c in G.cases("transpose") if "raises" not in c], ids=G.case_id)
def test_transpose(case):
    x, rs = _rs(case)
    out = O.transpose(rs, case["perm"])
    assert list(out.shape) == case["shape"] and out.split == case["split"]
    assert O.toarray(out).tobytes() == G.arr(case, "out").tobytes()


def _chunk_check(c, case):
    recs = sorted(c.records(), key=lambda kv: kv[0])
    assert [list(k) for k, _ in recs] == case["keys"]
    assert [list(v.shape) for _, v in recs] == case["shapes"]
    flat = np.concatenate([v.reshape(-1) for _, v in recs])
    assert flat.tobytes() == G.arr(case, "flat").tobytes()
    assert [int(p) for p in c.plan] == case["plan"]
    assert [int(p) for p in c.padding] == case["padding_out"]


@pytest.mark.parametrize("case", G.cases("chunk"), ids=G.case_id)
def test_chunk(case):
    x, rs = _rs(case)
    size = case["size"]
    size = size if isinstance(size, (str, int)) else tuple(size)
    pad = G.tup(case["padding"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.chunk(rs, size, G.tup(case["chunk_axis"]), pad)
        assert type(e.value).__name__ == case["raises"]
        return
    c = O.chunk(rs, size, G.tup(case["chunk_axis"]), pad)
    _chunk_check(c, case)
    if "unchunk_raises" in case:
        return
    u = O.unchunk(c)
    assert list(u.shape) == case["unchunk_shape"]
    assert O.toarray(u).tobytes() == G.arr(case, "unchunk").tobytes()


@pytest.mark.parametrize("case", G.cases("moves"), ids=G.case_id)
def test_moves(case):
    x, rs = _rs(case)
    size = case["size"]
    size = size if isinstance(size, (str, int)) or size is None else tuple(size)
    c = O.chunk(rs, size, None, G.tup(case["padding"]))

    def apply(c):
        for name, axes, z in case["steps"]:
            c = O.keys_to_values(c, tuple(axes), size=G.tup(z)) if name == "k2v" else O.values_to_keys(c, tuple(axes))
        return c
    if "raises" in case:
        with pytest.raises(Exception):
            apply(c)
        return
    c = apply(c)
    assert list(c.shape) == case["chunk_shape"] and c.split == case["split"]
    _chunk_check(c, case)
    u = O.unchunk(c)
    assert O.toarray(u).tobytes() == G.arr(case, "unchunk").tobytes()


@pytest.mark.parametrize("case", G.cases("getplan"), ids=G.case_id)
def test_getplan(case):
    plan, pad = O.getplan(case["vshape"], case["dtype"], case["size"])
    assert [int(p) for p in plan] == case["plan"]


def _light(case):
    # the C1 (100,64,64) inputs: keep the oracle run to a few seconds per case
    if case["input"]["shape"] == [100, 64, 64]:
        return case["reduce_axis"] in (0, [1, 2]) and not case["keepdims"]
    return True


@pytest.mark.parametrize("case", [c for c in G.cases("stat") if _light(c)], ids=G.case_id)
def test_stat(case):
    x = G.make_input(case["input"])
    rs = O.parallelize(x, axis=G.tup(case["axis"]), npartitions=case["npartitions"] or 2)
    name = {"var": "variance", "std": "stdev"}.get(case["name"], case["name"])
    ax = G.tup(case["reduce_axis"])
    red = {"sum": O.sum_, "min": O.min_, "max": O.max_}.get(name)
    f = (lambda: red(rs, ax, case["keepdims"])) if red else \
        (lambda: O.stat(rs, name, ax, case["keepdims"]))
    if "raises" in case:
        with pytest.raises(Exception) as e:
            f()
        assert type(e.value).__name__ == case["raises"]
        return
    got = f()
    want = G.arr(case, "out")
    assert str(np.asarray(got).dtype) == case["result_dtype"]
    assert np.asarray(got).shape == want.shape
    if want.dtype.kind in 'iub' or case["name"] in ("min", "max"):
        assert np.asarray(got).tobytes() == want.tobytes()
    else:
        truth = G.truth_stat(x, case["name"], ax)
        ok = G.stat_close(got, want, truth, want.dtype, x, case["name"])
        if not ok and case.get("numerics"):
            # offset / outlier inputs: the oracle restates the reference's
            # order-dependent Welford, whose error on this ill-conditioned data
            # is itself ~1e-12; the oracle's must be of the reference's order
            # (float32: the oracle accumulates in float32 too, in its own record
            # order, so allow float32 Welford's n-eps bound)
            g = np.asarray(got, dtype=np.longdouble)
            slack = (1e-4 if want.dtype == np.float32 else 1e-12) * np.abs(truth)
            ok = bool(np.all(np.abs(g - truth) <= 4 * np.abs(np.asarray(want, dtype=np.longdouble) - truth)
                             + slack))
        assert ok


@pytest.mark.parametrize("case", G.cases("getitem"), ids=G.case_id)
def test_getitem(case):
    x, rs = _rs(case, case["npartitions"])
    idx = G.index_arg(case["index"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.getitem(rs, idx)
        assert type(e.value).__name__ == case["raises"]
        return
    r = O.getitem(rs, idx)
    if "collect_raises" in case:
        with pytest.raises(ValueError):
            O.toarray(r)
        return
    want = G.arr(case, "out_sorted" if case.get("toarray_unsorted") else "out")
    if case["kind"] == "scalar":
        assert type(r).__name__ == case["result_type"] and np.asarray(r).tobytes() == want.tobytes()
        return
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert O.toarray(r).tobytes() == want.tobytes()


@pytest.mark.parametrize("case", G.cases("squeeze"), ids=G.case_id)
def test_squeeze(case):
    x, rs = _rs(case)
    q = G.tup(case["squeeze"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.squeeze(rs, q)
        assert type(e.value).__name__ == case["raises"]
        return
    r = O.squeeze(rs, q)
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert O.toarray(r).tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("concatenate"), ids=G.case_id)
def test_concatenate(case):
    x, rs = _rs(case, case["npartitions"])
    if case["other"] is None:
        other = [[1, 2, 3]]
    else:
        y = G.make_input(case["other"])
        other = y if case["other_kind"] != "spark" else O.parallelize(y, axis=G.tup(case["other_axis"]))
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.concatenate(rs, other, case["cat_axis"])
        assert type(e.value).__name__ == case["raises"]
        return
    r = O.concatenate(rs, other, case["cat_axis"])
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert O.toarray(r).tobytes() == G.arr(case, "out").tobytes()


def _close(got, want, exact):
    if exact:
        return got.dtype == want.dtype and got.tobytes() == want.tobytes()
    rtol = 1e-6 if want.dtype == np.float32 else 1e-12
    scale = float(np.max(np.abs(want))) if want.size else 0.0
    return got.dtype == want.dtype and np.allclose(got, want, rtol=rtol, atol=rtol * scale)


@pytest.mark.parametrize("case", G.cases("chunk_map"), ids=G.case_id)
def test_chunk_map(case):
    from funcs import FUNCS, EXACT
    x, rs = _rs(case)
    c = O.chunk(rs, G.size_arg(case["size"]), None, G.tup(case["padding"]))
    f = FUNCS[case["func"]]
    vs = G.tup(case["value_shape"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.chunk_map(c, f, vs)
        assert type(e.value).__name__ == case["raises"]
        return
    r = O.chunk_map(c, f, vs)
    assert list(r.shape) == case["shape"] and list(r.plan) == case["plan"]
    assert _close(O.toarray(O.unchunk(r)), G.arr(case, "out"), case["func"] in EXACT)


@pytest.mark.parametrize("case", G.cases("chunk_map_generic"), ids=G.case_id)
def test_chunk_map_generic(case):
    x, rs = _rs(case)
    c = O.chunk(rs, G.size_arg(case["size"]))
    d = O.chunk_map_generic(c, lambda v: [int(v.sum()), list(v.shape)])
    assert list(d.shape) == case["shape"]
    assert [list(o) for o in d.reshape(-1)] == case["objects"]


@pytest.mark.parametrize("case", G.cases("stack"), ids=G.case_id)
def test_stack(case):
    x, rs = _rs(case, case["npartitions"])
    st = O.stack(rs, case["size"])
    recs = st.records()
    assert [list(v.shape) for _, v in recs] == case["stack_shapes"]
    assert [[list(k) for k in ks] for ks, _ in recs] == case["stack_keys"]
    assert O.toarray(O.unstack(st)).tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("stack_map"), ids=G.case_id)
def test_stack_map(case):
    from funcs import FUNCS, EXACT
    x, rs = _rs(case, case["npartitions"])

    def go():
        st = O.stack(rs, case["size"])
        for name in case["funcs"]:
            st = O.stack_map(st, FUNCS[name])
        return O.unstack(st)
    if "raises" in case:
        with pytest.raises(Exception) as e:
            go()
        assert type(e.value).__name__ == case["raises"]
        return
    r = go()
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert _close(O.toarray(r), G.arr(case, "out"), all(f in EXACT for f in case["funcs"]))


@pytest.mark.parametrize("case", G.cases("map"), ids=G.case_id)
def test_map(case):
    from funcs import FUNCS, EXACT
    x, rs = _rs(case, case["npartitions"])
    r = O.map_(rs, FUNCS[case["func"]], G.tup(case["map_axis"]), G.tup(case["value_shape"]), case["dtype"],
               case["with_keys"])
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert _close(O.toarray(r), G.arr(case, "out"), case["func"] in EXACT)


@pytest.mark.parametrize("case", G.cases("filter"), ids=G.case_id)
def test_filter(case):
    from funcs import FUNCS
    x, rs = _rs(case, case["npartitions"])
    r = O.filter_(rs, FUNCS[case["func"]], G.tup(case["filter_axis"]), case["sort"])
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    if case["shape"] != [0]:
        assert O.toarray(r).tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("reduce"), ids=G.case_id)
def test_reduce(case):
    from funcs import RFUNCS
    x, rs = _rs(case, case["npartitions"])
    ax = tuple(case["reduce_axis"])
    f = RFUNCS[case["func"]]
    if "raises" in case:
        with pytest.raises(Exception) as e:
            O.reduce_(rs, f, ax, case["keepdims"])
        assert type(e.value).__name__ == case["raises"]
        return
    got = O.reduce_(rs, f, ax, case["keepdims"])
    a = np.asarray(got)
    assert str(a.dtype) == case["result_dtype"]
    assert G.reduce_close(a, G.arr(case, "out"), x, case["func"], ax)


@pytest.mark.parametrize("case", G.cases("reshape"), ids=G.case_id)
def test_reshape(case):
    x, rs = _rs(case, case["npartitions"])
    f = O.keys_reshape if case["which"] == "keys" else O.values_reshape
    if "raises" in case:
        with pytest.raises(Exception) as e:
            f(rs, tuple(case["new"]))
        assert type(e.value).__name__ == case["raises"]
        return
    out = f(rs, tuple(case["new"]))
    assert list(out.shape) == case["shape"] and out.split == case["split"]
    assert O.toarray(out).tobytes() == G.arr(case, "out").tobytes()
