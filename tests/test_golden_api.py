"""The mi355x mode against the reference's own outputs (tests/golden).

Runs on the GPU (HIP kernels, marker `gpu`) and on the CPU test executor
(host logic).  Data movement: bit for bit, plus shape/split/plan/padding/
chunk keys and exception types; statistics: result type, dtype, shape, and
golden_cases.stat_close.
"""
import numpy as np
import pytest

import bolt_amd as bolt
import golden_cases as G
from bolt_amd.mi355x.plan import getplan


def _b(case, bctx, npart=None):
    x = G.make_input(case["input"])
    return x, bolt.array(x, bctx, axis=G.tup(case["axis"]), npartitions=npart)


@pytest.mark.parametrize("case", G.cases("construct"), ids=G.case_id)
def test_construct(case, bctx):
    x = G.make_input(case["input"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            bolt.array(x, bctx, axis=G.tup(case["axis"]))
        assert type(e.value).__name__ == case["raises"]
        return
    b = bolt.array(x, bctx, axis=G.tup(case["axis"]), npartitions=case["npartitions"])
    assert list(b.shape) == case["shape"] and b.split == case["split"]
    assert b.toarray().tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("swap"), ids=G.case_id)
def test_swap(case, bctx):
    x, b = _b(case, bctx)
    size = G.size_arg(case["size"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b.swap(G.tup(case["kaxes"]), G.tup(case["vaxes"]), size=size)
        assert type(e.value).__name__ == case["raises"]
        return
    r = b.swap(G.tup(case["kaxes"]), G.tup(case["vaxes"]), size=size)
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    want = G.arr(case, "out_sorted" if case.get("toarray_unsorted") else "out")
    got = r.toarray()
    assert got.dtype == want.dtype and got.tobytes() == want.tobytes()


@pytest.mark.parametrize("case", G.cases("transpose") + G.cases("transpose_named"), ids=G.case_id)
def test_transpose(case, bctx):
    x, b = _b(case, bctx)
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b.transpose(case["perm"])
        assert type(e.value).__name__ == case["raises"]
        return
    if case["op"] == "transpose":
        r = b.transpose(case["perm"])
    else:
        r = {"T": lambda b: b.T,
             "perm20413": lambda b: b.transpose(2, 0, 4, 1, 3) if b.ndim == 5 else b.transpose(3, 1, 0, 2),
             "swapaxes": lambda b: b.swapaxes(0, b.ndim - 1)}[case["name"]](b)
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    want = G.arr(case, "out_sorted" if case.get("toarray_unsorted") else "out")
    assert r.toarray().tobytes() == want.tobytes()


def _chunk_check(c, case):
    recs = list(c.records())
    assert [list(k) for k, _ in recs] == case["keys"]
    assert [list(v.shape) for _, v in recs] == case["shapes"]
    flat = np.concatenate([v.reshape(-1) for _, v in recs])
    assert flat.tobytes() == G.arr(case, "flat").tobytes()
    assert [int(p) for p in c.plan] == case["plan"]
    assert [int(p) for p in c.padding] == case["padding_out"]


@pytest.mark.parametrize("case", G.cases("chunk"), ids=G.case_id)
def test_chunk(case, bctx):
    x, b = _b(case, bctx)
    size = case["size"]
    size = size if isinstance(size, (str, int)) else tuple(size)
    pad = G.tup(case["padding"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b.chunk(size, axis=G.tup(case["chunk_axis"]), padding=pad)
        assert type(e.value).__name__ == case["raises"]
        return
    c = b.chunk(size, axis=G.tup(case["chunk_axis"]), padding=pad)
    assert list(c.shape) == case["chunk_shape"] and c.split == case["split"]
    assert bool(c.uniform) == case["uniform"]
    _chunk_check(c, case)
    u = c.unchunk()
    assert list(u.shape) == case["unchunk_shape"] and u.split == case["unchunk_split"]
    if "unchunk_raises" in case:
        # the reference's removepad over-trims clipped chunks when 0 < d % s < p and its
        # toarray raises; bolt_amd strips exactly the padding getslices added
        assert u.toarray().tobytes() == x.tobytes()
        return
    assert u.toarray().tobytes() == G.arr(case, "unchunk").tobytes()


@pytest.mark.parametrize("case", G.cases("moves"), ids=G.case_id)
def test_moves(case, bctx):
    x, b = _b(case, bctx)
    size = case["size"]
    size = size if isinstance(size, (str, int)) or size is None else tuple(size)
    c = b.chunk(size, padding=G.tup(case["padding"]))

    def apply(c):
        for name, axes, z in case["steps"]:
            c = c.keys_to_values(tuple(axes), size=G.tup(z)) if name == "k2v" else c.values_to_keys(tuple(axes))
        return c
    if "raises" in case:
        # reference failure: values_to_keys down to all keys then
        # keys_to_values; bolt_amd completes it -- the chunking must still round trip
        c = apply(c)
        assert c.unchunk().toarray().size == x.size
        return
    c = apply(c)
    assert list(c.shape) == case["chunk_shape"] and c.split == case["split"]
    _chunk_check(c, case)
    u = c.unchunk()
    assert list(u.shape) == case["unchunk_shape"] and u.split == case["unchunk_split"]
    assert u.toarray().tobytes() == G.arr(case, "unchunk").tobytes()


@pytest.mark.parametrize("case", G.cases("getplan"), ids=G.case_id)
def test_getplan(case):
    plan, pad = getplan(case["vshape"], case["dtype"], case["size"])
    assert [int(p) for p in plan] == case["plan"]


@pytest.mark.parametrize("case", G.cases("stat"), ids=G.case_id)
def test_stat(case, bctx):
    x = G.make_input(case["input"])
    b = bolt.array(x, bctx, axis=G.tup(case["axis"]), npartitions=case["npartitions"])
    ax = G.tup(case["reduce_axis"])
    f = getattr(b, case["name"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            f(axis=ax, keepdims=case["keepdims"])
        assert type(e.value).__name__ == case["raises"]
        return
    got = f(axis=ax, keepdims=case["keepdims"])
    want = G.arr(case, "out")
    assert type(got).__name__ == case["result_type"]
    assert str(np.asarray(got).dtype) == case["result_dtype"]
    assert np.asarray(got).shape == want.shape
    if want.dtype.kind in 'iub' or case["name"] in ("min", "max"):
        assert np.asarray(got).tobytes() == want.tobytes()
    else:
        truth = G.truth_stat(x, case["name"], ax)
        assert G.stat_close(got, want, truth, want.dtype, x, case["name"])


@pytest.mark.parametrize("case", G.cases("getitem"), ids=G.case_id)
def test_getitem(case, bctx):
    x, b = _b(case, bctx, case["npartitions"])
    idx = G.index_arg(case["index"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b[idx]
        assert type(e.value).__name__ == case["raises"]
        return
    if "collect_raises" in case:
        # the reference builds an array it cannot collect; this backend refuses the index
        with pytest.raises(ValueError):
            b[idx].toarray()
        return
    r = b[idx]
    want = G.arr(case, "out_sorted" if case.get("toarray_unsorted") else "out")
    if case["kind"] == "scalar":
        assert type(r).__name__ == case["result_type"]
        assert np.asarray(r).tobytes() == want.tobytes()
        return
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    got = r.toarray()
    assert got.dtype == want.dtype and got.tobytes() == want.tobytes()


@pytest.mark.parametrize("case", G.cases("squeeze"), ids=G.case_id)
def test_squeeze(case, bctx):
    x, b = _b(case, bctx)
    q = G.tup(case["squeeze"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b.squeeze(q)
        assert type(e.value).__name__ == case["raises"]
        return
    r = b.squeeze(q)
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert r.toarray().tobytes() == G.arr(case, "out").tobytes()


def _other(case, bctx):
    y = G.make_input(case["other"]) if case["other"] else [[1, 2, 3]]
    kind = case["other_kind"]
    if kind == "local":
        return bolt.array(y)
    if kind == "spark":
        return bolt.array(y, bctx, axis=G.tup(case["other_axis"]), npartitions=case["npartitions"])
    return y


@pytest.mark.parametrize("case", G.cases("concatenate"), ids=G.case_id)
def test_concatenate(case, bctx):
    x, b = _b(case, bctx, case["npartitions"])
    other = _other(case, bctx)
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b.concatenate(other, axis=case["cat_axis"])
        assert type(e.value).__name__ == case["raises"]
        return
    r = b.concatenate(other, axis=case["cat_axis"])
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert r.toarray().tobytes() == G.arr(case, "out").tobytes()


def _close(got, want, exact):
    if exact:
        return got.dtype == want.dtype and got.tobytes() == want.tobytes()
    rtol = 1e-6 if want.dtype == np.float32 else 1e-12
    scale = float(np.max(np.abs(want))) if want.size else 0.0
    return got.dtype == want.dtype and np.allclose(got, want, rtol=rtol, atol=rtol * scale)


@pytest.mark.parametrize("case", G.cases("chunk_map"), ids=G.case_id)
def test_chunk_map(case, bctx):
    from funcs import FUNCS, EXACT
    x, b = _b(case, bctx)
    c = b.chunk(size=G.size_arg(case["size"]), padding=G.tup(case["padding"]))
    f = FUNCS[case["func"]]
    vs = G.tup(case["value_shape"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            c.map(f, value_shape=vs)
        assert type(e.value).__name__ == case["raises"]
        return
    r = c.map(f, value_shape=vs)
    assert list(r.shape) == case["shape"] and list(r.plan) == case["plan"]
    assert _close(r.unchunk().toarray(), G.arr(case, "out"), case["func"] in EXACT)


@pytest.mark.parametrize("case", G.cases("chunk_map_generic"), ids=G.case_id)
def test_chunk_map_generic(case, bctx):
    x, b = _b(case, bctx)
    c = b.chunk(size=G.size_arg(case["size"]))
    d = c.map_generic(lambda v: [int(v.sum()), list(v.shape)])
    assert list(d.shape) == case["shape"]
    assert [list(o) for o in np.asarray(d).reshape(-1)] == case["objects"]


@pytest.mark.parametrize("case", G.cases("stack"), ids=G.case_id)
def test_stack(case, bctx):
    x, b = _b(case, bctx, case["npartitions"])
    st = b.stack(case["size"])
    recs = st.tordd().collect()
    assert [list(v.shape) for _, v in recs] == case["stack_shapes"]
    assert [[list(k) for k in ks] for ks, _ in recs] == case["stack_keys"]
    assert list(st.shape) == case["shape"] and st.split == case["split"]
    assert st.unstack().toarray().tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("stack_map"), ids=G.case_id)
def test_stack_map(case, bctx):
    from funcs import FUNCS, EXACT
    x, b = _b(case, bctx, case["npartitions"])

    def go():
        st = b.stack(case["size"])
        for name in case["funcs"]:
            st = st.map(FUNCS[name])
        return st.unstack()
    if "raises" in case:
        with pytest.raises(Exception) as e:
            go()
        assert type(e.value).__name__ == case["raises"]
        return
    r = go()
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert _close(r.toarray(), G.arr(case, "out"), all(f in EXACT for f in case["funcs"]))


@pytest.mark.parametrize("case", G.cases("map"), ids=G.case_id)
def test_map(case, bctx):
    from funcs import FUNCS, EXACT
    x, b = _b(case, bctx, case["npartitions"])
    r = b.map(FUNCS[case["func"]], axis=G.tup(case["map_axis"]), value_shape=G.tup(case["value_shape"]),
              dtype=case["dtype"], with_keys=case["with_keys"])
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert _close(r.toarray(), G.arr(case, "out"), case["func"] in EXACT)


@pytest.mark.parametrize("case", G.cases("filter"), ids=G.case_id)
def test_filter(case, bctx):
    from funcs import FUNCS
    x, b = _b(case, bctx, case["npartitions"])
    r = b.filter(FUNCS[case["func"]], axis=G.tup(case["filter_axis"]), sort=case["sort"])
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    if case["shape"] != [0]:
        assert r.toarray().tobytes() == G.arr(case, "out").tobytes()


@pytest.mark.parametrize("case", G.cases("reduce"), ids=G.case_id)
def test_reduce(case, bctx):
    from funcs import RFUNCS
    x, b = _b(case, bctx, case["npartitions"])
    ax = tuple(case["reduce_axis"])
    f = RFUNCS[case["func"]]
    if "raises" in case:
        with pytest.raises(Exception) as e:
            b.reduce(f, axis=ax, keepdims=case["keepdims"])
        assert type(e.value).__name__ == case["raises"]
        return
    got = b.reduce(f, axis=ax, keepdims=case["keepdims"])
    assert type(got).__name__ == case["result_type"]
    a = np.asarray(got.toarray() if hasattr(got, "toarray") else got)
    assert str(a.dtype) == case["result_dtype"]
    assert G.reduce_close(a, G.arr(case, "out"), x, case["func"], ax)


@pytest.mark.parametrize("case", G.cases("reshape"), ids=G.case_id)
def test_reshape(case, bctx):
    x, b = _b(case, bctx, case["npartitions"])
    shp = getattr(b, case["which"])
    new = tuple(case["new"])
    if "raises" in case:
        with pytest.raises(Exception) as e:
            shp.reshape(new)
        assert type(e.value).__name__ == case["raises"]
        return
    r = shp.reshape(*new) if case.get("varargs") else shp.reshape(new)
    assert list(r.shape) == case["shape"] and r.split == case["split"]
    assert r.toarray().tobytes() == G.arr(case, "out").tobytes()
