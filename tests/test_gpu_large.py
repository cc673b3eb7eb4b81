"""Parity at the BASELINE.json sizes (GPU only), bit for bit and in full.

The oracle cannot run at 2-69 GB, so every output is compared, byte for byte
and over its WHOLE extent, with an independent reference built on the same
device by torch from the same input bytes:
  * swap / transpose: ``x.permute(perm).contiguous()`` (viewed as integers,
    so NaN payloads compare bitwise);
  * chunk / keys_to_values / values_to_keys: the packed chunk layout rebuilt
    with torch slicing from the reference's own slice rule
    (chunk.py:574-618: chunk j of an axis is [j s - (j>0) p, j s + s + p)
    clipped; records hold their chunks back to back in chunk-id order, each a
    dense box), independent of plan.ChunkGeometry and the record-map kernels;
  * statistics agree with float64 sums taken with torch on the device within
    the stated tolerance.
Configs: C2 swap, C3 swap and .T, C4 uint16 swap / .T / chunk('150'), C5 .T,
transpose(2,0,4,1,3) and chunk((16,16), padding=2) with its k2v / v2k, the
64 GiB target swap.  Inputs are generated in HBM; every test frees its
buffers (the target's working set -- input, swap, reference -- is 206 GB).
"""
import gc

import numpy as np
import pytest

import bolt_amd as bolt

pytestmark = pytest.mark.gpu

_INT = {1: "uint8", 2: "int16", 4: "int32", 8: "int64"}


@pytest.fixture(autouse=True)
def _free():
    yield
    import torch
    gc.collect()
    torch.cuda.empty_cache()


def _shard(ctx, shape, dtype, split, seed):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    raw = torch.randint(-128, 127, (n,), generator=g, device="cuda", dtype=torch.int8).view(torch.uint8)
    if np.dtype(dtype) == np.float32:
        raw = (torch.randn(n // 4, generator=g, device="cuda") * 50 + 1000).view(torch.uint8)
    return bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=split, dtype=dtype), raw


def _ints(buf, es):
    import torch
    return buf.view(getattr(torch, _INT[es]))


def _full_check(raw, shape, dtype, out, perm):
    """out = x.transpose(perm), every element, against torch's permute."""
    import torch
    es = np.dtype(dtype).itemsize
    want = _ints(raw, es).reshape(shape).permute(*perm).contiguous().reshape(-1)
    assert out._data.numel() == want.numel() * es
    assert torch.equal(_ints(out._data, es), want)
    del want


def _clear():
    import torch
    gc.collect()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg", [
    ("C2", (2000, 512, 512), np.float32, 1, ((0,), (0, 1))),
    ("C3", (4096, 256, 256, 32), np.float32, 2, ((0,), (0,))),
    ("C4", (10000, 1024, 1024), np.uint16, 1, ((0,), (0,))),
    ("C5", (64, 64, 64, 64, 64), np.float64, 3, ((0, 2), (1,))),
], ids=lambda c: c[0])
def test_swap_full_size(gpu_ctx, cfg):
    import torch
    name, shape, dtype, split, (kax, vax) = cfg
    b, raw = _shard(gpu_ctx, shape, dtype, split, 7)
    s = b.swap(kax, vax)
    from bolt_amd.mi355x.plan import swap_perm
    perm, nsplit = swap_perm(len(shape), split, kax, vax)
    inv = list(np.argsort(perm))
    if name == "C2":
        # padded rows (8192-B pitch), transposed back straight from the padding
        assert "_pbuf" in s.__dict__
        back = s.transpose(inv)
        assert "_pbuf" in s.__dict__
        assert torch.equal(back._data, b._data)
        del back
    assert s.shape == tuple(shape[p] for p in perm) and s.split == nsplit
    _full_check(raw, shape, dtype, s, perm)
    # undo the swap with the inverse permutation: bit-exact identity
    back = s.transpose(inv)
    assert torch.equal(back._data, b._data)
    del s, back


@pytest.mark.parametrize("cfg", [
    ((4096, 256, 256, 32), np.float32, 2, (3, 2, 1, 0)),        # C3 .T
    ((64,) * 5, np.float64, 3, (4, 3, 2, 1, 0)),                # C5 .T
    ((64,) * 5, np.float64, 3, (2, 0, 4, 1, 3)),                # C5 transpose(2,0,4,1,3)
    ((10000, 1024, 1024), np.uint16, 1, (2, 1, 0)),             # C4 .T: packed-word tiles
    ((2000, 1024, 2048), np.uint8, 1, (2, 1, 0)),               # uint8 .T
], ids=["C3_T", "C5_T", "C5_20413", "C4_T", "u8_T"])
def test_transpose_full_size(gpu_ctx, cfg):
    import torch
    shape, dtype, split, perm = cfg
    b, raw = _shard(gpu_ctx, shape, dtype, split, 3)
    t = b.transpose(perm)
    _full_check(raw, shape, dtype, t, perm)
    back = t.transpose(list(np.argsort(perm)))
    assert torch.equal(back._data, b._data)
    del b, raw, t, back


def _axis_slices(d, s, p):
    """getslices (chunk.py:574-618) for one axis: [j s - (j>0) p, j s + s + p) clipped."""
    out, j = [], 0
    while j * s < d:
        out.append(slice(max(0, j * s - (p if j else 0)), min(d, j * s + s + p)))
        j += 1
    return out


def _packed_ref(rec, vshape, plan, pad):
    """(records, *vshape) device tensor -> its packed chunk layout, by torch slicing."""
    import torch
    from itertools import product
    sl = [_axis_slices(vshape[a], plan[a], pad[a]) for a in range(len(vshape))]
    parts = [rec[(slice(None),) + tuple(c)].reshape(rec.shape[0], -1) for c in product(*sl)]
    return torch.cat(parts, dim=1).reshape(-1)


def test_chunk_c4_full_size(gpu_ctx):
    import torch
    b, raw = _shard(gpu_ctx, (10000, 1024, 1024), np.uint16, 1, 11)   # C4, size '150'
    c = b.chunk("150")
    assert tuple(c.plan) == (73, 1024) and tuple(c.padding) == (0, 0)
    want = _packed_ref(_ints(raw, 2).reshape(10000, 1024, 1024), (1024, 1024), (73, 1024), (0, 0))
    assert torch.equal(_ints(c._packed, 2), want)
    del want
    assert torch.equal(c.unchunk()._data, b._data)


def test_chunk_c5_full_size(gpu_ctx):
    import torch
    b, raw = _shard(gpu_ctx, (64,) * 5, np.float64, 3, 12)            # C5, padded
    x = _ints(raw, 8).reshape((64,) * 5)
    c = b.chunk((16, 16), padding=2)
    want = _packed_ref(x.reshape(64 ** 3, 64, 64), (64, 64), (16, 16), (2, 2))
    assert torch.equal(_ints(c._packed, 8), want)
    del want
    assert torch.equal(c.unchunk()._data, b._data)
    # keys_to_values((2,)): keys (k0, k1), values (k2, v0, v1), plan (64, 16, 16), padding (0, 2, 2)
    k = c.keys_to_values((2,))
    assert tuple(k.plan) == (64, 16, 16) and tuple(k.padding) == (0, 2, 2)
    want = _packed_ref(x.reshape(64 * 64, 64, 64, 64), (64, 64, 64), (64, 16, 16), (0, 2, 2))
    assert torch.equal(_ints(k._packed, 8), want)
    del want, k
    _clear()
    # values_to_keys((0,)): keys (k0, k1, k2, v0), values (v1,), plan (16,), padding (2,)
    v = c.values_to_keys((0,))
    assert tuple(v.plan) == (16,) and tuple(v.padding) == (2,)
    want = _packed_ref(x.reshape(64 ** 4, 64), (64,), (16,), (2,))
    assert torch.equal(_ints(v._packed, 8), want)
    del want
    assert torch.equal(v.unchunk()._data, b.swap((), (0,))._data)


def test_target64_swap_full_size(gpu_ctx):
    """The 64 GiB north_star array: float32 (8192, 256, 256, 32), split 2, swap((0,), (0,))."""
    shape = (8192, 256, 256, 32)
    b, raw = _shard(gpu_ctx, shape, np.float32, 2, 21)
    s = b.swap((0,), (0,))
    assert s.shape == (256, 256, 8192, 32) and s.split == 2
    _full_check(raw, shape, np.float32, s, (1, 2, 0, 3))


def test_stats_full_size_c2(gpu_ctx):
    import torch
    b, raw = _shard(gpu_ctx, (2000, 512, 512), np.float32, 1, 5)
    s = b.swap((0,), (0, 1))
    assert "_pbuf" in s.__dict__ and s._pitch == 2048  # 8000-B rows stored at an 8192-B pitch
    m, sd = s.mean(axis=2), s.std(axis=2)
    assert "_pbuf" in s.__dict__  # read in place (bm_reduce_rows)
    d = b.swap((0,), (0, 1))
    d._compact()
    assert d.mean(axis=2).tobytes() == m.tobytes() and d.std(axis=2).tobytes() == sd.tobytes()
    # the leading axis of the padded result: column kernels over the padded rows
    v0 = s.var(axis=0)
    assert "_pbuf" in s.__dict__
    assert np.allclose(v0, d.var(axis=0), rtol=1e-6, atol=0)  # (another column count: maybe another chunking)
    ref0 = raw.view(torch.float32).reshape(2000, 512, 512).double().var(dim=1, unbiased=False).t().cpu().numpy()
    assert v0.shape == (512, 2000) and np.all(np.abs(v0 - ref0) <= 1e-6 * ref0 + np.spacing(np.float32(ref0)))
    del d, ref0
    x = raw.view(torch.float32).reshape(2000, 512 * 512).double()
    mu = x.mean(0)
    var = ((x - mu) ** 2).mean(0)
    mref = mu.cpu().numpy().reshape(512, 512)
    sref = var.sqrt().cpu().numpy().reshape(512, 512)
    assert m.dtype == np.float32 and sd.dtype == np.float32
    # rtol 1e-6 on float32 results (+1 ulp of the float32 rounding of the result)
    assert np.all(np.abs(m - mref) <= 1e-6 * np.abs(mref) + np.spacing(np.float32(np.abs(mref))))
    assert np.all(np.abs(sd - sref) <= 1e-6 * np.abs(sref) + np.spacing(np.float32(np.abs(sref))))
    v = b.var(axis=0)
    vref = var.cpu().numpy().reshape(512, 512)
    # the var-scaled rule: rtol 1e-6 of the variance itself + the float32 rounding of the result
    assert v.dtype == np.float32
    assert np.all(np.abs(v - vref) <= 1e-6 * vref + np.spacing(np.float32(vref)))
    tot = b.sum()
    assert abs(float(tot) - float(x.sum())) <= 1e-6 * abs(float(x.sum()))
    # every axis of the padded result: per-column states over the padded rows
    # merged on the host, no dense copy; against the float64 truth and the
    # dense layout's answer (rtol 1e-6 + the float32 rounding)
    n = x.numel()
    t_mean = float(x.sum()) / n
    t_var = float(((x - t_mean) ** 2).sum()) / n
    d = b.swap((0,), (0, 1))
    d._compact()
    for name, truth in (("mean", t_mean), ("var", t_var), ("std", t_var ** 0.5)):
        got = getattr(s, name)()
        assert "_pbuf" in s.__dict__ and "_data" not in s.__dict__, name
        bar = 1e-6 * abs(truth) + float(np.spacing(np.float32(abs(truth))))
        assert np.float32(got).dtype == np.float32 and abs(float(got) - truth) <= bar, (name, got, truth)
        assert abs(float(got) - float(getattr(d, name)())) <= bar, name


def test_stats_full_size_c4_var(gpu_ctx):
    """C4 var(axis=0) and sum(axis=0) on ALL 1,048,576 outputs.  The reference
    values are exact: S1 = sum x and S2 = sum x^2 in int64 on the device (x < 2^16,
    n = 10,000: n*S2 and S1^2 < 2^59), var = (n*S2 - S1^2) / n^2 formed in
    exact integers; the kernel's result (2 ulp of the exact rational) must be
    within 3 ulp of this reference (its own rounding adds < 1 ulp), far inside
    the north_star's 1e-12.  sum keeps uint16 (mod 2^16),
    as the reference's treeReduce(add) in the record dtype does."""
    import torch
    b, raw = _shard(gpu_ctx, (10000, 1024, 1024), np.uint16, 1, 9)
    v = b.var(axis=0)
    s = np.asarray(b.sum(axis=0)).reshape(-1)
    assert v.dtype == np.float64 and s.dtype == np.uint16
    v = v.reshape(-1)
    x = raw.view(torch.int16).reshape(10000, 1024 * 1024)
    n = x.shape[0]
    step = 1 << 16
    for lo in range(0, x.shape[1], step):
        xs = x[:, lo:lo + step].to(torch.int64) & 0xFFFF
        s1 = xs.sum(0)
        s2 = (xs * xs).sum(0)
        del xs
        num = n * s2 - s1 * s1                       # exact: < 2^59
        # num / n^2 rounded once: split num = q*n^2 + r exactly, then q + r/n^2
        q, r = torch.div(num, n * n, rounding_mode="floor"), torch.remainder(num, n * n)
        exact = q.double() + r.double() / float(n * n)
        got = torch.from_numpy(np.ascontiguousarray(v[lo:lo + step])).to(x.device)
        ulp = torch.abs(exact) * 2.0 ** -52
        assert bool(torch.all(torch.abs(got - exact) <= 3 * ulp + 1e-300)), lo
        want_s = (s1 & 0xFFFF).cpu().numpy().astype(np.uint16)
        assert np.array_equal(s[lo:lo + step], want_s), lo


def test_getitem_full_size_c2(gpu_ctx):
    """Indexing at the C2 size against torch index_select on the same bytes
    (an independent device reference): reversed / strided slices, an int,
    a list on the value and on the key axis, and a 1M-point advanced gather."""
    import torch
    shape = (2000, 512, 512)
    b, raw = _shard(gpu_ctx, shape, np.float32, 1, 13)
    x = raw.view(torch.float32).reshape(shape)

    def sel(t, axis, idx):
        return torch.index_select(t, axis, torch.as_tensor(np.asarray(idx), device="cuda"))

    r = b[1999:0:-7, 100:400:3, 511:-513:-1]  # (::-1 is an empty-dimension error in bolt)
    want = sel(sel(sel(x, 0, np.arange(1999, 0, -7)), 1, np.arange(100, 400, 3)), 2, np.arange(511, -1, -1))
    assert r.shape == tuple(want.shape) and torch.equal(r._data.view(torch.float32).reshape(want.shape), want)
    r = b[:, 7]
    assert r.shape == (2000, 512) and torch.equal(r._data.view(torch.float32).reshape(2000, 512), x[:, 7])
    idx = [511, 0, 7, 300, 299]
    r = b[:, :, idx]
    assert torch.equal(r._data.view(torch.float32).reshape(2000, 512, 5), sel(x, 2, idx))
    kidx = list(range(1999, -1, -3))
    r = b[kidx]
    assert torch.equal(r._data.view(torch.float32).reshape(len(kidx), 512, 512), sel(x, 0, kidx))
    rng = np.random.default_rng(3)
    pts = [np.sort(rng.integers(0, 2000, 1 << 20))] + [rng.integers(0, d, 1 << 20) for d in shape[1:]]
    r = b[tuple(pts)]
    lin = torch.as_tensor(np.ravel_multi_index(pts, shape), device="cuda")
    # sorted keys: the reference's record order is the listed order only within a key's run
    assert r.shape == (1 << 20,) and r.split == 1
    assert torch.equal(r._data.view(torch.float32), x.reshape(-1)[lin])


def test_c1_step_against_oracle(gpu_ctx):
    """BASELINE C1 (the reference's CPU-runnable case), the whole bench step:
    float64 (100,64,64) N(0,1) (seed 0, as SURVEY 8(d)), swap((0,),(0,)), then
    sum / mean / var / std at axis=None and axis=(0,) of the swapped array,
    against the oracle's record-level restatement of the Spark path (8
    partitions): the swap bit for bit, the statistics by the stat_close rule
    (rtol 1e-12 for float64)."""
    import golden_cases as G
    from oracle import bolt_oracle as O
    x = np.random.default_rng(0).standard_normal((100, 64, 64))
    b = bolt.array(x, gpu_ctx, axis=(0,))
    s = b.swap((0,), (0,))
    rs = O.swap(O.parallelize(x, axis=(0,), npartitions=8), (0,), (0,))
    assert s.shape == (64, 100, 64) and s.split == 1
    assert s.toarray().tobytes() == O.toarray(rs).tobytes()
    y = x.transpose(1, 0, 2)
    for name in ("sum", "mean", "var", "std"):
        for ax in (None, (0,)):
            got = getattr(s, name)(axis=ax)
            if name == "sum":
                want = O.sum_(rs, ax)
            else:
                want = O.stat(rs, {"var": "variance", "std": "stdev"}.get(name, name), ax)
            truth = G.truth_stat(y, name, ax)
            assert np.asarray(got).dtype == np.asarray(want).dtype, (name, ax)
            assert G.stat_close(got, want, truth, np.float64, y, name), (name, ax)
