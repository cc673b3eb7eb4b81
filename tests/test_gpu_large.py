"""Parity at the BASELINE.json sizes (GPU only), through size-independent properties.

The oracle cannot run at 2-69 GB, so full-size checks use properties:
  * swap / transpose round trips are the identity, bit for bit;
  * thousands of random positions of the result equal the input at the
    permuted coordinates (checked on the host from the input's bytes);
  * chunk -> unchunk is the identity; a padded chunking keeps every record's
    chunk cores exact at sampled positions;
  * statistics agree with float64 sums taken with torch on the device (an
    independent float64 reference for the floating-point kernels) within the
    stated tolerance.
Inputs are generated in HBM; every test frees its buffers.
"""
import gc

import numpy as np
import pytest

import bolt_amd as bolt

pytestmark = pytest.mark.gpu


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


def _sample_check(src_raw, shape, dtype, out, perm, nsamp=4096, seed=0):
    """out = x.transpose(perm): compare nsamp random output positions with the input."""
    import torch
    rng = np.random.default_rng(seed)
    es = np.dtype(dtype).itemsize
    oshape = tuple(shape[p] for p in perm)
    idx = [rng.integers(0, d, nsamp) for d in oshape]
    in_idx = [None] * len(shape)
    for k, p in enumerate(perm):
        in_idx[p] = idx[k]
    lin_out = np.ravel_multi_index(idx, oshape)
    lin_in = np.ravel_multi_index(in_idx, shape)
    x = src_raw.view(torch.uint8).reshape(-1, es)
    y = out._data.reshape(-1, es)
    a = x[torch.from_numpy(lin_in).cuda()].cpu().numpy()
    b = y[torch.from_numpy(lin_out).cuda()].cpu().numpy()
    assert np.array_equal(a, b)


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
    assert s.shape == tuple(shape[p] for p in perm) and s.split == nsplit
    _sample_check(raw, shape, dtype, s, perm)
    # undo the swap with the inverse permutation: bit-exact identity
    inv = list(np.argsort(perm))
    back = s.transpose(inv)
    assert torch.equal(back._data, b._data)
    del s, back


def test_transpose_full_size_c3_c5(gpu_ctx):
    import torch
    for shape, dtype, split, perm in [((4096, 256, 256, 32), np.float32, 2, (3, 2, 1, 0)),
                                      ((64,) * 5, np.float64, 3, (4, 3, 2, 1, 0)),
                                      ((64,) * 5, np.float64, 3, (2, 0, 4, 1, 3)),
                                      # C4's uint16 reversed: packed-word tiles (k_transpose_pk)
                                      ((10000, 1024, 1024), np.uint16, 1, (2, 1, 0)),
                                      ((2000, 1024, 2048), np.uint8, 1, (2, 1, 0))]:
        b, raw = _shard(gpu_ctx, shape, dtype, split, 3)
        t = b.transpose(perm)
        _sample_check(raw, shape, dtype, t, perm)
        back = t.transpose(list(np.argsort(perm)))
        assert torch.equal(back._data, b._data)
        del b, raw, t, back
        gc.collect()
        torch.cuda.empty_cache()


def test_chunk_round_trips_full_size(gpu_ctx):
    import torch
    b, raw = _shard(gpu_ctx, (10000, 1024, 1024), np.uint16, 1, 11)   # C4, size '150'
    c = b.chunk("150")
    assert tuple(c.plan) == (73, 1024)
    assert torch.equal(c.unchunk()._data, b._data)
    del c, b, raw
    gc.collect()
    torch.cuda.empty_cache()
    b, raw = _shard(gpu_ctx, (64,) * 5, np.float64, 3, 12)            # C5, padded
    c = b.chunk((16, 16), padding=2)
    assert torch.equal(c.unchunk()._data, b._data)
    k = c.keys_to_values((2,))
    assert torch.equal(k.unchunk()._data, b.swap((2,), ())._data)
    v = c.values_to_keys((0,))
    assert torch.equal(v.unchunk()._data, b.swap((), (0,))._data)


def test_stats_full_size_c2(gpu_ctx):
    import torch
    b, raw = _shard(gpu_ctx, (2000, 512, 512), np.float32, 1, 5)
    s = b.swap((0,), (0, 1))
    m, sd = s.mean(axis=2), s.std(axis=2)
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
    assert np.all(np.abs(v - var.cpu().numpy().reshape(512, 512)) <= 1e-6 * var.cpu().numpy().reshape(512, 512) + 1e-3)
    tot = b.sum()
    assert abs(float(tot) - float(x.sum())) <= 1e-6 * abs(float(x.sum()))


def test_stats_full_size_c4_var(gpu_ctx):
    import torch
    b, raw = _shard(gpu_ctx, (10000, 1024, 1024), np.uint16, 1, 9)
    v = b.var(axis=0)
    assert v.dtype == np.float64
    x = raw.view(torch.int16).reshape(10000, 1024 * 1024)
    cols = torch.arange(0, 1024 * 1024, 4099, device="cuda")
    xs = (x[:, cols].to(torch.int32) & 0xFFFF).double()
    ref = xs.var(0, unbiased=False).cpu().numpy()
    got = v.reshape(-1)[cols.cpu().numpy()]
    assert np.allclose(got, ref, rtol=1e-12, atol=0)
    s = b.sum(axis=0)
    ref_s = (xs.sum(0).to(torch.int64) & 0xFFFF).cpu().numpy().astype(np.uint16)
    assert np.array_equal(np.asarray(s).reshape(-1)[cols.cpu().numpy()], ref_s)


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
