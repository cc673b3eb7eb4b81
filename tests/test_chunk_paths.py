"""Chunk pack / unpack: the record-map gather (bm_record_gather, small records)
against the strided-copy path (one bm_copy_strided per run of equal chunks)
and against the reference's chunk slicing restated with numpy
(getslices + removepad, bolt/spark/chunk.py:87-144, :514-618).

Runs on the CPU test executor and (marker `gpu`) through the C ABI on the
GPU.  Bit-exact: packed bytes of both paths are identical, every chunk equals
the reference's padded slice, and unchunk restores the input.
"""
import numpy as np
import pytest

import bolt_amd as bolt
from bolt_amd.mi355x import chunk as chunk_mod
from bolt_amd.mi355x.plan import getslices

CASES = [
    # (shape, split, dtype, size, padding)
    ((6, 64, 64), 1, np.float64, (16, 16), 2),      # C5's record geometry
    ((5, 20, 30), 1, np.float32, (7, 9), (1, 3)),   # ragged + asymmetric halos
    ((4, 3, 33, 17), 2, np.uint8, (5, 4), 2),       # 1-byte elements, odd record size
    ((7, 50, 11), 1, np.uint16, (8, 11), (3, 0)),   # an unchunked axis
    ((3, 2, 9, 8, 10), 2, np.int32, (4, 3, 5), 1),  # 3 value axes
    ((9, 100), 1, np.float64, (10,), 4),            # 1 value axis
    ((2, 128, 64), 1, np.float32, (128, 64), 0),    # one chunk: plan = vshape
    ((3, 4, 4), 1, np.complex128, (2, 2), 1),       # 16-B elements: strided path only
    ((2, 128, 100), 1, np.float32, (32, 25), 1),    # 51 KiB records: staged in parts (GPU)
    ((3, 3, 90, 60), 2, np.float64, (16, 16), 2),   # 43 KiB records, ragged chunks, parts
]


def _rand(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    n = int(np.prod(shape)) * np.dtype(dtype).itemsize
    return rng.integers(0, 256, size=n, dtype=np.uint8).view(dtype).reshape(shape)


def _expected_chunks(x, split, plan, padding):
    """(key + chunk id, padded chunk) in key order, as chunk.py:131-142 emits them."""
    from itertools import product
    vshape = x.shape[split:]
    slices = getslices(plan, padding, vshape)
    out = []
    for key in np.ndindex(*x.shape[:split]):
        v = x[key]
        for cid in product(*[range(len(s)) for s in slices]):
            out.append((tuple(key) + cid, v[tuple(s[i] for s, i in zip(slices, cid))]))
    return out


@pytest.mark.parametrize("case", range(len(CASES)))
def test_record_map_matches_strided_copies(bctx, case, monkeypatch):
    shape, split, dtype, size, padding = CASES[case]
    x = _rand(shape, dtype, case)
    b = bolt.array(x, bctx, axis=tuple(range(split)))
    packs = {}
    for use_map in (True, False):
        monkeypatch.setitem(chunk_mod.PATHS, "record_map", use_map)
        c = b.chunk(size, padding=padding)
        packs[use_map] = c
        assert np.asarray(c.unchunk().toarray()).tobytes() == x.tobytes()
    a, s = packs[True], packs[False]
    assert bytes(a._packed.cpu().numpy()) == bytes(s._packed.cpu().numpy())
    want = _expected_chunks(x, split, tuple(int(p) for p in a.plan), tuple(int(p) for p in a.padding))
    got = list(a.records())
    assert len(got) == len(want)
    for (gk, gv), (wk, wv) in zip(got, want):
        assert gk == wk and gv.shape == wv.shape and gv.tobytes() == np.ascontiguousarray(wv).tobytes()


def test_record_map_threshold():
    assert chunk_mod._use_record_map(8192, 8)          # 64 KiB: staged in LDS
    assert not chunk_mod._use_record_map(8193, 8)      # larger: strided copies
    assert not chunk_mod._use_record_map(4, 16)        # 16-B elements: strided copies


def test_record_map_inverse():
    from bolt_amd.mi355x.plan import ChunkGeometry
    g = ChunkGeometry((20, 30), (7, 9), (1, 3))
    pm, um = g.record_map(unpack=False), g.record_map(unpack=True)
    assert pm.size == g.size and um.size == 600
    # unpack reads, for each dense cell, a packed cell that pack filled from that same dense cell
    assert np.array_equal(pm[um], np.arange(600))


RECHUNK = [
    # (shape, split, chunk size, padding, op, axes, k2v size)
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "k2v", (2,), None),        # trailing key
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "k2v", (0,), None),        # leading key
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "k2v", (0, 2), None),      # two keys, not adjacent
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "k2v", (1,), (2,)),        # ragged key chunks (5 = 2+2+1)
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "k2v", (0, 1, 2), (3, 2, 4)),
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "v2k", (0,), None),
    ((4, 5, 6, 20, 30), 3, (7, 9), (1, 3), "v2k", (1,), None),
    ((3, 9, 8, 10), 1, (4, 3, 5), (1, 1, 2), "v2k", (0, 2), None),
    ((3, 9, 8, 10), 1, (4, 3, 5), (1, 1, 2), "k2v", (0,), None),
    ((2, 3, 70, 300), 2, (16, 64), (2, 5), "v2k", (0,), None),       # old record > 64 KiB: strided copies
    ((2, 3, 70, 300), 2, (16, 64), (2, 5), "v2k", (1,), None),
]


@pytest.mark.parametrize("case", range(len(RECHUNK)))
@pytest.mark.parametrize("dtype", [np.float64, np.uint8])
def test_fused_rechunk_matches_dense_path(bctx, case, dtype, monkeypatch):
    """keys_to_values / values_to_keys packed -> packed equals unpack -> permute -> pack."""
    shape, split, size, padding, op, axes, ksize = RECHUNK[case]
    x = _rand(shape, dtype, 100 + case)
    b = bolt.array(x, bctx, axis=tuple(range(split)))
    c = b.chunk(size, padding=padding)
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setitem(chunk_mod.PATHS, "fused_rechunk", fused == "1")
        res[fused] = c.keys_to_values(axes, size=ksize) if op == "k2v" else c.values_to_keys(axes)
    f, d = res["1"], res["0"]
    assert f.shape == d.shape and f.split == d.split
    assert np.array_equal(f.plan, d.plan) and np.array_equal(f.padding, d.padding)
    assert bytes(f._packed.cpu().numpy()) == bytes(d._packed.cpu().numpy())
    # and the content is the permuted array
    if op == "k2v":
        ks = [i for i in range(split) if i not in axes] + list(axes)
        perm = ks + list(range(split, len(shape)))
    else:
        vs = [split + a for a in axes] + [split + a for a in range(len(shape) - split) if a not in axes]
        perm = list(range(split)) + vs
    assert np.asarray(f.unchunk().toarray()).tobytes() == np.ascontiguousarray(x.transpose(perm)).tobytes()


def test_identity_geometry_matches_record_map():
    """ChunkGeometry.is_identity() is exactly "the pack map is the identity"
    (every chunk box at its own dense offset, nothing padded), over random
    value shapes, plans and paddings."""
    import itertools
    from bolt_amd.mi355x.plan import ChunkGeometry
    rng = np.random.default_rng(7)
    seen = {True: 0, False: 0}
    for _ in range(400):
        n = int(rng.integers(1, 4))
        vshape = tuple(int(v) for v in rng.integers(1, 7, n))
        plan = tuple(int(rng.integers(1, v + 1)) for v in vshape)
        pad = tuple(int(rng.integers(0, 2)) if rng.random() < 0.3 and p < v else 0
                    for p, v in zip(plan, vshape))
        g = ChunkGeometry(vshape, plan, pad)
        m = g.record_map(unpack=False)
        want = m.size == int(np.prod(vshape)) and np.array_equal(m, np.arange(m.size))
        assert g.is_identity() == want, (vshape, plan, pad)
        seen[want] += 1
    assert seen[True] > 20 and seen[False] > 20
    # C4's default chunk: (73, 1024) on (1024, 1024) records moves nothing
    assert ChunkGeometry((1024, 1024), (73, 1024), (0, 0)).is_identity()
    assert not ChunkGeometry((64, 64), (16, 16), (2, 2)).is_identity()


def test_identity_chunk_shares_bytes(bctx):
    """chunk / unchunk with an identity geometry alias the records' bytes and
    still match the reference semantics (chunk contents, round trip)."""
    x = np.arange(6 * 8 * 5, dtype=np.int16).reshape(6, 8, 5)
    b = bolt.array(x, bctx, axis=(0,))
    c = b.chunk((3, 5))
    assert c._packed.data_ptr() == b._data.data_ptr()
    u = c.unchunk()
    assert u._data.data_ptr() == b._data.data_ptr()
    assert u.toarray().tobytes() == x.tobytes()
    recs = sorted(c.tordd().collect(), key=lambda kv: kv[0])
    assert np.array_equal(recs[0][1], x[0, 0:3, :]) and np.array_equal(recs[1][1], x[0, 3:6, :])
    padded = b.chunk((3, 4), padding=(1, 0))
    assert padded._packed.data_ptr() != b._data.data_ptr()
    assert padded.unchunk().toarray().tobytes() == x.tobytes()


SCATTER_CASES = [
    # (shape, split, dtype, plan, padding): unchunk / k2v of the trailing key /
    # v2k through the record scatter, against the strided-copy / gather paths
    ((3, 4, 12, 10), 2, np.float64, (4, 5), (1, 2)),
    ((2, 5, 9, 8), 2, np.float32, (3, 4), (1, 0)),
    ((4, 3, 16, 16), 2, np.int16, (8, 8), (2, 2)),
    ((2, 3, 7, 6), 2, np.uint8, (7, 3), (0, 1)),
    ((3, 2, 10, 12), 2, np.complex64, (5, 4), (0, 1)),
]


@pytest.mark.parametrize("shape,split,dtype,plan,pad", SCATTER_CASES)
def test_record_scatter_paths_match(bctx, monkeypatch, shape, split, dtype, plan, pad):
    """unchunk, keys_to_values of the trailing key and values_to_keys give the
    same bytes through bm_record_scatter (forced, even where its writes would
    be piecewise) as through the strided copies / record gather."""
    rng = np.random.default_rng(5)
    x = rng.integers(0, 200, size=shape).astype(dtype)
    out = {}
    for mode in ("0", "force"):
        monkeypatch.setitem(chunk_mod.PATHS, "scatter", "off" if mode == "0" else mode)
        c = bolt.array(x, bctx, axis=tuple(range(split))).chunk(plan, padding=pad)
        k2v = c.keys_to_values((split - 1,))
        v2k = c.values_to_keys((0,))
        out[mode] = [c.unchunk().toarray().tobytes(), k2v._packed.cpu().numpy().tobytes(),
                     v2k._packed.cpu().numpy().tobytes(), k2v.unchunk().toarray().tobytes(),
                     v2k.unchunk().toarray().tobytes()]
    assert out["0"] == out["force"]
    assert out["force"][0] == x.tobytes()


def test_scatter_plans_invert_the_gather_maps():
    """plan.copies_to_scatter on an unpack is the inverse of the pack-side
    gather map of the cores (every dense element comes from exactly one
    packed element, halos dropped), scatter_vec's vectors satisfy their
    contract, and scatter_runs_ok accepts line-aligned runs only."""
    from bolt_amd.mi355x.plan import (ChunkGeometry, copies_to_scatter, copies_to_map, scatter_vec,
                                      scatter_runs_ok)
    rng = np.random.default_rng(11)
    for _ in range(60):
        n = int(rng.integers(1, 4))
        vshape = tuple(int(v) for v in rng.integers(2, 9, n))
        plan = tuple(int(rng.integers(1, v + 1)) for v in vshape)
        pad = tuple(int(rng.integers(0, 2)) if p < v and rng.random() < 0.5 else 0 for p, v in zip(plan, vshape))
        g = ChunkGeometry(vshape, plan, pad)
        rec = int(np.prod(vshape))
        sc = copies_to_scatter([(sh, ps, ds, po, do) for sh, ds, ps, do, po in g.copies(unpack=True)], g.size)
        assert sc is not None
        map_a, map_b = sc
        gather = copies_to_map([(sh, ps, ds, po, do) for sh, ds, ps, do, po in g.copies(unpack=True)], rec)
        keep = map_a >= 0
        assert keep.sum() == rec and np.array_equal(np.sort(map_a[keep]), np.arange(rec))
        assert np.array_equal(gather[map_a[keep]], np.flatnonzero(keep))
        for es in (1, 2, 4, 8):
            v = scatter_vec(map_a, map_b, g.size, rec, es)
            assert v * es <= 16 and g.size % v == 0
            a = map_a.reshape(-1, v)
            kept = a[:, 0] >= 0
            assert np.all((a >= 0) == kept[:, None])
            assert np.all(a[kept] == a[kept][:, :1] + np.arange(v)) and np.all(a[kept][:, 0] % v == 0)
    # whole 128-B lines (16 float64 per core row) pass, 144-B misaligned runs fail
    ok = ChunkGeometry((64, 64), (16, 16), (2, 2))
    m = copies_to_scatter([(sh, ps, ds, po, do) for sh, ds, ps, do, po in ok.copies(unpack=True)], ok.size)
    assert scatter_runs_ok(m[0], m[1], 8)
    runs18 = np.concatenate([np.arange(18) + 20 * k for k in range(4)]).astype(np.int32)
    assert not scatter_runs_ok(runs18, np.zeros(72, np.int32), 8)


RUNS_CASES = [
    # (shape, split, dtype, plan, padding): keys_to_values of the trailing key
    # whose chunk boxes are long runs (bm_record_runs), every vector width
    ((2, 3, 4, 40, 40), 3, np.float64, (20, 20), (2, 2)),   # C5-like: 16-B vectors, 3.9-KB boxes
    ((2, 3, 2, 36, 30), 3, np.float32, (18, 15), (1, 1)),   # 1.2-1.4-KB boxes
    ((2, 2, 3, 64, 64), 3, np.uint8, (48, 48), (1, 1)),     # odd box sizes: 1-B vectors
    ((3, 5, 64, 48), 2, np.int16, (64, 24), (0, 2)),        # 2 key axes, 1 moved
]


@pytest.mark.parametrize("shape,split,dtype,plan,pad", RUNS_CASES)
def test_record_runs_path_matches(bctx, monkeypatch, shape, split, dtype, plan, pad):
    """keys_to_values through bm_record_runs gives the same packed bytes as the
    map scatter and the strided copies, and unchunks to the input."""
    from bolt_amd.mi355x import _ops
    rng = np.random.default_rng(8)
    x = rng.integers(0, 250, size=shape).astype(dtype)
    calls = []
    be = _ops.backend_for(bctx.device)
    orig = be.record_runs
    monkeypatch.setattr(be, "record_runs", lambda *a, **k: (calls.append(a[4:8]), orig(*a, **k))[1])
    out = {}
    for runs, scatter in (("1", "1"), ("0", "1"), ("0", "0")):
        monkeypatch.setitem(chunk_mod.PATHS, "runs", runs == "1")
        monkeypatch.setitem(chunk_mod.PATHS, "scatter", "on" if scatter == "1" else "off")
        c = bolt.array(x, bctx, axis=tuple(range(split))).chunk(plan, padding=pad)
        k = c.keys_to_values((split - 1,))
        out[runs + scatter] = (k._packed.cpu().numpy().tobytes(), k.unchunk().toarray().tobytes())
    assert calls, "the runs path was not taken"
    assert out["11"] == out["01"] == out["00"]
    want = bolt.array(x, bctx, axis=tuple(range(split))).chunk(plan, padding=pad).keys_to_values(
        (split - 1,)).unchunk().toarray()
    assert out["11"][1] == np.asarray(want).tobytes()


def test_scatter_to_runs_table():
    """plan.scatter_to_runs: C5's k2v plan is 16 runs (one per chunk box) in
    16-B vectors; unchunk's 128-B rows stay with the map scatter; odd sizes
    narrow the vector."""
    from bolt_amd.mi355x.plan import (ChunkGeometry, copies_to_scatter, k2v_copies, scatter_to_runs)
    g = ChunkGeometry((64, 64), (16, 16), (2, 2))
    new = ChunkGeometry((64, 64, 64), (64, 16, 16), (0, 2, 2))
    sc = copies_to_scatter(k2v_copies(g, new, [1, 1, 64], np.array([False, False, True])), 64 * g.size,
                           group=64, src_rec=g.size)
    runs, vb = scatter_to_runs(sc[0], sc[1], g.size, new.size, 8)
    assert vb == 16 and runs.shape == (16, 4)
    lens = sorted(set((runs[:, 1] * 16).tolist()))
    assert lens == [2592, 2880, 3200]            # 18x18, 18x20 / 20x18, 20x20 float64 boxes
    assert np.array_equal(runs[:, 1], runs[:, 3])  # consecutive keys stack whole boxes
    un = copies_to_scatter([(sh, ps, ds, po, do) for sh, ds, ps, do, po in g.copies(unpack=True)], g.size)
    assert scatter_to_runs(un[0], un[1], g.size, 64 * 64, 8) is None
    a = np.arange(1089, dtype=np.int32)
    assert scatter_to_runs(a, np.zeros_like(a), 1089, 1089, 1)[1] == 1


def _runs_fuzz_cases(n=24, seed=21):
    """Random keys_to_values geometries of the trailing key whose scatter plan
    bm_record_runs takes (plan.scatter_to_runs: few runs of >= 1 KiB on
    average), every element size."""
    from bolt_amd.mi355x.plan import ChunkGeometry, copies_to_scatter, k2v_copies, scatter_to_runs
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        dt = [np.uint8, np.int16, np.float32, np.float64][int(rng.integers(0, 4))]
        es = np.dtype(dt).itemsize
        nv = int(rng.integers(1, 3))
        vshape = tuple(int(v) for v in rng.integers(8, 72, nv))
        plan = tuple(int(rng.integers(max(2, v // 4), v + 1)) for v in vshape)
        pad = tuple(int(rng.integers(0, min(3, v - p) + 1)) if p < v else 0 for p, v in zip(plan, vshape))
        if np.prod(vshape) * es > 40000:
            continue
        split = int(rng.integers(1, 3))
        kshape = tuple(int(k) for k in rng.integers(1, 4, split - 1)) + (int(rng.integers(2, 6)),)
        K = kshape[-1]
        g = ChunkGeometry(vshape, plan, pad)
        new = ChunkGeometry((K,) + vshape, (K,) + plan, (0,) + pad)
        sc = copies_to_scatter(k2v_copies(g, new, [1] * (split - 1) + [K], np.array([False] * (split - 1) + [True])),
                               K * g.size, group=K, src_rec=g.size)
        if sc is None or scatter_to_runs(sc[0], sc[1], g.size, new.size, es) is None:
            continue
        out.append((kshape + vshape, split, dt, plan, pad))
    return out


@pytest.mark.parametrize("case", range(24))
def test_record_runs_fuzz(bctx, monkeypatch, case):
    """Seeded random geometries: keys_to_values of the trailing key through the
    runs kernel (destination walk when the boxes tile the new records) equals
    the strided-copy path, and its unchunk restores the input."""
    shape, split, dtype, plan, pad = _runs_fuzz_cases()[case]
    rng = np.random.default_rng(case)
    x = rng.integers(0, 250, size=shape).astype(dtype)
    out = {}
    for runs, scatter in (("1", "1"), ("0", "0")):
        monkeypatch.setitem(chunk_mod.PATHS, "runs", runs == "1")
        monkeypatch.setitem(chunk_mod.PATHS, "scatter", "on" if scatter == "1" else "off")
        c = bolt.array(x, bctx, axis=tuple(range(split))).chunk(plan, padding=pad)
        k = c.keys_to_values((split - 1,))
        out[runs] = (k._packed.cpu().numpy().tobytes(), k.unchunk().toarray().tobytes(), k.plan.tolist(),
                     k.padding.tolist(), k.shape)
    assert out["1"] == out["0"], (shape, split, dtype, plan, pad)


@pytest.mark.gpu
@pytest.mark.parametrize("es", [1, 2, 4, 8])
def test_record_runs_untiled_table(gpu_ctx, es):
    """bm_record_runs WITHOUT BM_RUNS_TILED (k_record_runs: one wave per
    (record, run)), called directly: a table whose runs leave gaps in the
    destination, stack with a stride m != len and start mid-record, so no
    keys_to_values reaches it.  Every destination byte equals the numpy
    executor's (tests/cpu_backend.py) on the same bytes, gap bytes untouched;
    every element size, 16-B vectors."""
    import sys
    import os
    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import cpu_backend
    from bolt_amd.mi355x import _ops
    be = _ops.backend_for(gpu_ctx.device)
    vb = 16
    per = vb // es
    # [s, len, a, m] in 16-B vectors; group 3: run 0 -> [0,8) [10,18) [20,28),
    # run 1 -> [30,36) [37,43) [44,50), run 2 -> [52,62) [62,72) [72,82) of 90
    table = np.array([[0, 8, 0, 10], [12, 6, 30, 7], [30, 10, 52, 10]], np.int64)
    group, nrec = 3, 12
    src_rec, gstride = 40 * per, 90 * per
    rng = np.random.default_rng(es)
    src = rng.integers(0, 256, nrec * src_rec * es, dtype=np.uint8)
    dst0 = rng.integers(0, 256, nrec // group * gstride * es, dtype=np.uint8)
    g_src = torch.from_numpy(src).to(gpu_ctx.device)
    g_dst = torch.from_numpy(dst0.copy()).to(gpu_ctx.device)
    key = ("test_untiled", es)
    be.record_runs(g_src, 0, g_dst, 0, nrec, src_rec, group, gstride, (table, vb), key, es)
    assert be._maps[(g_src.device, key)][3] == 0  # the untiled kernel ran
    want = torch.from_numpy(dst0.copy())
    cpu_backend.CpuBackend().record_runs(torch.from_numpy(src.copy()), 0, want, 0, nrec, src_rec, group, gstride,
                                         (table, vb), key, es)
    assert torch.equal(g_dst.cpu(), want)
    assert not np.array_equal(want.numpy(), dst0)  # the runs moved bytes


@pytest.mark.gpu
def test_record_runs_wrong_tiled_flag_stays_in_bounds(gpu_ctx):
    """BM_RUNS_TILED on runs that do NOT tile the records (the flag is the
    caller's claim; the library cannot see the device table): the destination
    walk clamps every read into a run of a source record of its group, so the
    call completes -- wrong bytes, no access outside the buffers (the source
    sits between two guard regions that must stay unread-through: the result
    holds only bytes of the source proper)."""
    import ctypes
    import torch
    from bolt_amd.mi355x import _lib
    lib = _lib.load()
    es, vb = 8, 16
    table = np.array([[0, 8, 0, 10], [12, 6, 30, 7], [30, 10, 52, 10]], np.int64)  # not a tiling
    group, nrec = 3, 12
    src_rec, gstride = 40 * 2, 90 * 2
    n_src = nrec * src_rec
    guard = 4096
    buf = torch.full((guard + n_src + guard,), -1, dtype=torch.int64, device=gpu_ctx.device)
    buf[guard:guard + n_src] = torch.arange(n_src, dtype=torch.int64, device=gpu_ctx.device)
    src = buf[guard:guard + n_src]
    dst = torch.full((nrec // group * gstride,), -2, dtype=torch.int64, device=gpu_ctx.device)
    t = torch.from_numpy(table.reshape(-1).copy()).to(gpu_ctx.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(gpu_ctx.device).cuda_stream)
    rc = lib.bm_record_runs(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), nrec, src_rec, group,
                            gstride, 3, ctypes.c_void_p(t.data_ptr()), vb, _lib.RUNS_TILED, es, stream)
    assert rc == 0
    torch.cuda.synchronize(gpu_ctx.device)
    out = dst.cpu().numpy()
    assert out.min() >= 0 and out.max() < n_src  # every element came from the source proper
