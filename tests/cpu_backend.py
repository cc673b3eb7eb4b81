"""A numpy executor of the libbolt_mi355x kernel contracts, for CPU tests only.

The product has no CPU fallback (bolt_amd.mi355x._ops raises for a non-GPU
device).  Tests register this executor for the 'cpu' device type to check the
HOST logic -- chunk geometry and copy descriptors, swap/transpose planning,
reduction layouts, result formatting and the multi-rank orchestration over
gloo -- with world sizes > 1 on a machine without a GPU.  It implements each
C-ABI entry point's documented semantics (include/bolt_mi355x.h) with numpy:
strided copies through np.ndarray views, reductions in float64/longdouble
with the same output-dtype and modular-integer rules as the kernels.
"""
import numpy as np

STAT_MEAN, STAT_VAR, STAT_STD, STAT_SUM, STAT_MAX, STAT_MIN = range(6)
STAT_PROD, STAT_LAND, STAT_LOR, STAT_BAND, STAT_BOR, STAT_BXOR, STAT_FMAX, STAT_FMIN = range(6, 14)
_PICK = {STAT_MAX: np.maximum, STAT_MIN: np.minimum, STAT_FMAX: np.fmax, STAT_FMIN: np.fmin}
_BITOP = {STAT_BAND: np.bitwise_and, STAT_BOR: np.bitwise_or, STAT_BXOR: np.bitwise_xor}
_CODES = [np.bool_, np.uint8, np.int8, np.uint16, np.int16, np.uint32, np.int32, np.uint64,
          np.int64, np.float16, np.float32, np.float64]


def _np(t):
    return t.numpy()


def _view(buf, off, shape, strides, es):
    return np.ndarray(tuple(int(s) for s in shape), dtype=np.dtype((np.void, es)), buffer=buf,
                      offset=int(off), strides=tuple(int(s) * es for s in strides))


def _bits64(a):
    """Elements' bits in the low bytes of uint64 slots (the max/min state layout)."""
    a = np.ascontiguousarray(a)
    out = np.zeros(a.size, dtype=np.uint64)
    out.view(np.uint8).reshape(a.size, 8)[:, :a.itemsize] = a.view(np.uint8).reshape(a.size, a.itemsize)
    return out


def _unbits64(u, dt):
    u = np.ascontiguousarray(u, dtype=np.uint64)
    return u.view(np.uint8).reshape(u.size, 8)[:, :dt.itemsize].copy().view(dt).reshape(-1)


class CpuBackend(object):
    name = "cpu-test"
    transport = "torch"  # torch.distributed collectives on CPU tensors (gloo)

    def copy_strided(self, src, src_off, dst, dst_off, shape, sstrides, dstrides, es):
        if len(shape) == 0:
            shape, sstrides, dstrides = [1], [1], [1]
        if any(int(s) == 0 for s in shape):
            return
        s = _view(_np(src), src_off, shape, sstrides, es)
        d = _view(_np(dst), dst_off, shape, dstrides, es)
        d[...] = s

    def gather_rows(self, src, src_off, dst, dst_off, n_outer, src_rows, row_bytes, idx):
        idx = np.asarray(idx, dtype=np.int64).reshape(-1)
        if idx.size == 0 or n_outer == 0:
            return
        if idx.min() < 0 or idx.max() >= src_rows:
            raise IndexError("gather index out of range [0, %d)" % src_rows)
        s = _np(src)[src_off:src_off + n_outer * src_rows * row_bytes].reshape(n_outer, src_rows, row_bytes)
        d = _np(dst)[dst_off:dst_off + n_outer * idx.size * row_bytes].reshape(n_outer, idx.size, row_bytes)
        d[...] = s[:, idx, :]

    def record_gather(self, src, src_off, dst, dst_off, nrec, src_rec, dst_rec, rmap, key, es):
        if nrec == 0:
            return
        rmap = np.asarray(rmap, dtype=np.int64)
        assert rmap.size == dst_rec and rmap.min() >= 0 and rmap.max() < src_rec
        dt = np.dtype((np.void, es))
        s = _np(src)[src_off:src_off + nrec * src_rec * es].view(dt).reshape(nrec, src_rec)
        d = _np(dst)[dst_off:dst_off + nrec * dst_rec * es].view(dt).reshape(nrec, dst_rec)
        d[...] = s[:, rmap]

    def record_scatter(self, src, src_off, dst, dst_off, nrec, src_rec, group, gstride, plan, key, es):
        if nrec == 0:
            return
        map_a, map_b, vec = plan
        map_a = np.asarray(map_a, dtype=np.int64)
        map_b = np.asarray(map_b, dtype=np.int64)
        assert map_a.size == src_rec and map_b.size == src_rec and src_rec % vec == 0 and gstride % vec == 0
        dt = np.dtype((np.void, es))
        s = _np(src)[src_off:src_off + nrec * src_rec * es].view(dt).reshape(nrec, src_rec)
        d = _np(dst)[dst_off:].view(dt) if (len(_np(dst)) - dst_off) % es == 0 else None
        if d is None:
            d = _np(dst)[dst_off:dst_off + (len(_np(dst)) - dst_off) // es * es].view(dt)
        keep = map_a >= 0
        r = np.arange(nrec, dtype=np.int64)[:, None]
        idx = (r // group) * gstride + map_a[None, keep] + (r % group) * map_b[None, keep]
        assert idx.min(initial=0) >= 0 and idx.max(initial=-1) < d.size
        d[idx.reshape(-1)] = s[:, keep].reshape(-1)

    def record_runs(self, src, src_off, dst, dst_off, nrec, src_rec, group, gstride, runs, key, es):
        if nrec == 0:
            return
        table, vb = runs
        t = np.asarray(table, dtype=np.int64).reshape(-1, 4) * (vb // es)
        dt = np.dtype((np.void, es))
        s = _np(src)[src_off:src_off + nrec * src_rec * es].view(dt).reshape(nrec, src_rec)
        d = _np(dst)[dst_off:dst_off + nrec // group * gstride * es].view(dt).reshape(nrec // group, gstride)
        for s0, ln, a, m in t:
            assert s0 >= 0 and s0 + ln <= src_rec and a + (group - 1) * m + ln <= gstride
            for k in range(group):
                d[:, a + k * m:a + k * m + ln] = s[k::group, s0:s0 + ln]

    def permute(self, src, shape, perm, es, dst):
        a = _np(src).view(np.dtype((np.void, es))).reshape(tuple(shape))
        out = _np(dst).view(np.dtype((np.void, es)))
        out[...] = np.ascontiguousarray(a.transpose(perm)).reshape(-1)

    def _planes(self, stat, code, x):
        """x: (O, R, I) in the input dtype -> state planes (list of arrays (O*I,))."""
        dt = np.dtype(_CODES[code])
        if stat in _PICK:
            r = _PICK[stat].reduce(x, axis=1).reshape(-1)
            return [_bits64(r)]
        if stat in (STAT_LAND, STAT_LOR) or (stat == STAT_PROD and dt == np.bool_):
            f = np.all if stat != STAT_LOR else np.any
            return [f(x != 0, axis=1).reshape(-1).astype(np.uint64)]
        if stat in _BITOP:
            if dt.kind == 'f':
                raise ValueError("bitwise reduction of a float dtype")
            return [_BITOP[stat].reduce(_bits64(x).reshape(x.shape), axis=1).reshape(-1)]
        if stat == STAT_PROD:
            if dt.kind in 'iu':
                return [np.multiply.reduce(x.astype(np.int64).astype(np.uint64), axis=1).reshape(-1)]
            return [x.astype(np.float64).prod(axis=1).reshape(-1)]
        if stat == STAT_SUM:
            if dt == np.bool_:
                return [x.any(axis=1).reshape(-1).astype(np.uint64)]
            if dt.kind in 'iu':
                return [np.add.reduce(x.astype(np.uint64), axis=1).reshape(-1)]
            return [x.astype(np.float64).sum(axis=1).reshape(-1)]
        v = x.astype(np.longdouble)
        m = v.mean(axis=1)
        m2 = ((v - m[:, None, :]) ** 2).sum(axis=1)
        return [m.reshape(-1).astype(np.float64), m2.reshape(-1).astype(np.float64)]

    def _finish(self, stat, code, planes, n, out, out_code):
        dt = np.dtype(_CODES[code])
        odt = np.dtype(_CODES[out_code])
        o = _np(out).view(odt)
        if stat in _PICK or stat in _BITOP:
            o[...] = _unbits64(planes[0], dt)
            return
        if stat in (STAT_LAND, STAT_LOR) or (stat == STAT_PROD and dt == np.bool_):
            o[...] = planes[0] != 0
            return
        if stat in (STAT_SUM, STAT_PROD):
            if dt.kind in 'iub':
                o[...] = planes[0].astype(dt) if dt != np.bool_ else planes[0] != 0
            else:
                o[...] = planes[0].astype(odt)
            return
        if stat == STAT_MEAN:
            o[...] = planes[0].astype(odt)
            return
        var = planes[1] / n
        o[...] = (var if stat == STAT_VAR else np.sqrt(var)).astype(odt)

    def reduce(self, stat, src, code, O, R, I, out, out_code):
        x = _np(src).view(_CODES[code]).reshape(O, R, I)
        # (columns over a row-padded array include the pad's unwritten values;
        # their outputs are dropped, so their overflows are not reported)
        with np.errstate(all="ignore"):
            self._finish(stat, code, self._planes(stat, code, x), float(R), out, out_code)

    def reduce_rows(self, stat, src, code, O, R, pitch, out, out_code):
        assert pitch >= R
        x = _np(src).view(_CODES[code])[:O * pitch].reshape(O, pitch)[:, :R].reshape(O, R, 1)
        self._finish(stat, code, self._planes(stat, code, x), float(R), out, out_code)

    def state_bytes(self, stat, code, nout):
        mom = stat in (STAT_VAR, STAT_STD)  # max / min / sum / mean: one 8-byte plane
        return (2 if mom else 1) * nout * 8

    def reduce_state(self, stat, src, code, O, R, I, state):
        x = _np(src).view(_CODES[code]).reshape(O, R, I)
        planes = self._planes(stat, code, x)
        if stat == STAT_MEAN:
            planes = planes[:1]  # the mean state is one plane (M2 is not kept)
        buf = _np(state)
        for i, p in enumerate(planes):
            buf[i * O * I * 8:(i + 1) * O * I * 8] = p.view(np.uint8)

    def reduce_combine(self, stat, code, states, counts, nout, out, out_code):
        buf = _np(states)
        mom = stat in (STAT_VAR, STAT_STD)
        npl = 2 if mom else 1
        per = npl * nout * 8
        dt = np.dtype(_CODES[code])
        n, m, q = 0.0, np.zeros(nout), np.zeros(nout)
        acc_u = np.zeros(nout, dtype=np.uint64)
        acc_f = np.zeros(nout)
        acc_m = None
        for p, c in enumerate(counts):
            if c <= 0:
                continue
            part = buf[p * per:(p + 1) * per]
            if stat in _PICK:
                v = _unbits64(part[:nout * 8].view(np.uint64), dt)
                acc_m = v.copy() if acc_m is None else _PICK[stat](acc_m, v)
                continue
            if stat in _BITOP or stat in (STAT_LAND, STAT_LOR) or stat == STAT_PROD:
                u = part[:nout * 8].view(np.uint64)
                if stat == STAT_PROD and dt.kind == 'f':
                    u = u.view(np.float64)
                if acc_m is None:
                    acc_m = u.copy()
                elif stat in _BITOP:
                    acc_m = _BITOP[stat](acc_m, u)
                elif stat == STAT_LOR:
                    acc_m = acc_m | u
                elif stat == STAT_LAND or dt == np.bool_:
                    acc_m = acc_m & u
                else:
                    acc_m = acc_m * u
                continue
            if stat == STAT_SUM:
                if dt.kind in 'iub':
                    u = part[:nout * 8].view(np.uint64)
                    acc_u = (acc_u | u) if dt == np.bool_ else (acc_u + u)
                else:
                    acc_f = acc_f + part[:nout * 8].view(np.float64)
                continue
            mb = part[:nout * 8].view(np.float64)
            qb = part[nout * 8:2 * nout * 8].view(np.float64) if mom else np.zeros(nout)
            if n == 0:
                n, m, q = float(c), mb.copy(), qb.copy()
            else:
                tot = n + c
                d = mb - m
                m = m + d * (c / tot)
                q = q + qb + d * d * (n * c / tot)
                n = tot
        if stat in _PICK:
            planes = [_bits64(acc_m)]
        elif stat in _BITOP or stat in (STAT_LAND, STAT_LOR) or stat == STAT_PROD:
            planes = [acc_m]
        elif stat == STAT_SUM:
            planes = [acc_u] if dt.kind in 'iub' else [acc_f]
        else:
            planes = [m, q]
        self._finish(stat, code, planes, n, out, out_code)


def install():
    from bolt_amd.mi355x._ops import register_backend
    register_backend("cpu", CpuBackend())


def install_host_staged_gpu():
    """The one-GPU multi-rank rehearsal: the HIP kernels, with the records
    exchanged over a gloo group through the host (RCCL refuses two ranks on one
    GPU).  A test executor only -- production contexts exchange over RCCL."""
    from bolt_amd.mi355x._ops import HipBackend, register_backend

    class HostStagedHip(HipBackend):
        name = "hip-host-staged-rehearsal"
        transport = "host"

    register_backend("cuda", HostStagedHip())


def uninstall():
    from bolt_amd.mi355x._ops import register_backend
    register_backend("cpu", None)
