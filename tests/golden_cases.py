"""Loader and comparison rules for the reference-generated golden fixtures.

tests/golden/golden.json + golden.npz are written by tests/golden/make_golden.py
from the reference bolt itself (Spark mode over an in-process RDD).  Inputs
are regenerated from their specs (tests/golden/inputs.py).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)

from inputs import make_input  # noqa: E402,F401

_META = None
_ARR = None


def meta():
    global _META, _ARR
    if _META is None:
        with open(os.path.join(GOLDEN, "golden.json")) as f:
            _META = json.load(f)
        _ARR = np.load(os.path.join(GOLDEN, "golden.npz"))
    return _META


def cases(op):
    return [c for c in meta()["cases"] if c["op"] == op]


def arr(case, name):
    meta()
    return _ARR["c%d_%s" % (case["id"], name)]


def case_id(c):
    return "c%d" % c["id"]


def tup(v):
    if v is None:
        return None
    if isinstance(v, list):
        return tuple(v)
    return v


def size_arg(v):
    return v if isinstance(v, str) else tup(v)


def truth_stat(x, name, axis):
    """float128 truth of a statistic (population var/std), kept axes ascending."""
    ax = tuple(range(x.ndim)) if axis is None else (tuple(axis) if isinstance(axis, (list, tuple)) else (axis,))
    v = x.astype(np.longdouble)
    if name == "mean":
        return v.mean(axis=ax)
    if name == "sum":
        return v.sum(axis=ax)
    if name in ("min", "max"):
        return getattr(v, name)(axis=ax)
    var = v.var(axis=ax)
    return var if name == "var" else np.sqrt(var)


def stat_close(got, ref, truth, out_dtype, x, name="mean"):
    """The parity rule of SURVEY.md 8(c): |got-ref| <= rtol*|ref| + atol, with
    rtol 1e-6 (float32/float16 outputs) / 1e-12 (float64).  For mean and sum
    atol = rtol*max|x| (the statistic's units).  For var / std the bar is the
    pure relative one, rtol*|ref|, plus only an eps-sized floor
    atol = rtol*eps*max|ref| so that a zero variance may come out as a tiny
    positive one -- never max|x| (which would relax the bar on offset data) and
    never a second rtol*|ref| (which would double it).  A result that is at
    least as close to the float128 truth as the reference's also passes (the
    reference accumulates float32 statistics in float32, order-dependently)."""
    got = np.asarray(got, dtype=np.longdouble)
    ref = np.asarray(ref, dtype=np.longdouble)
    truth = np.asarray(truth, dtype=np.longdouble).reshape(ref.shape)
    rtol = 1e-12 if np.dtype(out_dtype) == np.float64 else 1e-6
    if np.dtype(out_dtype) == np.float16:
        rtol = 1e-3
    finite = np.abs(ref[np.isfinite(ref)]) if ref.size else ref
    if name in ("var", "std", "variance", "stdev"):
        # pure relative per output; the eps floor lets a zero variance come out (near) zero
        scale = np.finfo(out_dtype).eps * (float(np.max(finite)) if finite.size else 0.0)
    else:
        xa = np.abs(np.asarray(x, dtype=np.longdouble))
        xa = xa[np.isfinite(xa)]
        scale = max(float(np.max(xa)) if xa.size else 0.0,
                    float(np.max(finite)) if finite.size else 0.0, 1e-300)
    ok1 = np.abs(got - ref) <= rtol * np.abs(ref) + rtol * scale
    eps = np.finfo(out_dtype).eps if np.dtype(out_dtype).kind == 'f' else 0
    # a NaN the reference's accumulation order made (inf * 0 after a partial
    # product overflowed) where the truth is a number is infinitely far from it
    ref_err = np.where(np.isnan(ref) & ~np.isnan(truth), np.inf, np.abs(ref - truth))
    ok2 = np.abs(got - truth) <= ref_err + 2 * eps * np.abs(truth) + eps * rtol * scale
    both_nan = np.isnan(got) & np.isnan(ref)
    return bool(np.all(ok1 | ok2 | both_nan))


def _dec_item(i):
    if isinstance(i, dict) and "slice" in i:
        return slice(*i["slice"])
    if isinstance(i, dict) and "array" in i:
        return np.array(i["array"])
    return i


def index_arg(enc):
    """The index of a getitem case (make_golden.enc_item encoding)."""
    if "tuple" in enc:
        return tuple(_dec_item(i) for i in enc["tuple"])
    return _dec_item(enc["item"])


def truth_reduce(x, func_name, axis):
    """float128 truth of a float reduce (sum / product) over ``axis``, or None."""
    ax = tuple(axis)
    v = np.asarray(x, dtype=np.longdouble)
    if func_name in ("add", "np_add", "lam_add"):
        return v.sum(axis=ax)
    if func_name in ("multiply", "mul", "lam_mul"):
        return v.prod(axis=ax)
    if func_name == "lam_absadd":
        return np.abs(v).sum(axis=ax)
    return None


def reduce_close(got, want, x, func_name, axis):
    """Reduce parity: bit-exact for integer / bool results and for the selecting
    ufuncs (maximum, minimum, fmax, fmin); floating sums and products by
    stat_close's rule against their float128 truth (the reference accumulates
    in the record dtype, in its treeReduce order)."""
    got = np.asarray(got)
    want = np.asarray(want)
    if got.dtype != want.dtype or got.shape != want.shape:
        return False
    truth = truth_reduce(x, func_name, axis)
    if want.dtype.kind != 'f' or truth is None:
        return got.tobytes() == want.tobytes()
    return stat_close(got, want, truth, want.dtype, x, "sum")
