"""User functions of the map / stack golden cases, by name.

Each works on a numpy array (the reference, in make_golden.py) and on a torch
tensor (the mi355x mode, whose user functions see device tensors); EXACT says
whether the two agree bit for bit (elementwise IEEE arithmetic) or only to
rounding (reductions, whose summation order differs).
"""
import operator

import numpy as np


def _torch(v):
    return type(v).__module__.startswith("torch")


def _cat(a, b, axis):
    if _torch(a):
        import torch
        return torch.cat((a, b), dim=axis)
    return np.concatenate((a, b), axis=axis)


def _flip(v, axis):
    if _torch(v):
        import torch
        return torch.flip(v, (axis,))
    return np.flip(v, axis)


def _astype(v, dt):
    if _torch(v):
        from bolt_amd.mi355x.functional import torch_dtype
        return v.to(torch_dtype(dt))
    return v.astype(dt)


def _ones(shape, like):
    if _torch(like):
        import torch
        return torch.ones(shape, dtype=torch.float64, device=like.device)
    return np.ones(shape)


FUNCS = {
    "double": lambda v: 2 * v,
    "affine": lambda v: v * 3 - 1,
    "square": lambda v: v * v,
    "crop_last": lambda v: v[..., :4],
    "dup_last": lambda v: _cat(v, v, -1),
    "flip_last": lambda v: _flip(v, -1),
    "to_f64": lambda v: _astype(v, np.float64),
    "center0": lambda v: v - v.mean(axis=0, keepdims=True),
    "first_row": lambda v: v[0],
    "shrink0": lambda v: v[:2],
    "sum1": lambda v: v.sum(axis=1),
    "sum0": lambda v: v.sum(axis=0),
    "ones22": lambda v: _ones((2, 2), v),
    "tile12": lambda v: _cat(v, v, 1),
    "scalar2": lambda v: 2,
    "none": lambda v: None,
    "zerodiv": lambda v: 1 / 0,
    "norm_rows": lambda v: v / (1 + (v * v).sum(axis=-1, keepdims=True)),
    "arr1": lambda v: np.asarray([2]),
    "arr0": lambda v: np.asarray(2),
    # int(): numpy-2 promotes float32 * numpy.int64 key scalar to float64 (numpy 1 did not)
    "keyed": lambda kv: kv[1] * (int(kv[0][0]) + 1),
    "gt_mean": lambda v: v.sum() > 0,
    "gt_big": lambda v: v.max() > 100,
    "never": lambda v: v.sum() < -1e30,
}

EXACT = {"double", "affine", "square", "crop_last", "dup_last", "flip_last", "to_f64", "first_row", "shrink0",
         "ones22", "tile12", "arr1", "arr0", "keyed"}

# binary functions of the reduce golden cases (array.py:243-282): numpy ufuncs
# and operator spellings run as one device reduction; the lambdas take the
# generic path (a pairwise tree of the function on device tensors)
RFUNCS = {
    "add": operator.add, "np_add": np.add, "multiply": np.multiply, "mul": operator.mul,
    "maximum": np.maximum, "minimum": np.minimum, "fmax": np.fmax, "fmin": np.fmin,
    "logical_and": np.logical_and, "logical_or": np.logical_or,
    "bitwise_and": np.bitwise_and, "bitwise_or": np.bitwise_or, "bitwise_xor": np.bitwise_xor,
    "and_": operator.and_, "or_": operator.or_, "xor": operator.xor,
    "lam_add": lambda a, b: a + b,
    "lam_absadd": lambda a, b: abs(a) + abs(b),
    "lam_mul": lambda a, b: a * b,
}
