"""Deterministic inputs of the golden cases (shared by make_golden.py and the tests).

An input is named by a spec {"shape", "dtype", "kind", "seed"}; numpy's
PCG64 default_rng streams are stable across numpy versions, so the arrays are
regenerated instead of stored.
"""
import numpy as np


def make_input(spec):
    shape = tuple(spec["shape"])
    dtype = np.dtype(spec["dtype"])
    kind = spec.get("kind", "arange")
    rng = np.random.default_rng(spec.get("seed", 0))
    n = int(np.prod(shape))
    if kind == "arange":
        return np.arange(n).astype(dtype).reshape(shape)
    if kind == "normal":
        x = rng.standard_normal(shape)
        if "shift" in spec:  # offset data: shift + N(0,1), e.g. 1e6 + N(0,1)
            x = spec["shift"] + x
        if "outlier" in spec:  # value at index 0 of one axis, e.g. x[:, 0] = 100
            ax, v = spec["outlier"]
            idx = [slice(None)] * len(shape)
            idx[ax] = 0
            x[tuple(idx)] = v
        if "nan_every" in spec:  # NaNs at every k-th element (fmax / fmin / maximum cases)
            x.reshape(-1)[::spec["nan_every"]] = np.nan
        return x.astype(dtype)
    if kind == "imaging":  # 1000 + 50 N(0,1): SURVEY.md 8(d) C2
        return (1000 + 50 * rng.standard_normal(shape)).astype(dtype)
    if kind == "bits":  # random bit patterns (NaN payloads included)
        raw = rng.integers(0, 256, size=n * dtype.itemsize, dtype=np.uint8)
        return raw.view(dtype).reshape(shape)
    if kind == "ints":
        info = np.iinfo(dtype)
        lo = max(info.min, -(1 << 20)) if spec.get("small") else info.min
        hi = min(info.max, 1 << 20) if spec.get("small") else info.max
        return rng.integers(lo, hi, size=shape, dtype=dtype, endpoint=True)
    if kind == "bool":
        return rng.integers(0, 2, size=shape).astype(bool)
    raise ValueError(kind)
