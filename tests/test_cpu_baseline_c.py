"""oracle/c/local_step.c (the OpenMP port of the local mode's C2 step that
bench.py times as an extra CPU line) against numpy on the same input."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("omp") / "liblocal_step.so"
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle", "c"), "OUT=%s" % out],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("gcc / OpenMP unavailable: %s" % r.stderr[-300:])
    lib = ctypes.CDLL(str(out))
    f32p = ctypes.POINTER(ctypes.c_float)
    for fn in (lib.local_swap, lib.local_mean, lib.local_std):
        fn.argtypes = [f32p, f32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    return lib


@pytest.mark.parametrize("shape", [(200, 24, 16), (67, 9, 130), (1, 5, 7)])
def test_local_step_matches_numpy(lib, shape):
    rng = np.random.default_rng(3)
    x = (1000 + 50 * rng.standard_normal(shape)).astype(np.float32)
    T, P = shape[0], shape[1] * shape[2]
    y = np.empty((P, T), np.float32)
    m = np.empty(P, np.float32)
    sd = np.empty(P, np.float32)
    f32p = ctypes.POINTER(ctypes.c_float)
    p = lambda a: a.ctypes.data_as(f32p)
    lib.local_swap(p(x), p(y), T, P, 4)
    lib.local_mean(p(y), p(m), T, P, 4)
    lib.local_std(p(y), p(sd), T, P, 4)
    want = np.ascontiguousarray(x.transpose(1, 2, 0)).reshape(P, T)
    assert y.tobytes() == want.tobytes()
    x64 = x.astype(np.float64)
    assert np.allclose(m, x64.mean(axis=0).reshape(P), rtol=1e-6)
    assert np.allclose(sd, x64.std(axis=0).reshape(P), rtol=1e-5, atol=1e-6)
