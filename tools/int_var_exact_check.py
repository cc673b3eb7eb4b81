"""Bit-for-bit comparison of two libbolt_mi355x builds on the exact integer
variance / standard deviation / mean (2-byte records), and a float64 numpy
truth (diagnostic, one GPU).

    python tools/int_var_exact_check.py libA.so libB.so

Column reductions of [O][R][I] uint16 / int16 arrays (values drawn over the
whole range, extremes included) for shapes that take the main loop, its tail,
row phases and R-chunks with a combine; every output of B must equal A's
bytes (numpy's float64 result is printed for information only: it is not
exact itself).  Prints one line per case and ALL_EXACT at the end.
"""
import ctypes
import sys

import numpy as np
import torch

CODES = {np.dtype(np.uint16): 3, np.dtype(np.int16): 4}
F64 = 11


def load(path):
    lib = ctypes.CDLL(path)
    lib.bm_reduce.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                              ctypes.c_void_p]
    lib.bm_reduce_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int64, ctypes.POINTER(ctypes.c_size_t)]
    lib.bm_last_error.restype = ctypes.c_char_p
    return lib


def run(lib, stat, x, O, R, I):
    code = CODES[x.dtype]
    n = ctypes.c_size_t(0)
    assert lib.bm_reduce_workspace_bytes(stat, code, O, R, I, ctypes.byref(n)) == 0
    src = torch.from_numpy(x.reshape(-1).view(np.uint8).copy()).cuda()
    out = torch.empty(O * I * 8, dtype=torch.uint8, device="cuda")
    ws = torch.empty(max(1, n.value), dtype=torch.uint8, device="cuda")
    rc = lib.bm_reduce(stat, src.data_ptr(), code, O, R, I, out.data_ptr(), F64, ws.data_ptr(), n.value,
                       torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.bm_last_error()
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.float64).reshape(O, I)


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    rng = np.random.default_rng(7)
    shapes = [(1, 10000, 1024 * 64), (1, 8, 4096), (1, 9, 4096), (1, 4001, 1024), (3, 777, 2048),
              (1, 200000, 64), (2, 33, 8 * 512), (1, 65536, 128)]
    ok = True
    for dt in (np.uint16, np.int16):
        info = np.iinfo(dt)
        for O, R, I in shapes:
            x = rng.integers(info.min, int(info.max) + 1, size=(O, R, I), dtype=np.int64).astype(dt)
            x[:, : min(R, 3)] = info.max          # extremes in the first rows
            x[:, -1:] = info.min
            for stat, name in ((1, "var"), (2, "std"), (0, "mean")):
                ra, rb = run(a, stat, x, O, R, I), run(b, stat, x, O, R, I)
                same = ra.tobytes() == rb.tobytes()
                xf = x.astype(np.float64)
                truth = {0: xf.mean(axis=1), 1: xf.var(axis=1), 2: xf.std(axis=1)}[stat]
                rel = float(np.max(np.abs(rb - truth) / np.maximum(np.abs(truth), 1e-300)))
                ok &= same  # the numpy column is information (float64 numpy is not exact)
                print("%-6s %-16s %-4s bytes %s  max rel err vs numpy %.2e" % (np.dtype(dt).name, (O, R, I), name,
                                                                               "same" if same else "DIFFER", rel),
                      flush=True)
    print("ALL_EXACT" if ok else "MISMATCH")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
