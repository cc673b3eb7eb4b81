"""Rows-kernel numerics of libbolt_mi355x builds against float64 / long-double
numpy: mean / var / std over rows (bm_reduce I=1 and bm_reduce_rows with a
pitch) on offset, outlier and plain data, rows from 7 to 300000 elements
(chunked rows included).  Prints each build's worst error in units of the
tolerance (tests/golden_cases.stat_close's scale: rtol 1e-6 float32 /
1e-12 float64 of max|x| for the mean, of the variance for var / std).

    python tools/rows_numerics_check.py libA.so [libB.so ...]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_bench import load, stream  # noqa: E402

CODES = {np.dtype(np.float32): 10, np.dtype(np.float64): 11}


def data(kind, O, P, dt, rng):
    x = rng.standard_normal((O, P))
    if kind == "offset":
        x = 1e6 + x
    elif kind == "outlier":
        x[:, 0] = 100.0
    return x.astype(dt)


def main():
    libs = [(p, load(p)) for p in sys.argv[1:]]
    rng = np.random.default_rng(11)
    worst = {p: 0.0 for p, _ in libs}
    ws = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    for dt in (np.float32, np.float64):
        rtol = 1e-6 if dt == np.float32 else 1e-12
        for O, R, P in ((512, 2000, 2048), (300, 300, 320), (100, 700, 704), (8, 300000, 300032), (2000, 7, 8),
                        (64, 520, 520), (64, 1100, 1100)):
            for kind in ("plain", "offset", "outlier"):
                x = data(kind, O, P, dt, rng)
                src = torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy()).cuda()
                xl = x[:, :R].astype(np.longdouble)
                truth = {0: xl.mean(1), 1: xl.var(1), 2: np.sqrt(xl.var(1))}
                for stat in (0, 1, 2):
                    scale = np.abs(xl).max(1) if stat == 0 else np.abs(truth[stat])
                    for p, lib in libs:
                        out = torch.zeros(O * np.dtype(dt).itemsize, dtype=torch.uint8, device="cuda")
                        if P == R:
                            rc = lib.bm_reduce(stat, ctypes.c_void_p(src.data_ptr()), CODES[np.dtype(dt)], O, R, 1,
                                               ctypes.c_void_p(out.data_ptr()), CODES[np.dtype(dt)],
                                               ctypes.c_void_p(ws.data_ptr()), ws.numel(), stream())
                        else:
                            rc = lib.bm_reduce_rows(stat, ctypes.c_void_p(src.data_ptr()), CODES[np.dtype(dt)], O, R,
                                                    P, ctypes.c_void_p(out.data_ptr()), CODES[np.dtype(dt)],
                                                    ctypes.c_void_p(ws.data_ptr()), ws.numel(), stream())
                        assert rc == 0, lib.bm_last_error()
                        torch.cuda.synchronize()
                        got = out.cpu().numpy().view(dt).astype(np.longdouble)
                        err = np.abs(got - truth[stat]) / (rtol * scale + np.spacing(dt(np.abs(truth[stat]))))
                        worst[p] = max(worst[p], float(err.max()))
    for p, _ in libs:
        print("%-40s worst error / tolerance %.3f %s" % (p.split("/")[-1], worst[p], "ok" if worst[p] <= 1 else "FAIL"))
    return 0 if all(v <= 1 for v in worst.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
