"""Column-kernel numerics of libbolt_mi355x builds against long-double numpy:
mean / var / std over the leading axis (bm_reduce O=1, R rows, I columns) on
plain, offset and outlier data, float32 / float64, shapes that take one and
several row chunks.  Prints each build's worst error in units of the
tolerance (tools/rows_numerics_check.py's rule).

    python tools/cols_numerics_check.py libA.so [libB.so ...]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_bench import load, stream  # noqa: E402

CODES = {np.dtype(np.float32): 10, np.dtype(np.float64): 11}


def main():
    libs = [(p, load(p)) for p in sys.argv[1:]]
    rng = np.random.default_rng(13)
    worst = {p: 0.0 for p, _ in libs}
    ws = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    for dt in (np.float32, np.float64):
        rtol = 1e-6 if dt == np.float32 else 1e-12
        for R, I in ((2000, 65536), (64, 262144), (5000, 1000), (300, 4096), (17, 100000)):
            for kind in ("plain", "offset", "outlier"):
                x = rng.standard_normal((R, I))
                if kind == "offset":
                    x = 1e6 + x
                elif kind == "outlier":
                    x[0] = 100.0
                x = x.astype(dt)
                src = torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy()).cuda()
                xl = x.astype(np.longdouble)
                truth = {0: xl.mean(0), 1: xl.var(0), 2: np.sqrt(xl.var(0))}
                for stat in (0, 1, 2):
                    scale = np.abs(xl).max(0) if stat == 0 else np.abs(truth[stat])
                    for p, lib in libs:
                        out = torch.zeros(I * np.dtype(dt).itemsize, dtype=torch.uint8, device="cuda")
                        rc = lib.bm_reduce(stat, ctypes.c_void_p(src.data_ptr()), CODES[np.dtype(dt)], 1, R, I,
                                           ctypes.c_void_p(out.data_ptr()), CODES[np.dtype(dt)],
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
