"""Two libbolt_mi355x builds give byte-identical bm_reduce / bm_reduce_rows
outputs over the rows kernel's cases (short rows, chunked long rows, padded
pitches, every dtype the rows kernel reads, mean / var / std / sum / max).

    python tools/rows_peel_check.py libA.so libB.so
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_bench import load, stream  # noqa: E402

CODES = {np.dtype(np.float32): 10, np.dtype(np.float64): 11, np.dtype(np.uint16): 3, np.dtype(np.int32): 6}


def main():
    libs = [load(p) for p in sys.argv[1:3]]
    rng = np.random.default_rng(3)
    bad = n = 0
    for dt in (np.float32, np.float64, np.uint16):
        for O, R, P in ((1000, 2000, 2048), (64, 300000, 300032), (5000, 7, 8), (333, 129, 129), (2, 5000000, 5000000),
                        (4096, 260, 260), (100, 1000, 1000)):
            x = (rng.standard_normal(O * P) * 30 + 1000).astype(dt) if np.dtype(dt).kind == "f" else \
                rng.integers(0, 60000, O * P).astype(dt)
            src = torch.from_numpy(x.view(np.uint8).copy()).cuda()
            ws = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
            for stat in (0, 1, 2, 3, 4):
                keep = stat in (3, 4)
                odt = np.dtype(dt) if keep else (np.dtype(np.float32) if dt == np.float32 else np.dtype(np.float64))
                outs = []
                for lib in libs:
                    out = torch.zeros(O * odt.itemsize, dtype=torch.uint8, device="cuda")
                    if P == R:
                        rc = lib.bm_reduce(stat, ctypes.c_void_p(src.data_ptr()), CODES[np.dtype(dt)], O, R, 1,
                                           ctypes.c_void_p(out.data_ptr()), CODES[odt], ctypes.c_void_p(ws.data_ptr()),
                                           ws.numel(), stream())
                    else:
                        rc = lib.bm_reduce_rows(stat, ctypes.c_void_p(src.data_ptr()), CODES[np.dtype(dt)], O, R, P,
                                                ctypes.c_void_p(out.data_ptr()), CODES[odt],
                                                ctypes.c_void_p(ws.data_ptr()), ws.numel(), stream())
                    assert rc == 0, lib.bm_last_error()
                    torch.cuda.synchronize()
                    outs.append(out.cpu().numpy())
                n += 1
                if outs[0].tobytes() != outs[1].tobytes():
                    bad += 1
                    print("DIFFER", np.dtype(dt), O, R, P, stat, flush=True)
    print("rows_peel_check: %d cases, %d differ" % (n, bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
