"""Is the C5 chunk pack's bench-to-bench spread the kernel's or the buffers'?

Runs bench.py's main() in this process with every large record gather
(the C5 chunk pack, values_to_keys' repack) followed, on the SAME source and
destination buffers, by a plain 16-B copy of the source bytes into the
destination and the gather again (so the result stays right for the later
ops and checks).  Per call: the first gather, the copy and the second
gather's hipEvent times, and the buffers' addresses -- the copy is the
placement's own ceiling, so gather / copy separates the kernel from the
pages it was handed.

    python tools/c5_place_bench.py [bench.py args ...] > out.json 2> err.log
Prints one JSON line per large gather on stderr (prefix "GATHER ") and
bench.py's own line on stdout.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from bolt_amd.mi355x import _ops, _lib  # noqa: E402

MIN_BYTES = 1 << 32
_orig = _ops.HipBackend.record_gather


def _patched(self, src, src_off, dst, dst_off, nrec, src_rec, dst_rec, rmap, key, es):
    nb = int(nrec) * int(src_rec) * int(es)
    if nb < MIN_BYTES:
        return _orig(self, src, src_off, dst, dst_off, nrec, src_rec, dst_rec, rmap, key, es)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record()
    _orig(self, src, src_off, dst, dst_off, nrec, src_rec, dst_rec, rmap, key, es)
    ev[1].record()
    out_b = int(nrec) * int(dst_rec) * int(es)
    n16 = min(nb, out_b) // 16   # the copy stays inside BOTH buffers
    _lib.check(self.lib.bm_copy_strided(self._ptr(src, src_off), self._ptr(dst, dst_off), 1,
                                        _lib.i64_array([n16]), _lib.i64_array([1]), _lib.i64_array([1]), 16,
                                        self._stream(src)), "bm_copy_strided")
    ev[2].record()
    _orig(self, src, src_off, dst, dst_off, nrec, src_rec, dst_rec, rmap, key, es)
    ev[3].record()
    ev[3].synchronize()
    g1, cp, g2 = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3])
    rec = {"nrec": int(nrec), "src_rec": int(src_rec), "dst_rec": int(dst_rec),
           "src": hex(self._ptr(src, src_off)), "dst": hex(self._ptr(dst, dst_off)),
           "gather_ms": round(g1, 4), "copy_ms": round(cp, 4), "gather2_ms": round(g2, 4),
           "gather_frac": round((nb + out_b) / (g1 * 1e-3) / 8e12, 4),
           "copy_frac": round(2 * n16 * 16 / (cp * 1e-3) / 8e12, 4)}
    sys.stderr.write("GATHER " + json.dumps(rec) + "\n")
    sys.stderr.flush()


_ops.HipBackend.record_gather = _patched

if __name__ == "__main__":
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    sys.exit(bench.main())
