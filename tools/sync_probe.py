"""Host wait strategy for statistics results (diagnostic, one GPU).

Times the C2 step (swap((0,),(0,1)) + mean(axis=2) + std(axis=2)) and each
statistic's call + wait, with the blocking stream synchronize (SPIN_US = 0)
against polling the stream (bm_stream_wait), alternating to cancel drift.
Run against a build with bm_stream_wait and transfer.SPIN_US
(profiles/r01_sync_probe.log): no difference -- the runtime's synchronize
already polls -- so neither was kept; on the current tree both legs are the
blocking synchronize.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd.mi355x import transfer  # noqa: E402


def main():
    ctx = bolt.MI355XContext()
    shape = (2000, 512, 512)
    raw = (torch.randn(int(np.prod(shape)), device="cuda") * 50 + 1000).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=1, dtype=np.float32)
    s = b.swap((0,), (0, 1))
    ref_m = s.mean(axis=2).toarray().copy()
    ref_sd = s.std(axis=2).toarray().copy()
    res = {}
    for rep in range(3):
        for spin in (0, 20000):
            transfer.SPIN_US = spin
            for _ in range(3):
                s2 = b.swap((0,), (0, 1)); s2.mean(axis=2); s2.std(axis=2)
            torch.cuda.synchronize()
            ws = []
            for _ in range(30):
                torch.cuda.synchronize()
                t = time.perf_counter()
                m = s.mean(axis=2)
                ws.append(time.perf_counter() - t)
                assert m.toarray().tobytes() == ref_m.tobytes()
            res.setdefault(("mean", spin), []).append(np.median(ws) * 1e6)
            torch.cuda.synchronize()
            K = 40
            t = time.perf_counter()
            for _ in range(K):
                s2 = b.swap((0,), (0, 1)); m = s2.mean(axis=2); sd = s2.std(axis=2)
            torch.cuda.synchronize()
            res.setdefault(("step", spin), []).append((time.perf_counter() - t) / K * 1e6)
            assert sd.toarray().tobytes() == ref_sd.tobytes()
    for k, v in sorted(res.items()):
        print("%-5s spin_us=%-6d %s us" % (k[0], k[1], " ".join("%.1f" % x for x in v)), flush=True)


if __name__ == "__main__":
    main()
