"""toarray() egress of a row-padded array (round 6: windowed compaction into
the host result, array.py _padded_to_host) against a dense array of the same
bytes, C2 size: b = (2000, 512, 512) float32, s = b.swap((0,), (0, 1)) stored
at 8192-B rows.  3 calls each, GB/s of result bytes, bytes checked against
a torch permute of the source.

    python tools/egress_padded_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd.mi355x.construct import ConstructMI355X  # noqa: E402

ctx = bolt.MI355XContext(device="cuda:0")
g = torch.Generator(device="cuda")
g.manual_seed(1)
x = torch.randn((2000, 512, 512), generator=g, device="cuda", dtype=torch.float32)
b = ConstructMI355X.fromshards(x, (2000, 512, 512), context=ctx, split=1, dtype=np.float32)
s = b.swap((0,), (0, 1))
print("swap result padded:", "_pbuf" in s.__dict__, "pitch", s.__dict__.get("_pitch"), flush=True)
ref = x.permute(1, 2, 0).contiguous()
probe_idx = torch.arange(0, ref.numel(), 9973, device="cuda")
probe = ref.reshape(-1)[probe_idx].cpu().numpy()
sd = b.swap((0,), (0, 1))
sd._data  # noqa: B018  (compacts: a dense array of the same bytes)
dense = ConstructMI355X.fromshards(sd._data.view(torch.float32).view(512, 512, 2000), (512, 512, 2000),
                                   context=ctx, split=2, dtype=np.float32)
del sd
nbytes = ref.numel() * 4
for name, arr in (("dense", dense), ("padded", s)):
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h = arr.toarray()
        dt = time.perf_counter() - t0
        ok = np.array_equal(h.reshape(-1)[probe_idx.cpu().numpy()], probe)
        print("%-7s call %d: %6.1f GB/s %s" % (name, i, nbytes / dt / 1e9, "ok" if ok else "MISMATCH"), flush=True)
        del h
