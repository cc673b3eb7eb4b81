"""Attribution probe for k_red_rows' PMC over-fetch (diagnostic, PMC passes only).

mean(axis=1) over float32 (262144, R) for R = 2000 (C2's 8000-B rows: every
other row starts mid 128-B line) and R = 2048 (8192-B rows: line aligned),
three launches each.  If the measured FETCH_SIZE excess over N*s disappears at
R = 2048, the C2 excess is the shared boundary lines of unaligned rows (and
the gfx950 FETCH_SIZE doubling applied to their half-line reads)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402

ctx = bolt.MI355XContext()
for R in (2000, 2048):
    shape = (262144, R)
    raw = (torch.randn(int(np.prod(shape)), device="cuda") * 50 + 1000).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=1, dtype=np.float32)
    for _ in range(3):
        b.mean(axis=1)
    torch.cuda.synchronize()
    del b, raw
    torch.cuda.empty_cache()
print("ok")
