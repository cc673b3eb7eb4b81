"""The C2 statistics alone (diagnostic for PMC passes): swap once, then
mean(axis=2) and std(axis=2) three times each on float32 (512, 512, 2000)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402

ctx = bolt.MI355XContext()
shape = (2000, 512, 512)
raw = (torch.randn(int(np.prod(shape)), device="cuda") * 50 + 1000).view(torch.uint8)
b = bolt.ConstructMI355X.fromshards(raw, shape, context=ctx, split=1, dtype=np.float32)
s = b.swap((0,), (0, 1))
for _ in range(3):
    s.mean(axis=2)
    s.std(axis=2)
torch.cuda.synchronize()
print("ok")
