"""Host-side time of one statistic call on the GPU (cProfile over 200 calls of
C2's mean over time): what the GPU waits for between kernels."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd import MI355XContext  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = MI355XContext(device=dev)
    shard = (1000 + 50 * torch.randn(200 * 512 * 512, device=dev)).view(torch.uint8)
    b = bolt.ConstructMI355X.fromshards(shard, (200, 512, 512), context=ctx, split=1, dtype=np.float32)
    s = b.swap((0,), (0, 1))
    for _ in range(20):
        s.mean(axis=2)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        s.mean(axis=2)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
