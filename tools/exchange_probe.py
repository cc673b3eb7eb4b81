"""Local work of the multi-GPU swap exchange, timed on ONE GPU (diagnostic).

    python tools/exchange_probe.py

Rank 0 of a G-rank C2 job (float32 (2000*G, 512, 512), swap((0,),(0,1))):
dist.permute_sharded runs its pack and unpack kernels for every stage as in
production, with the all-to-all replaced by handing back a buffer of the
received size (no communication).  Reports the pack + unpack time per swap and
its HBM rate: the part of the exchange that must hide under the xGMI transfer.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bolt_amd.mi355x import dist  # noqa: E402
from bolt_amd.mi355x._ops import backend_for  # noqa: E402
from bolt_amd.mi355x.context import MI355XContext  # noqa: E402


class FakeCtx(MI355XContext):
    def __init__(self, G):
        super().__init__(device=torch.device("cuda", 0))
        self.world_size, self.rank = G, 0


def main():
    dev = torch.device("cuda", 0)
    be = backend_for(dev)

    def fake_a2a(ctx, send, send_sizes, recv_sizes, unit=1, async_op=False):
        recv = dist._empty(sum(recv_sizes), send.device)
        return (recv, None) if async_op else recv

    dist.all_to_all_bytes = fake_a2a
    for G in (2, 4, 8):
        ctx = FakeCtx(G)
        shape = (2000 * G, 512, 512)
        data = torch.empty(2000 * 512 * 512 * 4, dtype=torch.uint8, device=dev)
        perm = (1, 2, 0)
        dist.permute_sharded(ctx, be, data, shape, perm, 4)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            dist.permute_sharded(ctx, be, data, shape, perm, 4)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        ms = float(np.median(ts)) * 1e3
        nb = 4 * data.numel()  # pack reads + writes the slab, unpack reads + writes it
        print("G=%d  pack+unpack (all stages) %.3f ms  %.1f GB/s of HBM traffic" % (G, ms, nb / ms / 1e6),
              flush=True)
        del data


if __name__ == "__main__":
    main()
