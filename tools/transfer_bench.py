"""Ingest / egress throughput of the mi355x mode vs a plain pageable torch copy.

    python tools/transfer_bench.py [--mb 2000]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bolt_amd as bolt  # noqa: E402
from bolt_amd.mi355x.transfer import to_device, to_host  # noqa: E402


def best(f, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=2000)
    a = ap.parse_args()
    n = a.mb << 20
    host = np.random.default_rng(0).integers(0, 256, size=n, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    ctx = bolt.MI355XContext(device=dev)
    t_naive_in = best(lambda: torch.from_numpy(host).to(dev))
    t_in = best(lambda: to_device(host, dev))
    d = to_device(host, dev)
    t_naive_out = best(lambda: d.cpu().numpy())
    t_out = best(lambda: to_host(d, np.uint8, (n,)))
    x = host.view(np.float32).reshape(-1, 512, 512)
    t_array = best(lambda: bolt.array(x, ctx))
    b = bolt.array(x, ctx)
    t_toarray = best(lambda: b.toarray())
    gb = n / 1e9
    for name, t in [("H2D torch pageable .to()", t_naive_in), ("H2D bolt_amd staged", t_in),
                    ("D2H torch pageable .cpu()", t_naive_out), ("D2H bolt_amd staged", t_out),
                    ("bolt.array(x) ingest", t_array), ("b.toarray() egress", t_toarray)]:
        print("%-28s %7.3f s  %6.1f GB/s" % (name, t, gb / t), flush=True)


if __name__ == "__main__":
    main()
