"""Host-path probe of the C1 step (float64 (100,64,64), swap + sum/mean/var/std
at axis None and 0): wall time per op on one GPU after warm-up, the kernels each
op launches (rocprofv3 not needed: torch.profiler is not used either -- plain
wall clock around each call), and a cProfile of the step's host side."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
import bolt_amd as bolt
from bolt_amd import MI355XContext

ctx = MI355XContext(device="cuda:0")
x = np.random.default_rng(0).standard_normal((100, 64, 64))
b = bolt.array(x, ctx, axis=(0,))
ops = bench.steps_of("C1", b)
for _ in range(50):
    for _, f, _ in ops:
        f()
torch.cuda.synchronize()
reps = 300
for name, f, _ in ops:
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    print("%-10s %8.1f us" % (name, (time.perf_counter() - t) / reps * 1e6))
t = time.perf_counter()
for _ in range(reps):
    for _, f, _ in ops:
        f()
torch.cuda.synchronize()
print("step       %8.1f us" % ((time.perf_counter() - t) / reps * 1e6))
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    for _, f, _ in ops:
        f()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
