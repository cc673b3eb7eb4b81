"""Host wait policy A/B on the C2 step (swap + mean + std, float32 (2000,512,512)):
the runtime's stream synchronize (default) vs spinning on hipStreamQuery from C
(ctypes into libamdhip64, GIL released) before the statistic's result is read.
Variants alternate in rounds inside one process; also reports the step's
GPU-idle share (step wall time minus the kernels' event time)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
import bolt_amd as bolt
from bolt_amd import MI355XContext
from bolt_amd.mi355x import array as barray, transfer

dev = torch.device("cuda", 0)
ctx = MI355XContext(device=dev)
shard = bench.synth_shard(torch, (2000, 512, 512), np.float32, dev, 1234)
b = bolt.ConstructMI355X.fromshards(shard, (2000, 512, 512), context=ctx, split=1, dtype=np.float32)
del shard
ops = bench.steps_of("C2", b)

hip = ctypes.CDLL("libamdhip64.so")
hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
hip.hipStreamQuery.restype = ctypes.c_int
NOT_READY = 600  # hipErrorNotReady

orig = transfer.finish_host_result


def spin_finish(host, device, dtype, shape):
    s = ctypes.c_void_p(transfer.current_stream(device).cuda_stream)
    while True:
        rc = hip.hipStreamQuery(s)
        if rc != NOT_READY:
            break
    if rc != 0:
        raise RuntimeError("hipStreamQuery failed: %d" % rc)
    return host.numpy().view(np.dtype(dtype)).reshape(shape)


def torch_spin_finish(host, device, dtype, shape):
    st = transfer.current_stream(device)
    while not st.query():
        pass
    return host.numpy().view(np.dtype(dtype)).reshape(shape)


variants = {"sync": orig, "c_spin": spin_finish, "torch_spin": torch_spin_finish}
ref = None
for name, fn in variants.items():  # warm-up + results identical across policies
    barray.finish_host_result = fn
    for _ in range(3):
        out = [f() for _, f, _ in ops]
    got = [np.asarray(o) for o in out[1:]]
    if ref is None:
        ref = got
    assert all(np.array_equal(a, c) for a, c in zip(ref, got)), name
torch.cuda.synchronize()

steps = 20
res = {k: [] for k in variants}
for rnd in range(7):
    for name, fn in variants.items():
        barray.finish_host_result = fn
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            for _, f, _ in ops:
                r = f()
                del r
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t) / steps * 1e3)
barray.finish_host_result = orig
for name, v in res.items():
    v = np.array(v)
    print("%-11s step median %.4f ms  min %.4f  (%s)" % (name, np.median(v), v.min(),
                                                         " ".join("%.4f" % x for x in v)))
