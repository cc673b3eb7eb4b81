"""Host-path A/B of the C2 step (diagnostic, one GPU): the step (swap +
mean + std, each statistic returned to the host) timed with the package
imported from TREE (argv[1]); run alternately for two trees in fresh
processes.  Prints ms per step (median of REPS x STEPS).

    python tools/host_ab.py <tree with bolt_amd/> [reps] [steps]
"""
import os
import statistics
import sys
import time

tree = os.path.abspath(sys.argv[1])
sys.path.insert(0, tree)
os.environ.setdefault("BOLT_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                    "bolt_amd", "libbolt_mi355x.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bolt_amd as bolt  # noqa: E402
from bolt_amd import MI355XContext  # noqa: E402

assert os.path.dirname(os.path.dirname(os.path.abspath(bolt.__file__))) == tree, bolt.__file__
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
dev = torch.device("cuda", 0)
ctx = MI355XContext(device=dev)
shape = (2000, 512, 512)
g = torch.Generator(device=dev)
g.manual_seed(1234)
x = torch.randn(shape, generator=g, device=dev).mul_(50).add_(1000)
b = bolt.ConstructMI355X.fromshards(x, shape, context=ctx, split=1, dtype=np.float32)
del x


def step():
    s = b.swap((0,), (0, 1))
    s.mean(axis=2)
    s.std(axis=2)


for _ in range(5):
    step()
torch.cuda.synchronize()
ms = []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms.append((time.perf_counter() - t0) / steps * 1e3)
tag = (os.path.basename(tree.rstrip("/")) or tree) + " pitch=" + os.environ.get("BOLT_AMD_ROW_PITCH", "1")
print("%s ms/step median %.4f  min %.4f  all %s" % (tag, statistics.median(ms), min(ms),
                                                    " ".join("%.4f" % m for m in ms)), flush=True)
