"""CPU soak of the multi-rank oracle fuzz (tests/test_dist_fuzz.py's worker)
over seed ranges beyond the suite's, at several world sizes over gloo with the
numpy test executor: ragged and empty slabs, exchanges, sharded statistics,
each case compared with the oracle.

    python tools/dist_fuzz_soak.py 2:200:700 3:700:1200 8:1700:2700
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), HERE]
import torch.multiprocessing as mp  # noqa: E402

import test_dist_fuzz as T  # noqa: E402
from test_dist_gloo import _free_port  # noqa: E402


def run(world, seeds):
    T.SEEDS = seeds
    ctx = mp.get_context("fork")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=T._worker, args=(r, world, port, errq, "cpu")) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=3000)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    return errs, [p.exitcode for p in procs]


def main(specs):
    bad = 0
    for spec in specs:
        world, lo, hi = (int(v) for v in spec.split(":"))
        t0 = time.time()
        errs, codes = run(world, range(lo, hi))
        print("world %d seeds %d..%d: %d failed ranks, exit codes %s, %.0f s"
              % (world, lo, hi - 1, len(errs), codes, time.time() - t0), flush=True)
        for rank, tb in errs:
            print("rank %d:\n%s" % (rank, tb[-3000:]))
        bad += len(errs) + sum(1 for c in codes if c)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["2:200:700", "3:700:1200"]))
