"""Soak of the seeded fuzz suites on several ranks over gloo -- on the CPU
with the numpy test executor, or (device cuda:0) every rank on the one GPU
with the HIP kernels and the exchanges staged through the host (the
rehearsal executor: RCCL refuses two ranks on one GPU).  Every rank runs the
same seeded case on a context that
spans the ranks, so arrays are sharded (ragged and empty slabs) and every
exchange path runs -- swaps, sharded statistics, chunk moves (suite
"oracle", tests/test_fuzz_oracle.py), indexing and its row exchanges
("getitem", tests/test_getitem_fuzz.py), chunk chains ("chunk",
tests/test_chunk_fuzz.py), reshapes / squeeze / concatenate /
reductions / map / filter / stacks ("api", tests/test_api_fuzz.py) -- each
compared with the oracle.

    python tools/dist_fuzz_soak.py oracle:2:200:700 getitem:3:0:2000 api:4:0:1000
    BOLT_AMD_SOAK_DEVICE=cuda:0 python tools/dist_fuzz_soak.py getitem:2:0:500
"""
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), HERE]
import torch.multiprocessing as mp  # noqa: E402

from test_dist_gloo import _free_port  # noqa: E402


def _case_fn(suite):
    if suite == "oracle":
        from test_fuzz_oracle import check_case
        return check_case
    if suite == "getitem":
        from test_getitem_fuzz import test_getitem_fuzz
        return test_getitem_fuzz
    if suite == "chunk":
        from test_chunk_fuzz import test_chunk_fuzz
        return test_chunk_fuzz
    from test_api_fuzz import test_api_fuzz
    return test_api_fuzz


def _worker(rank, world, port, errq, suite, seeds):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from bolt_amd import MI355XContext
        import cpu_backend
        device = os.environ.get("BOLT_AMD_SOAK_DEVICE", "cpu")
        if device == "cpu":
            cpu_backend.install()
        else:
            cpu_backend.install_host_staged_gpu()
        ctx = MI355XContext(device=device)
        case = _case_fn(suite)
        ran = skipped = 0
        for seed in seeds:
            try:
                case(ctx, seed)
                ran += 1
            except BaseException as e:  # pytest's skip is a BaseException
                if type(e).__name__ == "Skipped":
                    skipped += 1
                    continue
                raise AssertionError("%s seed %d failed: %s" % (suite, seed, traceback.format_exc()[-2500:]))
        if rank == 0:
            print("  rank 0 on %s (%s): %d cases compared, %d skipped"
                  % (ctx.device, type(ctx.backend).__name__ if hasattr(ctx, "backend") else "-", ran, skipped),
                  flush=True)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        errq.put((rank, traceback.format_exc()))
        raise


def run(suite, world, seeds):
    # fork before anything touches a GPU; spawn when the ranks use one
    ctx = mp.get_context("fork" if os.environ.get("BOLT_AMD_SOAK_DEVICE", "cpu") == "cpu" else "spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, errq, suite, seeds)) for r in range(world)]
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
        suite, world, lo, hi = spec.split(":")
        world, lo, hi = int(world), int(lo), int(hi)
        t0 = time.time()
        errs, codes = run(suite, world, range(lo, hi))
        print("%s world %d seeds %d..%d: %d failed ranks, exit codes %s, %.0f s"
              % (suite, world, lo, hi - 1, len(errs), codes, time.time() - t0), flush=True)
        for rank, tb in errs[:1]:
            print("rank %d:\n%s" % (rank, tb[-4000:]))
        bad += len(errs) + sum(1 for c in codes if c)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:] or ["oracle:2:200:700", "getitem:3:0:500", "api:2:0:300"]))
