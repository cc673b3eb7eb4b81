"""A Spark ``local[N]`` analogue of the oracle, for bench.py's CPU baseline.

TEST INFRASTRUCTURE ONLY (imported by bench.py's cpu_baseline leg and tests/;
never by bolt_amd).  Spark ``local[N]`` cannot run here (no JVM, no pyspark;
SURVEY.md 8(c)), so this runs the oracle's record-level restatement
(oracle/bolt_oracle.py) with Spark's stage structure on N host processes:
one task per partition, tasks of a stage spread over a pool of N workers,
shuffles through the parent with the records pickled both ways (what PySpark's
shuffle write / read does to them).

The C2 step, swap((0,), (0, 1)) then mean(axis=2) and std(axis=2):

  stage 1  N tasks, one per input partition (parallelize's contiguous split,
           spark/construct.py:69): ChunkedArray._chunk's flatMap
           (chunk.py:131-142) and keys_to_values' _relabel (chunk.py:240-246);
           the records are bucketed by partitionBy's key (chunk.py:251-261:
           one partition per (stationary keys, chunk ids) group).
  stage 2  one task per group: _rebuild (chunk.py:266-280), values_to_keys
           (chunk.py:291-347) and unchunk (chunk.py:146-200; after the swap the
           plan equals the value shape, so no second shuffle).
  stats    _align (array.py:85-115) swaps the time axis back into the keys:
           every key axis moves, so keys_to_values' partitionBy has ONE group
           and the whole stage -- and each StatCounter pass
           (statcounter.py:51-99, treeReduce array.py:321-323) -- is a single
           task in the reference too.  It runs in the parent.

Arithmetic and record contents are the oracle's; only the scheduling is
parallel.  Returns the statistics and the wall time of each phase.
"""
import multiprocessing as mp
import time

import numpy as np

from oracle import bolt_oracle as O

_STATE = {}  # the input partitions, inherited by forked workers (no pickling of the input)


def _stage1(i):
    """Map side of shuffle #1 for input partition i: chunk + relabel + bucket."""
    rs, kaxes = _STATE["rs"], _STATE["kaxes"]
    part = O.RecSet([rs.parts[i]], rs.shape, rs.split, rs.dtype)
    cs = O.chunk(part, _STATE["size"])
    split = cs.split
    kmask = np.zeros(split, dtype=bool)
    kmask[list(kaxes)] = True
    ksize = cs.kshape[kmask]
    buckets = {}
    for k, v in cs.records():
        keys, chks = np.asarray(k[:split]), tuple(k[split:])
        mov, sta = keys[kmask], keys[~kmask]
        gk = tuple(int(s) for s in sta) + tuple(int(m) for m in mov // ksize) + chks
        buckets.setdefault(gk, []).append((k, v))
    meta = (cs.shape, cs.split, cs.dtype, cs.plan, cs.padding)
    return meta, buckets


def _stage2(args):
    """Reduce side of shuffle #1 for one group: rebuild, values_to_keys, unchunk."""
    meta, recs = args
    kaxes, vaxes = _STATE["kaxes"], _STATE["vaxes"]
    shape, split, dtype, plan, padding = meta
    cs = O.ChunkSet([recs], shape, split, dtype, plan, padding)
    c = O.keys_to_values(cs, kaxes)
    c = O.values_to_keys(c, [v + len(kaxes) for v in vaxes])
    if not np.array_equal(c.plan, c.vshape):
        raise NotImplementedError("swap needs unchunk's second shuffle; only the BASELINE C2 swap is staged")
    out = O.unchunk(c)
    return out.records(), out.shape, out.split


def c2_step(x, kaxes=(0,), vaxes=(0, 1), stat_axis=2, workers=8, npartitions=8, size="150"):
    """swap(kaxes, vaxes) + mean / std over ``stat_axis`` on ``workers`` host
    processes.  Returns (mean, std, {phase: seconds}, tasks per stage)."""
    rs = O.parallelize(x, axis=(0,), npartitions=npartitions)
    _STATE.update(rs=rs, kaxes=list(kaxes), vaxes=list(vaxes), size=size)
    ctx = mp.get_context("fork")
    t = {}
    try:
        with ctx.Pool(workers) as pool:
            t0 = time.perf_counter()
            s1 = pool.map(_stage1, range(npartitions), chunksize=1)
            groups = {}
            for meta, buckets in s1:
                for gk, recs in buckets.items():
                    groups.setdefault(gk, []).extend(recs)
            del s1
            t1 = time.perf_counter()
            tasks = [(meta, groups[gk]) for gk in sorted(groups)]
            ngroups = len(tasks)
            s2 = pool.map(_stage2, tasks, chunksize=1)
            del tasks, groups
            t2 = time.perf_counter()
    finally:
        _STATE.clear()
    # the swapped records stay in their stage-2 partitions
    shape, split = s2[0][1], s2[0][2]
    sw = O.RecSet([r for r, _, _ in s2], shape, split, x.dtype)
    del s2
    t3 = time.perf_counter()
    mean = O.stat(sw, "mean", axis=stat_axis)
    t4 = time.perf_counter()
    std = O.stat(sw, "stdev", axis=stat_axis)
    t5 = time.perf_counter()
    t.update(stage1=t1 - t0, stage2=t2 - t1, collect=t3 - t2, mean=t4 - t3, std=t5 - t4, total=t5 - t0)
    return mean, std, t, {"stage1": npartitions, "stage2": ngroups, "stats": 1}
