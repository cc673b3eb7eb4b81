"""oracle/spark_local.py -- the Spark local[N] analogue behind bench.py's
cpu_baseline.spark_local8 -- computes exactly what the one-process oracle
computes (same records, same StatCounter order), only scheduled over N
host processes."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_local_n_matches_oracle():
    sys.path.insert(0, ROOT)
    from oracle import bolt_oracle as O
    from oracle import spark_local as SL
    rng = np.random.default_rng(0)
    x = (1000 + 50 * rng.standard_normal((96, 40, 24))).astype(np.float32)
    m, s, t, tasks = SL.c2_step(x, workers=4, size="1")   # 1 KB chunks: several reduce groups
    rs = O.parallelize(x, axis=(0,), npartitions=8)
    sw = O.swap(rs, (0,), (0, 1), size="1")
    assert tasks["stage1"] == 8 and tasks["stage2"] > 1
    assert np.array_equal(m, O.stat(sw, "mean", axis=2))
    assert np.array_equal(s, O.stat(sw, "stdev", axis=2))
    assert t["total"] > 0


def test_bench_local8_fields():
    sys.path.insert(0, ROOT)
    import bench
    x = np.ones((16, 8, 8), np.float32)
    r = bench.spark_local8_baseline(x, np.float32, workers=2)
    assert r["cores"] == 2 and r["kind"].startswith("port, local[2]") and r["value"] > 0
