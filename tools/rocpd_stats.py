"""Per-kernel statistics from a rocprofv3 rocpd database (run_results.db):
calls, average / median / min ns, total ms, for kernels above 1% of the total.

    python tools/rocpd_stats.py gpurun_out/<dir>/run_results.db [...]
"""
import sqlite3
import statistics
import sys


def stats(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, duration from kernels").fetchall()
    by = {}
    for name, d in rows:
        by.setdefault(name, []).append(d)
    total = sum(sum(v) for v in by.values())
    out = []
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) < 0.01 * total:
            continue
        out.append("%6d  avg %10.0f  med %10.0f  min %10.0f  tot %9.3f ms  %s"
                   % (len(v), sum(v) / len(v), statistics.median(v), min(v), sum(v) / 1e6, name[:110]))
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        for line in stats(p):
            print("  " + line)
