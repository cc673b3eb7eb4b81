"""In-process stand-in for the few pyspark RDD calls bolt's Spark path makes.

Used ONLY by tests/golden/make_golden.py, in the build container, to run the
reference bolt's Spark-mode code (which needs a SparkContext) and record its
outputs as fixtures.  It models Spark's partitioning the way local[N] does:
contiguous parallelize slices, hash-bucketed partitionBy keeping input order,
per-partition then cross-partition treeReduce.
"""
import copy
from functools import reduce as _reduce


class FakeRDD(object):

    def __init__(self, parts, ctx):
        self._parts = [list(p) for p in parts]
        self.context = ctx

    # transformations
    def mapPartitionsWithIndex(self, f, preservesPartitioning=False):
        return FakeRDD([list(f(i, iter(p))) for i, p in enumerate(self._parts)], self.context)

    def mapPartitions(self, f, preservesPartitioning=False):
        return FakeRDD([list(f(iter(p))) for p in self._parts], self.context)

    def map(self, f, preservesPartitioning=False):
        return FakeRDD([[f(x) for x in p] for p in self._parts], self.context)

    def flatMap(self, f, preservesPartitioning=False):
        return FakeRDD([[y for x in p for y in f(x)] for p in self._parts], self.context)

    def mapValues(self, f):
        return FakeRDD([[(k, f(v)) for k, v in p] for p in self._parts], self.context)

    def filter(self, f):
        return FakeRDD([[x for x in p if f(x)] for p in self._parts], self.context)

    def values(self):
        return FakeRDD([[v for _, v in p] for p in self._parts], self.context)

    def keys(self):
        return FakeRDD([[k for k, _ in p] for p in self._parts], self.context)

    def partitionBy(self, numPartitions, partitionFunc=hash):
        parts = [[] for _ in range(numPartitions)]
        for p in self._parts:
            for kv in p:
                parts[int(partitionFunc(kv[0])) % numPartitions].append(kv)
        return FakeRDD(parts, self.context)

    def sortByKey(self, ascending=True, numPartitions=None, keyfunc=lambda x: x):
        allrec = [kv for p in self._parts for kv in p]
        return FakeRDD([sorted(allrec, key=lambda kv: keyfunc(kv[0]), reverse=not ascending)], self.context)

    def union(self, other):
        return FakeRDD(self._parts + other._parts, self.context)

    def join(self, other):
        right = {}
        for p in other._parts:
            for k, v in p:
                right.setdefault(k, []).append(v)
        out = []
        for p in self._parts:
            for k, v in p:
                for w in right.get(k, []):
                    out.append((k, (v, w)))
        return FakeRDD([out], self.context)

    def zipWithIndex(self):
        i, parts = 0, []
        for p in self._parts:
            q = []
            for x in p:
                q.append((x, i))
                i += 1
            parts.append(q)
        return FakeRDD(parts, self.context)

    def repartition(self, n):
        return self.context.parallelize([x for p in self._parts for x in p], n)

    def cache(self):
        return self

    def unpersist(self):
        return self

    # actions
    def collect(self):
        return [x for p in self._parts for x in p]

    def count(self):
        return sum(len(p) for p in self._parts)

    def first(self):
        for p in self._parts:
            if p:
                return p[0]
        raise ValueError("RDD is empty")

    def take(self, n):
        return self.collect()[:n]

    def getNumPartitions(self):
        return len(self._parts)

    def treeReduce(self, f, depth=2):
        partials = [_reduce(f, p) for p in self._parts if p]
        if not partials:
            raise ValueError("Cannot reduce empty RDD.")
        return _reduce(f, partials)

    def reduce(self, f):
        return self.treeReduce(f)


class FakeContext(object):

    def __init__(self, defaultParallelism=2):
        self.defaultParallelism = defaultParallelism

    def parallelize(self, data, numSlices=None):
        data = list(data)
        n = numSlices or self.defaultParallelism
        L = len(data)
        return FakeRDD([data[i * L // n:(i + 1) * L // n] for i in range(n)], self)
