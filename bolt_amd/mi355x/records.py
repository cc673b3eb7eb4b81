"""Host view of an array's records, for inspection and parity tests.

The Spark path exposes its records through ``tordd()`` (array.py:1016-1020,
chunk.py:638-646) and the reference tests read them back with
``.sortByKey().collect()`` / ``.values().collect()``.  ``RecordView`` offers
those few read-only calls over a host copy of the records (already in key
order), so such checks read the same against the mi355x mode.
"""


class RecordView(object):

    def __init__(self, records, npartitions=1, cached=False):
        self._records = list(records)
        self._npartitions = npartitions
        self.is_cached = cached

    def map(self, func):
        return _ListView([func(kv) for kv in self._records])

    def mapValues(self, func):
        return RecordView([(k, func(v)) for k, v in self._records], self._npartitions)

    def collect(self):
        return list(self._records)

    def sortByKey(self):
        return RecordView(sorted(self._records, key=lambda kv: kv[0]), self._npartitions)

    def values(self):
        return RecordView([(None, v) for _, v in self._records], self._npartitions)._vals()

    def _vals(self):
        return _ListView([v for _, v in self._records])

    def keys(self):
        return _ListView([k for k, _ in self._records])

    def count(self):
        return len(self._records)

    def first(self):
        return self._records[0]

    def getNumPartitions(self):
        return self._npartitions


class _ListView(object):

    def __init__(self, items):
        self._items = items

    def collect(self):
        return list(self._items)

    def count(self):
        return len(self._items)

    def first(self):
        return self._items[0]
