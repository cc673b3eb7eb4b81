"""Shim so bolt's ConstructSpark._argcheck (spark/construct.py:180-190) routes
to the spark mode with the in-process FakeContext (golden generation only)."""
from fakerdd import FakeContext as SparkContext  # noqa: F401
from fakerdd import FakeRDD as RDD  # noqa: F401
