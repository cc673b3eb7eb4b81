"""The drop-in, proven against the reference itself (build container only).

Runs the REFERENCE's own Spark-mode test files (/root/reference/test/spark)
unmodified, plus tests/dropin/test_dropin_factory.py, in a child pytest whose
plugin (tests/dropin/dropin_plugin.py) applies INTEGRATION.md section 2 to the
imported reference bolt: ('mi355x', ConstructMI355X) appended to
bolt.factory.constructors, the lookup mode= fix, bolt_amd's stand-in
base/local/construct modules replaced by bolt's own (so BoltArrayMI355X is a
bolt.base.BoltArray).  The reference tests' `sc` is an MI355XContext on the
CPU test executor, so `array(x, sc)` routes through the reference's
factory.lookup -> ConstructMI355X._argcheck -> ConstructBase.dispatch
(bolt/factory.py:37-83, bolt/construct.py:3-8).  Skipped where the reference
is absent (the GPU box); nothing from it is copied or shipped.
"""
import os
import re
import subprocess
import sys

import pytest

REF = os.environ.get("BOLT_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

# reference tests that cannot hold for any non-Spark mode, with the reason
EXPECTED_FAIL = {
    "test_spark_construct.py::test_array": "asserts isinstance(b, BoltArraySpark) and tordd() partitions",
    "test_spark_functional.py::test_filter": "generic.filter_suite calls ndarray.tostring() on the record; "
                                             "user functions here receive device tensors",
    "test_spark_stacking.py::test_stack_2D": "re-partitions the RDD itself (_rdd.partitionBy)",
    "test_spark_stacking.py::test_stack_3D": "re-partitions the RDD itself (_rdd.partitionBy)",
    "test_spark_stacking.py::test_stacked_map": "re-partitions the RDD itself (_rdd.partitionBy)",
    "test_spark_stacking.py::test_stacked_shape_inference": "re-partitions the RDD itself (_rdd.partitionBy)",
    "test_spark_stacking.py::test_stacked_conversion": "imports pyspark",
}


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "bolt", "spark")), reason="reference not present")
def test_reference_spark_suite_through_the_factory(tmp_path):
    env = dict(os.environ)
    env["PYTHONDONTWRITEBYTECODE"] = "1"  # the reference tree is read-only
    env["PYTHONPATH"] = os.pathsep.join([REF, os.path.join(REF, "test"), HERE, os.path.join(HERE, "dropin"),
                                         ROOT, env.get("PYTHONPATH", "")])
    cmd = [sys.executable, "-m", "pytest", "-p", "no:cacheprovider", "--noconftest", "-p", "dropin_plugin",
           "-q", "-rA", "-W", "ignore", "--rootdir", str(tmp_path),
           os.path.join(REF, "test", "spark"), os.path.join(HERE, "dropin", "test_dropin_factory.py")]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    # "PASSED <path>::<test>": paths outside the child's rootdir print without
    # their file name, so the factory tests are matched by test name
    passed = set(re.findall(r"^PASSED \S*?(test_\w+\.py::\w+)", out, re.M))
    passed |= set("test_dropin_factory.py::" + n
                  for n in re.findall(r"^PASSED \S*::(test_\w+)", out, re.M)
                  if n in ("test_lookup_routes_to_mi355x", "test_ones_zeros_concatenate",
                           "test_statistics_are_bolt_local"))
    failed = set(re.findall(r"^FAILED \S*?(test_\w+\.py::\w+)", out, re.M))
    failed |= set(re.findall(r"^FAILED ::(test_\w+)", out, re.M))
    assert passed, out[-3000:]
    assert failed == set(EXPECTED_FAIL), out[-3000:]
    # the hot-path tests the verdict names, by file
    for name in ("test_spark_shaping.py::test_swap", "test_spark_shaping.py::test_transpose",
                 "test_spark_shaping.py::test_t", "test_spark_shaping.py::test_swapaxes",
                 "test_spark_shaping.py::test_reshape_keys", "test_spark_shaping.py::test_reshape_values",
                 "test_spark_chunking.py::test_chunk", "test_spark_chunking.py::test_unchunk",
                 "test_spark_chunking.py::test_keys_to_values", "test_spark_chunking.py::test_values_to_keys",
                 "test_spark_chunking.py::test_padding", "test_spark_functional.py::test_mean",
                 "test_spark_functional.py::test_var", "test_spark_functional.py::test_std",
                 "test_spark_functional.py::test_sum", "test_spark_functional.py::test_reduce",
                 "test_dropin_factory.py::test_lookup_routes_to_mi355x",
                 "test_dropin_factory.py::test_ones_zeros_concatenate",
                 "test_dropin_factory.py::test_statistics_are_bolt_local"):
        assert name in passed, (name, out[-3000:])
    assert len(passed) >= 62
