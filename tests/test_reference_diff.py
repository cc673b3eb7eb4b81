"""bolt_amd against the reference itself on random inputs (build container
only): tools/reference_diff_fuzz.py runs random arrays through random chains
of operations on the reference's Spark mode (over tests/golden's fake RDD) and
on bolt_amd's CPU executor of the kernel contracts, in a child process, and
must report no difference beyond the reference bugs docs/HISTORY.md §4 lists.
Skipped where the reference is absent (the GPU box); nothing from it is copied
or shipped.  (profiles/r05p_reference_diff_fuzz.txt: 12,000 seeds.)

The second test draws length-1 axes too (BOLT_AMD_DIFF_MIN_EXTENT=1): every
result the reference returns must have its shape and split (its swap chain
squeezes unit value axes, plan.swap_shape); where the reference raises and
numpy has an answer, bolt_amd's numpy answer is counted, not failed
(profiles/r06a_reference_diff_unit_axes.txt).
"""
import os
import subprocess
import sys

import pytest

REF = os.environ.get("BOLT_REFERENCE", "/root/reference")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "bolt", "spark")), reason="reference not present")
def test_random_chains_match_the_reference(tmp_path):
    env = dict(os.environ)
    env["PYTHONDONTWRITEBYTECODE"] = "1"  # the reference tree is read-only
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "reference_diff_fuzz.py"), "0", "1500"],
                       env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "seeds 0..1499: 0 failed" in out, out[-4000:]


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "bolt", "spark")), reason="reference not present")
def test_random_chains_with_unit_axes_match_the_reference(tmp_path):
    env = dict(os.environ)
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    env["BOLT_AMD_DIFF_MIN_EXTENT"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "reference_diff_fuzz.py"), "0", "1500"],
                       env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "seeds 0..1499: 0 failed" in out, out[-4000:]


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "bolt", "spark")), reason="reference not present")
@pytest.mark.parametrize("seed,min_extent,op", [(15168, "2", "getitem"), (31731, "1", "getitem"),
                                                (204533, "1", "getitem"),
                                                (60771, "1", "ufunc"), (65282, "2", "ufunc")])
def test_soak_chains_replayed(tmp_path, seed, min_extent, op):
    """Chains of the round-6 soak (930,000 seeds) where the reference's
    answer differed, replayed:
      getitem  a list index on every axis (a plain list on a 1-D array too) of
               an array whose RDD a transpose had shuffled: the reference numbers the selected records in the
               RDD's current order (array.py:552), the partitioner's; bolt_amd
               in key order, the reference's answer on the same array in key
               order (docs/HISTORY.md §4 item 9), which the fuzz compares to;
      ufunc    reduce(np.multiply) of float32 records whose product overflows:
               the reference's treeReduce order makes inf * 0 = NaN where the
               float128 truth is 0; bolt_amd's answer is at least as close to
               the truth (tests/golden_cases.stat_close)."""
    env = dict(os.environ)
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    env["BOLT_AMD_DIFF_MIN_EXTENT"] = min_extent
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "reference_diff_fuzz.py"), str(seed), str(seed + 1)],
                       env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "seeds %d..%d: 0 failed" % (seed, seed) in out and "'%s': 1" % op in out, out[-4000:]
