"""bolt_amd against the reference itself on random inputs (build container
only): tools/reference_diff_fuzz.py runs random arrays through random chains
of operations on the reference's Spark mode (over tests/golden's fake RDD) and
on bolt_amd's CPU executor of the kernel contracts, in a child process, and
must report no difference beyond the reference bugs docs/HISTORY.md §4 lists.
Skipped where the reference is absent (the GPU box); nothing from it is copied
or shipped.  (profiles/r05p_reference_diff_fuzz.txt: 12,000 seeds.)
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
