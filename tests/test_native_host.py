"""Host-side native checks (no GPU): the FastDiv mul-hi division shared by the
copy kernels (bolt_amd/csrc/bm_common.h) equals integer division exactly."""
import os
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fastdiv_exact():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "fastdiv_check")
        subprocess.run([hipcc, "-O2", "-std=c++17", "--offload-arch=gfx950", "-o", exe, os.path.join(HERE, "native", "fastdiv_check.cpp")],
                       check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert " 0 bad" in r.stdout
