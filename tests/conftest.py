import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


# tests/dropin/ runs only inside tests/test_reference_dropin.py's child pytest
# (it imports the reference bolt, which the main session must not)
collect_ignore = ["dropin"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libbolt_mi355x.so")


def pytest_collection_modifyitems(config, items):
    """Without a HIP device, tests marked gpu are skipped (not failed), so a plain
    `pytest tests` is green on a CPU-only build host."""
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="needs an MI355X (no HIP device here)")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bolt_amd import MI355XContext
    return MI355XContext(device="cuda:0")


@pytest.fixture(scope="session", params=["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
def bctx(request):
    """A context on the GPU (HIP kernels) or on the CPU test executor (host logic)."""
    from bolt_amd import MI355XContext
    if request.param == "gpu":
        import torch
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        return MI355XContext(device="cuda:0")
    import cpu_backend
    cpu_backend.install()
    return MI355XContext(device="cpu")
