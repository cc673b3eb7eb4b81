import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libbolt_mi355x.so")


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
