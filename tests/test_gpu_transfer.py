"""Staged host <-> HBM transfers (bolt_amd/mi355x/transfer.py): byte-exact round
trips across the small / chunked boundaries and odd sizes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 4095, (8 << 20) - 1, (8 << 20) + 1, (64 << 20) * 3 + 12345])
def test_round_trip(n):
    import torch
    from bolt_amd.mi355x.transfer import to_device, to_host
    rng = np.random.default_rng(n)
    host = rng.integers(0, 256, size=n, dtype=np.uint8)
    dev = to_device(host, torch.device("cuda", 0))
    assert dev.numel() == n and dev.device.type == "cuda"
    back = to_host(dev, np.uint8, (n,))
    assert back.tobytes() == host.tobytes()
    if n % 8 == 0 and n:
        assert to_host(dev, np.float64, (n // 8,)).tobytes() == host.tobytes()
