"""Shared test setup.  `-m "not gpu"` runs on CPU; `-m gpu` needs an MI355X (gfx950)."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP device)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def rq():
    import rqhip
    rqhip.lib()
    return rqhip


@pytest.fixture(scope="session")
def gpu(rq):
    """Device fixture for -m gpu tests: fails loudly (never skips) when no device is usable."""
    import torch
    assert torch.cuda.is_available(), "gpu test needs a HIP device"
    assert rq.device_count() > 0, "librqhip.so sees no HIP device"
    return torch.device("cuda:0")
