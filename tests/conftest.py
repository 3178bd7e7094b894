import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import coracle
    coracle.build()
    return coracle


@pytest.fixture(scope="session")
def gpu():
    """Skips when no GPU; on a GPU box the HIP path must load (fail loudly otherwise)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from mcp_amd import _lib
    L = _lib.lib()
    assert L.mcpx_device_count() >= 1
    return L
