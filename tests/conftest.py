import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mujoco-panda-pnp_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); runs on the GPU box")


@pytest.fixture(scope="session")
def model():
    from pnp_amd.model import load_model
    return load_model()


@pytest.fixture(scope="session")
def engine():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    from pnp_amd.engine import get_engine
    return get_engine()
