"""Shared pytest setup.  Marker ``gpu``: needs an MI355X (run via gpurun)."""

from __future__ import annotations

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a ROCm GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def emu():
    from tests.helpers import build_emu
    return build_emu()


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
