"""Test configuration.

Markers: ``gpu`` -- needs an MI355X (run with ``-m gpu``); everything else
runs on the CPU-only build container in a few minutes.
"""
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
PROJECT = REPO / "3d-navigation-reinforcement-learning_amd"
for p in (str(REPO), str(PROJECT)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = REPO / "tests" / "golden"
REFERENCE = Path(os.environ.get("VOXNAV_REFERENCE", "/root/reference"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False
