"""Shared pytest setup: markers, import paths, seeded helpers.

`-m "not gpu"` runs the oracle-vs-golden, host-logic and C-ABI load tests on CPU;
`-m gpu` runs the HIP parity tests through libzasr.so on an MI355X.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "sherpa-vietnamese-asr_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP parity tests through libzasr.so)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")
