"""Shared pytest setup: markers, repo paths, and the oracle (test infrastructure only)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle20():
    from oracle.oracle import Oracle
    return Oracle(20, 4, 5)


@pytest.fixture(scope="session")
def oracle7():
    from oracle.oracle import Oracle
    return Oracle(7, 2, 5)


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False
