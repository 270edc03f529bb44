import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (ROCm GPU)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_runtime():
    """Build the host runtime (g++, seconds) once per session if it is missing."""
    from llm_consensus_amd.utils.native import runtime

    runtime()
    yield


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture
def cuda():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch

    return torch.device("cuda", 0)
