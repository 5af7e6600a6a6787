import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(TESTS, "golden")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


def pytest_collection_finish(session):
    """The same ordering for module- and session-scoped fixtures, which run before any function-scoped
    one: if a GPU test is selected, torch's HIP runtime comes up before a fixture can load libfc2.so."""
    if any(it.get_closest_marker("gpu") is not None for it in session.items):
        try:
            import torch
            torch.cuda.is_available()
        except Exception:
            pass


@pytest.fixture(autouse=True)
def _torch_hip_runtime_first(request):
    """One HIP runtime per process: before a GPU test can reach the C ABI, torch's
    runtime is brought up, so that the torch-based tests after a torch-free one still see the device."""
    if request.node.get_closest_marker("gpu") is not None:
        try:
            import torch
            torch.cuda.is_available()
        except Exception:
            pass
    yield
