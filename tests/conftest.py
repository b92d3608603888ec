import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: multi-second CPU case")


@pytest.fixture(autouse=True)
def _torch_hip_first(request):
    """GPU tests: torch's HIP runtime initialises before librfx creates its first context (some tests hand torch
    device memory to the C-ABI after building renderers)."""
    if request.node.get_closest_marker("gpu"):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
