import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stage-indexorganized_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def gpu():
    """Fail -- not skip -- when a gpu-marked test runs without a HIP device or library."""
    import stage
    n = stage.device_count()
    if n < 1:
        pytest.fail("no HIP device visible to libstage_hip.so")
    return n
