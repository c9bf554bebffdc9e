import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(autouse=True)
def _fault_tracebacks(request):
    """The HIP runtime installs its own SIGSEGV handler when it initialises, replacing faulthandler's: re-arm
    faulthandler before every GPU test, so a host crash prints the Python stack of every thread."""
    if request.node.get_closest_marker("gpu") is not None:
        import faulthandler

        faulthandler.enable(all_threads=True)
    yield
