import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "zkevm-prover_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the libzkgpu C-ABI)")
    config.addinivalue_line("markers", "slow: large CPU case")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as oc
    oc.lib()
    return oc


@pytest.fixture(scope="session")
def zkgpu():
    """The product library (HIP path); GPU tests only."""
    import zkgpu as z
    z.init()
    return z
