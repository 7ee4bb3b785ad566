import os
import sys

import pytest

try:  # import torch before the HIP library is loaded (see knn_amd.lib())
    import torch  # noqa: F401
except Exception:
    pass

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


def cout_double(x):
    """std::cout << double with default precision (6 significant, %g)."""
    return "%g" % x


@pytest.fixture(scope="session")
def fmt_cout():
    return cout_double
