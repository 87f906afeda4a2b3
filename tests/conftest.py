import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))

REF_TEST = "/root/reference/test"
# The GPU box has no /root/reference: tests that need the reference's mesh files use the copies
# the product ships under data/ (identical bytes, checked by test_data_copies when the
# reference is present).
DATA = os.path.join(ROOT, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(HERE, "golden")
