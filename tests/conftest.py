import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "aeron-cluster-client-cpp_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; parity tests of the HIP codec")
    config.addinivalue_line("markers", "late: runs after every other test (multi-threaded harness tests, so a "
                                       "harness stall under -x cannot keep the parity tests from running)")


def pytest_collection_modifyitems(session, config, items):
    # stable: the late tests keep their relative order, after everything else
    items[:] = [it for it in items if it.get_closest_marker("late") is None] + \
               [it for it in items if it.get_closest_marker("late") is not None]


@pytest.fixture(scope="session")
def codec():
    """The product binding; on a GPU box a missing library or device is an error, not a skip."""
    import torch

    import sbecodec

    sbecodec.require_device()
    torch.cuda.init()
    return sbecodec
