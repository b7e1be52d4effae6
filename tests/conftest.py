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


@pytest.fixture(scope="session")
def codec():
    """The product binding; on a GPU box a missing library or device is an error, not a skip."""
    import torch

    import sbecodec

    sbecodec.require_device()
    torch.cuda.init()
    return sbecodec
