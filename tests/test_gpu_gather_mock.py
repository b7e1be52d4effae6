"""GPU: the product's multi-rank gather (sbe_gather_encoded: size all-gather, grouped
ncclSend / ncclRecv into the root's prefix offsets, offset rebase) at world 2 / 3 / 4 / 8 on one
device, the ranks as threads and RCCL replaced by the test stand-in tests/mock_rccl (the product
loads it only because SBE_RCCL_LIB names it).  The root's stream and offsets must equal a
single-batch encode of the whole batch (oracle), for roots other than 0, zero-record shards and
both SBE_ENOSPC limits (tests/cpp/test_gather_mock.cpp)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_gather_multi_rank_mock(codec):
    d = os.path.join(HERE, "cpp")
    subprocess.run(["make", "-s", "-C", d, "test_gather_mock", "../mock_rccl/libmock_rccl.so"], check=True)
    env = dict(os.environ, SBE_RCCL_LIB=os.path.join(HERE, "mock_rccl", "libmock_rccl.so"))
    r = subprocess.run([os.path.join(d, "test_gather_mock")], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gather mock test: ok" in r.stdout
