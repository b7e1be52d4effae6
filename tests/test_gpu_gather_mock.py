"""GPU: the product's multi-rank gather (sbe_gather_encoded: size all-gather, grouped
ncclSend / ncclRecv into the root's prefix offsets, offset rebase) at world 2 / 3 / 4 / 8 on one
device, the ranks as threads and RCCL replaced by the test stand-in tests/mock_rccl (the product
loads it only because SBE_RCCL_LIB names it).  The root's stream and offsets must equal a
single-batch encode of the whole batch (oracle), for roots other than 0, zero-record shards and
both SBE_ENOSPC limits (tests/cpp/test_gather_mock.cpp)."""
import os
import subprocess

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.late, pytest.mark.timeout(200)]
HERE = os.path.dirname(os.path.abspath(__file__))


def test_gather_multi_rank_mock(codec):
    d = os.path.join(HERE, "cpp")
    subprocess.run(["make", "-s", "-C", d, "test_gather_mock", "../mock_rccl/libmock_rccl.so"], check=True)
    # every wait inside the stand-in gives up after 30 s and reports the world's state (stderr)
    env = dict(os.environ, SBE_RCCL_LIB=os.path.join(HERE, "mock_rccl", "libmock_rccl.so"),
               SBE_MOCK_DEADLINE_S="30")
    r = subprocess.run([os.path.join(d, "test_gather_mock")], capture_output=True, text=True, timeout=150, env=env)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr[-20000:]
    assert "gather mock test: ok" in r.stdout
    # 20 cases (plain + sized), each well inside the limit
    assert r.stdout.count(" -> ok (") == 20, r.stdout
