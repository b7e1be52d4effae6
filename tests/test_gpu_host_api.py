"""GPU: the C++ host mirror of the reference API (SBEEncoder / MessageParser / decode_ack /
MessageHandler::on_egress / offer_batch) against SURVEY probes and the oracle (tests/cpp)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_host_api_binary(codec):
    d = os.path.join(HERE, "cpp")
    subprocess.run(["make", "-s", "-C", d], check=True)
    r = subprocess.run([os.path.join(d, "test_host_api")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
