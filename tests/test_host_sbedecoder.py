"""CPU: the host mirror's SBEDecoder statics and SBEEncoder::get_current_timestamp
(include/aeron_cluster/sbe_messages.hpp:169, :189-247; src/sbe_encoder.cpp:169-323) against
hand-built probes and the oracle restatement (orc_sbedecoder_*), tests/cpp/test_sbedecoder.cpp.
These are host-side struct readers; no device is needed."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_sbedecoder_binary():
    d = os.path.join(HERE, "cpp")
    subprocess.run(["make", "-s", "-C", d, "test_sbedecoder"], check=True)
    r = subprocess.run([os.path.join(d, "test_sbedecoder")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sbedecoder test: ok" in r.stdout
