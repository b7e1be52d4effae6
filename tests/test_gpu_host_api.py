"""GPU: the C++ host mirror of the reference API (SBEEncoder / MessageParser / decode_ack /
MessageHandler::on_egress / offer_batch) against SURVEY probes and the oracle (tests/cpp), and its
batch pipeline past one chunk with distinct records (tests/cpp/test_host_pipeline.cpp) under
three chunk settings: 4 KiB chunks (thousands of chunks through the 3-slot stream ring), the
defaults (multi-chunk batches above 65536 records, one-chunk batches on the zero-copy path) and
the zero-copy path switched off (every one-chunk batch through the DMA copy engines); and the
small-batch serve kernel (sbe_server_*) taking every one-chunk batch up to 4096 records on one
wave, or none (the defaults: one wave up to 96 records, several workgroups up to 4096)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


ENV_KEYS = ("AERON_AMD_CHUNK_BYTES", "AERON_AMD_ZC_BYTES", "AERON_AMD_SERVE_RECORDS", "AERON_AMD_SERVE_WIDE_RECORDS")
NO_SERVE = {"AERON_AMD_SERVE_RECORDS": "0", "AERON_AMD_SERVE_WIDE_RECORDS": "0"}


@pytest.mark.parametrize("env", [{}, NO_SERVE], ids=["default", "no_serve"])
def test_host_api_binary(codec, env):
    d = os.path.join(HERE, "cpp")
    subprocess.run(["make", "-s", "-C", d, "test_host_api"], check=True)
    e = {k: v for k, v in os.environ.items() if k not in ENV_KEYS}
    e.update(env)
    r = subprocess.run([os.path.join(d, "test_host_api")], capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("env", [{"AERON_AMD_CHUNK_BYTES": "4096"}, {}, {"AERON_AMD_ZC_BYTES": "0"},
                                 {"AERON_AMD_SERVE_RECORDS": "4096"}, NO_SERVE],
                         ids=["chunks4k", "default", "no_zero_copy", "serve4096", "no_serve"])
def test_host_pipeline_multichunk(codec, env):
    d = os.path.join(HERE, "cpp")
    subprocess.run(["make", "-s", "-C", d, "test_host_pipeline"], check=True)
    e = {k: v for k, v in os.environ.items() if k not in ENV_KEYS}
    e.update(env)
    r = subprocess.run([os.path.join(d, "test_host_pipeline")], capture_output=True, text=True, timeout=110, env=e)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host pipeline test: ok" in r.stdout
