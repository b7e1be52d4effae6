"""CPU: every C / C++ snippet of INTEGRATION.md (the boundary document) compiles verbatim against
include/sbecodec.h and aeron-cluster-client-cpp_amd/host/aeron_cluster_amd.hpp.

Each ```cpp block is tagged <!-- snippet: NAME --> and pasted unchanged into the context function
snippet_NAME of tests/cpp/test_integration_snippets.cpp (g++ -fsyntax-only, compile only).  A block
without a tag, or a tag without a context function, fails the test, so the document cannot drift
from the ABI it documents (a 10-argument sbe_gather_encoded call against an 11-argument
ABI)."""
import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def snippets():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    out, untagged = {}, []
    for m in re.finditer(r"(?:<!-- snippet: (\w+) -->\n)?```(cpp|c)\n(.*?)```", text, re.S):
        name, body = m.group(1), m.group(3)
        if not name:
            untagged.append(body.splitlines()[0] if body else "")
            continue
        assert name not in out, f"duplicate snippet tag {name}"
        out[name] = body
    return out, untagged


def test_every_snippet_is_tagged():
    snips, untagged = snippets()
    assert not untagged, f"INTEGRATION.md has C/C++ blocks without a snippet tag: {untagged}"
    assert len(snips) >= 6


def test_snippets_compile(tmp_path):
    snips, _ = snippets()
    src = os.path.join(HERE, "cpp", "test_integration_snippets.cpp")
    ctx = open(src).read()
    wanted = set(re.findall(r'#include "snip_(\w+)\.inc"', ctx))
    assert wanted == set(snips), f"context functions {sorted(wanted)} != tagged snippets {sorted(snips)}"
    for name, body in snips.items():
        (tmp_path / f"snip_{name}.inc").write_text(body)
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wno-unused-variable", "-Wno-unused-but-set-variable",
           "-D__HIP_PLATFORM_AMD__", f"-I{tmp_path}", f"-I{os.path.join(ROOT, 'include')}",
           f"-I{os.path.join(ROOT, 'aeron-cluster-client-cpp_amd', 'host')}", "-I/opt/rocm/include", src]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-4000:]
