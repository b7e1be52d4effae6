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


def test_sbedecoder_address_sanitizer(tmp_path):
    """The mirror library and the same test built with AddressSanitizer + UBSan (host code only;
    no device call is made): no invalid access or undefined behaviour on the random and mutated
    records."""
    root = os.path.dirname(HERE)
    pkg = os.path.join(root, "aeron-cluster-client-cpp_amd")
    san = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(root, "include"),
           "-I", os.path.join(pkg, "host"), "-I", "/opt/rocm/include"]
    lib = str(tmp_path / "libaeron_cluster_amd.so")
    subprocess.check_call(["g++", *san, "-fPIC", "-shared", "-o", lib, os.path.join(pkg, "host", "aeron_cluster_amd.cpp"),
                           "-L", pkg, "-lsbecodec", "-L/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{pkg}", "-Wl,-rpath,/opt/rocm/lib"])
    exe = str(tmp_path / "test_sbedecoder_asan")
    subprocess.check_call(["g++", *san, "-o", exe, os.path.join(HERE, "cpp", "test_sbedecoder.cpp"),
                           "-L", str(tmp_path), "-laeron_cluster_amd", "-L", pkg, "-lsbecodec",
                           "-L", os.path.join(root, "oracle"), "-loracle", "-L/opt/rocm/lib", "-lamdhip64",
                           f"-Wl,-rpath,{tmp_path}", f"-Wl,-rpath,{pkg}", f"-Wl,-rpath,{os.path.join(root, 'oracle')}",
                           "-Wl,-rpath,/opt/rocm/lib"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "sbedecoder test: ok" in r.stdout and "runtime error" not in r.stderr
