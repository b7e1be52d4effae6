"""CPU: the host mirror's worker pool (aeron-cluster-client-cpp_amd/host/workers.hpp) under stress:
tests/cpp/test_workers.cpp built with g++ and run (every task once, bounded helpers, exceptions,
concurrent callers, sleeping and spinning workers)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_worker_pool(tmp_path):
    exe = str(tmp_path / "test_workers")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-pthread",
                           "-I", os.path.join(ROOT, "aeron-cluster-client-cpp_amd", "host"),
                           os.path.join(HERE, "cpp", "test_workers.cpp"), "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "worker pool test: ok" in r.stdout


def test_worker_pool_thread_sanitizer(tmp_path):
    """The same stress test built with ThreadSanitizer (host code only): no data race reported."""
    exe = str(tmp_path / "test_workers_tsan")
    subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=thread",
                           "-I", os.path.join(ROOT, "aeron-cluster-client-cpp_amd", "host"),
                           os.path.join(HERE, "cpp", "test_workers.cpp"), "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "worker pool test: ok" in r.stdout and "ThreadSanitizer" not in r.stderr
