"""CPU: bench.py's multi-GPU launch contract — `--gpus N` outside a launcher re-runs the script
under torch.distributed.run with N ranks (127.0.0.1 rendezvous) as a child process, before any
GPU call; under a launcher it does not spawn again."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_gpus_n_spawns_ranks(monkeypatch):
    import bench
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 0

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    for k in ("LOCAL_RANK", "MASTER_ADDR"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


def test_launched_rank_does_not_respawn(monkeypatch):
    import bench
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    assert bench.launched_distributed()
