"""bench.py's multi-GPU launch contract on the CPU (no GPU call): ``--gpus N`` without a
launcher starts N ranks through torch.distributed.run as a child process; under a
launcher ``--gpus`` must equal WORLD_SIZE."""
import os
import subprocess
import sys

import pytest

from conftest import REPO


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gpus_spawns_ranks(monkeypatch):
    bench = _bench()
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.setattr(subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    args = bench.parse()
    assert bench.launch_ranks(args) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_gpus_one_and_launcher_consistency(monkeypatch):
    bench = _bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.launch_ranks(bench.parse()) is None           # N = 1: run in this process
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.launch_ranks(bench.parse()) is None           # launched rank: run
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.launch_ranks(bench.parse())
