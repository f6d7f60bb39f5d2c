"""bench.py's driver contract on the CPU: argument plumbing and the N-GPU launcher
(the parent starts torch.distributed.run as a child — never an exec, never a GPU call —
and exits with its status)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_defaults():
    a = bench.parse([])
    assert (a.gpus, a.steps, a.warmup, a.k) == (1, 5, 1, 500)


def test_launch_command_shape():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3", "--warmup", "1"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]


@pytest.mark.parametrize("rc", [0, 3])
def test_parent_launches_ranks_as_child(monkeypatch, rc):
    """--gpus N without WORLD_SIZE: bench.main() runs the launcher via subprocess.call
    and exits with the child's status before importing torch.cuda / touching a GPU."""
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and rc)
    monkeypatch.setattr(bench.os, "execv", lambda *a: pytest.fail("exec"), raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == rc
    assert "--nproc-per-node=2" in seen["cmd"]
    assert seen["cmd"][-4:] == ["--gpus", "2", "--steps", "1"]


def test_rank_does_not_relaunch(monkeypatch):
    """Inside torch.distributed.run (WORLD_SIZE set) the launcher branch is skipped."""
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: pytest.fail("relaunched"))
    # stop right after the launcher decision: the first thing a rank does is the gloo group
    import torch.distributed as tdist
    monkeypatch.setattr(tdist, "init_process_group", lambda *a, **k: (_ for _ in ()).throw(
        RuntimeError("rank path reached")))
    with pytest.raises(RuntimeError, match="rank path reached"):
        bench.main()


def test_host_info():
    h = bench.host_info()
    assert h["nproc"] >= 1 and h["allowed_cpus"] >= 1
