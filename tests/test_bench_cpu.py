"""bench.py's host logic on CPU: the --gpus N self-launch (no launcher in the environment)
and the pose list.  No GPU is touched: the launcher is stubbed."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_self_launch_starts_torchrun_child(monkeypatch):
    seen = {}

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 7)

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "8", "--warmup", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7                      # the child's status
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index(os.path.abspath(bench.__file__)) + 1:] == ["--gpus", "4", "--steps", "8", "--warmup", "2"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # the parent never initialised a GPU runtime (torch may not even be imported by it)
    assert "torch.cuda" not in sys.modules or not __import__("torch").cuda.is_initialized()


def test_under_a_launcher_no_child(monkeypatch):
    """With WORLD_SIZE set (driver's torch.distributed.run) bench.py runs the rank itself."""
    called = []
    monkeypatch.setattr(bench.subprocess, "run", lambda *a, **k: called.append(a))
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as e:       # WORLD_SIZE != --gpus is refused before any GPU work
        bench.main()
    assert "WORLD_SIZE" in str(e.value.code) and not called


def test_random_poses():
    p = bench.random_poses()
    assert len(p) == 8 and p == bench.random_poses()
    assert all(-30 <= rx <= 30 and 0 <= ry < 360 for rx, ry in p)


def test_config_presets(monkeypatch):
    """--config picks a BASELINE config; explicit flags override it; c5 is replicas."""
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.config, a.geometry, a.size, a.precision, a.max_steps, a.replicas) == ("c2", "plane_1", 1024, "fp32", 128, False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "c3", "--size", "512"])
    a = bench.parse()
    assert (a.geometry, a.size, a.precision, a.max_steps) == ("car_1", 512, "bf16", 256)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "c5", "--gpus", "8"])
    a = bench.parse()
    assert a.replicas and a.geometry is None and (a.size, a.precision) == (2048, "fp16")


def test_c5_rank_geometries():
    """c5: rank r renders bundled geometry r % 5 (BASELINE configs[4], one geometry per GPU)."""
    g = [bench.GEOMS[r % len(bench.GEOMS)] for r in range(8)]
    assert g[:5] == bench.GEOMS and g[5:] == bench.GEOMS[:3]
    assert all(os.path.exists(os.path.join(REPO, "data", "neuralGeometries", x + ".h5")) for x in bench.GEOMS)
