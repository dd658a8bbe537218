"""bench.py's host logic on CPU: the --gpus N self-launch (no launcher in the environment)
and the pose list.  No GPU is touched: the launcher is stubbed."""
import os
import shutil
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


def _fake_rocprof(monkeypatch, values, rc=0):
    """Stub of the two rocprofv3 --pmc child runs: each writes a counter_collection.csv holding
    `values[counter]` per k_trace dispatch (plus a dispatch of another kernel) under its -d directory."""
    calls = []

    def fake_run(cmd, cwd=None, env=None, stdout=None, stderr=None, timeout=None):
        calls.append(cmd)
        counter = cmd[cmd.index("--pmc") + 1]
        out = os.path.join(cmd[cmd.index("-d") + 1], "host", "1")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "run_counter_collection.csv"), "w") as f:
            f.write("Kernel_Name,Counter_Name,Counter_Value\n")
            for v in values.get(counter, []):
                f.write(f"\"void nr::k_trace<0, false, false, true, false, false>(RenderArgs, MlpArgs, TraceArgs)\",{counter},{v}\n")
            f.write(f"k_assemble,{counter},999999\n")
        return subprocess.CompletedProcess(cmd, rc)

    monkeypatch.setattr(shutil, "which", lambda name: "/opt/rocm/bin/rocprofv3")
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.delenv("ROCPROF_OUTPUT_PATH", raising=False)
    return calls


def test_live_traffic_applies_gfx950_corrections(monkeypatch):
    """roofline.traffic measured in the run: FETCH_SIZE (KiB, wide reads under-counted 2x) and
    WRITE_SIZE (KiB) from two separate --pmc passes, averaged over the k_trace dispatches only."""
    calls = _fake_rocprof(monkeypatch, {"FETCH_SIZE": [5000, 5100, 5200], "WRITE_SIZE": [230000, 231000, 232000]})
    got = bench.live_traffic(32, "fp32", 1024, 128)
    assert got is not None
    hbm, detail = got
    assert hbm == int(5100 * 1024 * 2 + 231000 * 1024)
    assert detail["dispatches"] == [3, 3] and detail["frames_per_launch"] == 32
    assert detail["algorithmic_bytes_per_launch"] == 1024 * 1024 * 4 * 32 + 30 * 1024 + 1024 * 1024
    # two passes, one counter each, the program itself after "--" (no shell or env hop under the profiler)
    assert [c[c.index("--pmc") + 1] for c in calls] == ["FETCH_SIZE", "WRITE_SIZE"]
    for c in calls:
        assert c[c.index("--") + 1] == sys.executable
        assert sum(x.startswith("-") and "trace" in x for x in c) == 0   # counters only, no trace domain
        assert c[:2] == ["timeout", "-k"]


def test_live_traffic_falls_back(monkeypatch):
    """A failed pass, a pass with no k_trace dispatch, a profiled parent or no rocprofv3: None (the
    caller then reports the committed figure)."""
    _fake_rocprof(monkeypatch, {"FETCH_SIZE": [5000], "WRITE_SIZE": [230000]}, rc=124)
    assert bench.live_traffic(32, "fp32", 1024, 128) is None
    _fake_rocprof(monkeypatch, {"FETCH_SIZE": [5000]})
    assert bench.live_traffic(32, "fp32", 1024, 128) is None
    _fake_rocprof(monkeypatch, {"FETCH_SIZE": [5000], "WRITE_SIZE": [230000]})
    monkeypatch.setenv("ROCPROF_OUTPUT_PATH", "/tmp/x")
    assert bench.live_traffic(32, "fp32", 1024, 128) is None
    monkeypatch.delenv("ROCPROF_OUTPUT_PATH")
    monkeypatch.setattr(shutil, "which", lambda name: None)
    assert bench.live_traffic(32, "fp32", 1024, 128) is None
