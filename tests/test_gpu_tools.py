"""The headless drivers (tools/: the reference's main.cpp and simpleInfer.cpp restated
over the C++ API of include/nr/*.hh) on the GPU, against the oracle."""
import os
import subprocess

import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tools", "bin")


def run(args, **kw):
    return subprocess.run(args, capture_output=True, text=True, timeout=120, **kw)


def test_simple_infer_batch():
    p = run([os.path.join(BIN, "simpleInfer"), nr.geometry_path("plane_1"), "1000000"])
    assert p.returncode == 0, p.stdout + p.stderr
    assert "Woah there aren't any!!" in p.stdout
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    y0 = oracle.OracleNet(K, B).forward(np.zeros((1, 3), np.float32))[0, 0]
    assert f"(0.000000,0.000000,0.000000):{y0:f}" in p.stdout


@pytest.mark.parametrize("matcap,scene", [("Chrome", "v1"), (None, "tanh")])
def test_renderer_single_png(tmp_path, matcap, scene):
    args = [os.path.join(BIN, "neuralSDFRenderer"), "-i", nr.geometry_path("plane_1"), "-o", str(tmp_path) + "/",
            "-W", "96", "-H", "80", "-rx", "-20", "-ry", "30", "--single", "--max-steps", "128", "--scene", scene,
            "--ppm"]
    if matcap:
        args += ["-M", nr.matcap_path(matcap)]
    p = run(args)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "volumeRender, Throughput =" in p.stdout
    png = nr.load_png(str(tmp_path / "plane_1.h5.png"))
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    iv, nm = nr.camera(-20, 30, 2.0)  # the CLI's default camera arithmetic (f64, rounded once)
    mc = nr.load_png(nr.matcap_path(matcap)) if matcap else None
    ref, _ = oracle.OracleNet(K, B).render(96, 80, iv, nm, color_type=1 if matcap else 0,
                                           scene=0 if scene == "v1" else 1, matcap=mc, max_steps=128)
    # savePNG reverses the byte stream: the saved image is the frame rotated 180 degrees
    assert np.array_equal(png, ref[::-1, ::-1])
    ppm = open(str(tmp_path / "plane_1.h5.png.ppm"), "rb").read()
    assert ppm.startswith(b"P6\n96\n80\n255\n")


def test_renderer_spin(tmp_path):
    """--spin (doABarrelRoll, main.cpp:470-478): 360 frames, rotY = frame number = i,
    saved as 000.png ... 359.png (main.cpp:445-458 naming)."""
    args = [os.path.join(BIN, "neuralSDFRenderer"), "-i", nr.geometry_path("car_1"), "-o", str(tmp_path) + "/",
            "-W", "24", "-H", "20", "-rx", "-15", "--spin", "--max-steps", "96", "-M", nr.matcap_path("Chrome")]
    p = run(args)
    assert p.returncode == 0, p.stdout + p.stderr
    names = sorted(os.listdir(tmp_path))
    assert len(names) == 360 and names[0] == "000.png" and names[-1] == "359.png"
    dims, K, B = nr.read_keras_h5(nr.geometry_path("car_1"))
    mc = nr.load_png(nr.matcap_path("Chrome"))
    net = oracle.OracleNet(K, B)
    for i in (0, 45, 200, 359):
        iv, nm = nr.camera(-15, float(i), 2.0)
        ref, _ = net.render(24, 20, iv, nm, frame=i, color_type=1, matcap=mc, max_steps=96)
        png = nr.load_png(str(tmp_path / f"{i:03d}.png"))
        assert np.array_equal(png, ref[::-1, ::-1]), i


def test_renderer_camera_eigen(tmp_path):
    """--camera eigen: the frame of nr_camera_ex's restatement of Eigen's scalar float path
    (unpinned against the reference's SSE build; the CLI default is f64)."""
    args = [os.path.join(BIN, "neuralSDFRenderer"), "-i", nr.geometry_path("plane_1"), "-o", str(tmp_path) + "/",
            "-W", "64", "-H", "48", "-rx", "-33.3", "-ry", "71.7", "--single", "--max-steps", "128",
            "-M", nr.matcap_path("Chrome"), "--camera", "eigen"]
    p = run(args)
    assert p.returncode == 0, p.stdout + p.stderr
    png = nr.load_png(str(tmp_path / "plane_1.h5.png"))
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    iv, nm = nr.camera(-33.3, 71.7, 2.0, mode="eigen")
    ref, _ = oracle.OracleNet(K, B).render(64, 48, iv, nm, color_type=1, matcap=nr.load_png(nr.matcap_path("Chrome")),
                                           max_steps=128)
    assert np.array_equal(png, ref[::-1, ::-1])


def test_renderer_gpus_group(tmp_path):
    """--gpus N (nr_group_render_batch: row-band shards on N GPUs, one RCCL gather): on the
    one-GPU box N = 1, whose frame (through the RCCL send/recv and the re-interleave) equals the
    single-GPU render_kernel path's."""
    base = [os.path.join(BIN, "neuralSDFRenderer"), "-i", nr.geometry_path("car_1"), "-W", "72", "-H", "56",
            "-rx", "-12", "-ry", "40", "--single", "--max-steps", "128", "-M", nr.matcap_path("Chrome")]
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    p = run(base + ["-o", str(a) + "/"])
    assert p.returncode == 0, p.stdout + p.stderr
    p = run(base + ["-o", str(b) + "/", "--gpus", "1"])
    assert p.returncode == 0, p.stdout + p.stderr
    assert "NumDevsUsed = 1" in p.stdout
    ia, ib = nr.load_png(str(a / "car_1.h5.png")), nr.load_png(str(b / "car_1.h5.png"))
    assert np.array_equal(ia, ib) and (ia != 0).any()
