"""NR_PRECISION_FP32X3: fp32-class MLP on the fp16 matrix core (three-term split, nr_mlp16.h
mlp32_x3_nt; pack nr_pack.cpp pack_x3_32), checked against the fp32 oracle and an exact (fp64)
evaluation of the same network.

Why the contract is a band and not bit-parity.  The reference's dense layer is a CUTLASS SIMT
GEMM (denseLayer.cu:126-176) whose summation order is unpinned; any fp32-class evaluation order
moves some march steps by an ulp, and one moved step re-rolls the rounding of that ray's four
normal samples (surfaceNormal, volumeRender_kernel.cu:361-377), i.e. its texel.  How far that
goes is measured by the oracle marching with the EXACT network (oracle precision 3: fp64
products and sums, fp32 normals): on C2 it agrees with the fp32 oracle on 99.3 % of the pixels,
on the C3 crop on only 88.6 %.  fp32x3 (~2-3x the fp32 chain's error against fp64) must land in
that band:
  * MLP: max |y - fp64| <= 1e-5 on the KAT points of every geometry, mean <= 5x the fp32
    chain's mean error;
  * frames (C2 full, the C3 / C4 / C5 crops of test_gpu_lowp_contract): identical pixels within
    6 points of the exact-MLP frame's agreement with the fp32 oracle, coverage IoU within 0.006
    of it, mean |delta| at most 2x its + 0.1; C2 itself >= 98.5 % identical and IoU >= 0.9995;
    ray-steps within 0.1 %;
  * the fallback (a wave with an input beyond the pack's bounds, or nr_set_debug bit 9, runs
    the fp32 MLP) is bit-exact with the fp32 oracle.
Since round 4 every frame and MLP value is also BIT-EXACT with the oracle's restatement of the
fp32x3 arithmetic (oracle precision 4: nr_oracle.c mlp_point_gpu_x3 over the library's pack,
each MFMA summed as gfx950's matrix core sums -- mfma_sum_e, profiles/r4_mfma_model.txt); the band
above is what fp32x3 costs against the fp32 contract.
Measured (round 3, gpurun_out/x3_contract.json -> profiles/r3_x3_contract.json): C2 99.1 %
identical vs the exact MLP's 99.3 %, the crops 1-4 points below the exact MLP's agreement."""
import json
import os

import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
from conftest import GEOMS, REPO, compare_frames

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


@pytest.fixture(scope="module")
def record():
    out = []
    yield out
    d = os.path.join(REPO, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "x3_contract.json"), "w") as f:
        json.dump(out, f, indent=1)


@pytest.mark.parametrize("geom", GEOMS)
def test_x3_mlp_matches_oracle_emulation(golden, nets, geom, record):
    """The oracle's fp32x3 restatement (nr_oracle.c mlp_point_gpu_x3, from the library's own pack,
    each MFMA summed as the matrix core sums: mfma_sum_e) against the GPU's fp32x3 MLP on the KAT
    points and a uniform cloud -- bit-exact.  It also pins the bf16/fp16 tracers' normals."""
    dims, K, B = nets[geom]
    rng = np.random.default_rng(11)
    X = np.concatenate([golden["kat"]["X"], rng.uniform(-1.2, 1.2, size=(8192, 3)).astype(np.float32)])
    with nr.Renderer(0) as r:
        y = r.load_h5(nr.geometry_path(geom)).set_precision("fp32x3").mlp_forward(X)[:, 0]
    pack = nr.pack_x3(dims, K, B)
    assert pack[2]
    e = oracle.OracleNet(K, B, x3_pack=pack[:2]).forward(X, precision=4)[:, 0]
    d = np.abs(y.astype(np.float64) - e)
    same = float((y == e).mean())
    record.append({"test": "x3_emulation", "geometry": geom, "identical": same, "max_abs": float(d.max())})
    assert np.array_equal(y, e), (same, d.max())


@pytest.mark.parametrize("geom", GEOMS)
def test_x3_mlp_kat(golden, nets, geom):
    dims, K, B = nets[geom]
    X = golden["kat"]["X"]
    ref = golden["kat"][geom]
    with nr.Renderer(0) as r:
        y = r.load_h5(nr.geometry_path(geom)).set_precision("fp32x3").mlp_forward(X)[:, 0]
    y32 = oracle.OracleNet(K, B).forward(X)[:, 0]
    e, e32 = np.abs(y.astype(np.float64) - ref), np.abs(y32.astype(np.float64) - ref)
    assert e.max() <= 1e-5, (e.max(), e32.max())
    assert e.mean() <= 5 * e32.mean(), (e.mean(), e32.mean())
    # and it is not the fp32 path in disguise
    assert not np.array_equal(y, y32)


def test_x3_mlp_out_of_bound_points_fall_back_bitexact(nets):
    """A point with an input beyond X3_INPUT_BOUND (4) runs the fp32 MLP: bit-exact with the
    oracle.  Every other point stays on the split -- its chunk-mates included, whose values equal
    those of the same points evaluated with no outlier anywhere (the fallback used to
    take the whole 64-point wave, so a point's value depended on its chunk)."""
    dims, K, B = nets["plane_1"]
    rng = np.random.default_rng(5)
    X = rng.uniform(-1.2, 1.2, size=(64 * 64, 3)).astype(np.float32)
    clean = X.copy()
    far = [64 * c + 11 for c in (3, 17, 40, 63)] + [64 * 20 + k for k in range(64)]  # + one whole chunk
    for i in far:
        X[i, 1] = 5.0 if i % 2 else -7.5
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision("fp32x3")
        y = r.mlp_forward(X)[:, 0]
        yc = r.mlp_forward(clean)[:, 0]
        # and the same points shifted by 32: other chunks, other lane halves, same values
        ys = r.mlp_forward(np.concatenate([clean[:32], X]))[32:, 0]
    y32 = oracle.OracleNet(K, B).forward(X)[:, 0]
    mask = np.zeros(len(X), bool)
    mask[far] = True
    assert np.array_equal(y[mask], y32[mask])
    assert np.array_equal(y[~mask], yc[~mask])
    assert np.array_equal(ys, y)
    assert not np.array_equal(y[~mask], y32[~mask])
    assert np.abs(y[~mask] - y32[~mask]).max() <= 1e-5


def test_x3_debug_fallback_renders_fp32_bitexact(nets, chrome):
    """nr_set_debug bit 9 sends every fp32x3 wave to the fp32 MLP: the frame is the fp32 oracle's."""
    dims, K, B = nets["plane_1"]
    iv, nm = nr.camera(-10.0, 30.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision("fp32x3").set_debug(512)
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(160, 120, 128)
    ref, rst = oracle.OracleNet(K, B).render(160, 120, iv, nm, color_type=1, matcap=chrome, max_steps=128)
    assert np.array_equal(img, ref)
    assert st["ray_steps"] == rst["ray_steps"]


def test_x3_unscalable_network_falls_back_bitexact():
    """A network whose activation bound leaves the pack's scale range (a bias of 1e35: scale
    2^-106) has no fp32x3 pack: every wave runs the fp32 MLP, bit-exact with the oracle.  (A
    merely large weight, e.g. 1e30, is scaled like any other: the layer's scale follows it.)"""
    rng = np.random.default_rng(9)
    dims = [3] + [32] * 8 + [1]
    K = [rng.uniform(-0.5, 0.5, size=(dims[i], dims[i + 1])).astype(np.float32) for i in range(len(dims) - 1)]
    B = [rng.uniform(-0.05, 0.05, size=dims[i + 1]).astype(np.float32) for i in range(len(dims) - 1)]
    B[2][0] = 1e35
    X = rng.uniform(-1, 1, size=(1000, 3)).astype(np.float32)
    with nr.Renderer(0) as r:
        r.load_mlp(dims, K, B).set_precision("fp32x3")
        y = r.mlp_forward(X)
    assert np.array_equal(y, oracle.OracleNet(K, B).forward(X))


def test_x3_four_input_network(nets):
    """Animation networks (numInputs 4, the frame as 4th input, volumeRender_kernel.cu:524-545):
    the frame enters layer 0 unscaled; MLP within fp32-class error of the exact evaluation."""
    rng = np.random.default_rng(3)
    dims = [4] + [32] * 8 + [1]
    K = [rng.normal(0, 0.3, size=(dims[i], dims[i + 1])).astype(np.float32) for i in range(len(dims) - 1)]
    K[0][3] *= 0.01
    B = [rng.normal(0, 0.05, size=dims[i + 1]).astype(np.float32) for i in range(len(dims) - 1)]
    X = np.concatenate([rng.uniform(-1.2, 1.2, size=(4096, 3)), rng.integers(0, 360, size=(4096, 1))], 1).astype(np.float32)
    with nr.Renderer(0) as r:
        y = r.load_mlp(dims, K, B).set_precision("fp32x3").mlp_forward(X)[:, 0]
    net = oracle.OracleNet(K, B)
    y64 = net.forward(X, precision=3)[:, 0].astype(np.float64)
    y32 = net.forward(X)[:, 0].astype(np.float64)
    scale = np.abs(y64).max()
    assert np.abs(y - y64).max() <= 1e-5 * max(scale, 1.0), (np.abs(y - y64).max(), np.abs(y32 - y64).max())
    assert np.abs(y - y64).mean() <= 5 * np.abs(y32 - y64).mean() + 1e-9


def test_x3_schedules_agree(chrome):
    """The split's result for a point does not depend on its tile or wave (no input beyond the
    bounds at this camera): persistent, batched and wavefront schedules give the same pixels."""
    iv, nm = nr.camera(0.0, 0.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("car_1")).set_precision("fp32x3")
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        a, sa = r.render(256, 256, 128)
        imgs, sb = r.render_batch(256, 256, [(iv, nm, 0)] * 3, 128)
        r.set_schedule("wavefront")
        c, sc = r.render(256, 256, 128)
    assert all(np.array_equal(a, b) for b in imgs)
    assert np.array_equal(a, c)
    assert sb["ray_steps"] == 3 * sa["ray_steps"] and sc["ray_steps"] == sa["ray_steps"]


CASES = [("C2", "plane_1", 1024, 128, None)]
CASES += [("C3", "car_1", 2048, 256, (896, 1152)), ("C4", "plane_2", 4096, 128, (1984, 2112))]
CASES += [("C5", g, 2048, 128, (960, 1088)) for g in GEOMS]


@pytest.mark.parametrize("name,geom,size,steps,rows", CASES, ids=[f"{c[0]}-{c[1][:8]}" for c in CASES])
def test_x3_pixel_contract(chrome, record, name, geom, size, steps, rows):
    dims, K, B = nr.read_keras_h5(nr.geometry_path(geom))
    iv, nm = nr.camera(0.0, 0.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path(geom)).set_precision("fp32x3")
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(size, size, steps)
    y0, y1 = rows if rows else (0, size)
    pack = nr.pack_x3(dims, K, B)
    net = oracle.OracleNet(K, B, x3_pack=pack[:2])
    kw = dict(color_type=1, matcap=chrome, max_steps=steps, nthreads=16, rows=(y0, y1))
    f32, s32 = net.render(size, size, iv, nm, precision=0, **kw)
    f64, _ = net.render(size, size, iv, nm, precision=3, **kw)
    # the restatement (~15x the fp32 oracle's cost per evaluation) on 16 rows through the centre
    xr = ((y0 + y1) // 2 - 8, (y0 + y1) // 2 + 8)
    fx3, _ = net.render(size, size, iv, nm, precision=4, **dict(kw, rows=xr))
    gpu = img[y0:y1]
    res = {"config": name, "geometry": geom, "size": size, "steps": steps, "rows": [y0, y1],
           "x3_vs_fp32_oracle": compare_frames(gpu, f32), "exact_mlp_vs_fp32_oracle": compare_frames(f64, f32),
           "x3_vs_exact_mlp": compare_frames(gpu, f64), "x3_vs_oracle_x3_rows": compare_frames(img[xr[0]:xr[1]], fx3)}
    record.append(res)
    # bit-exact with the oracle's restatement of the fp32x3 arithmetic (nr_oracle.c
    # mlp_point_gpu_x3 over the matrix core's summation, mfma_sum_e; round 4)
    assert pack[2] and np.array_equal(img[xr[0]:xr[1]], fx3), res
    assert (fx3 != 0).any()
    x, band = res["x3_vs_fp32_oracle"], res["exact_mlp_vs_fp32_oracle"]
    assert x["identical"] >= band["identical"] - 0.06, res
    assert x["iou"] >= band["iou"] - 0.006, res
    assert max(x["mean_abs"][:3]) <= 2 * max(band["mean_abs"][:3]) + 0.1, res
    if name == "C2":
        assert x["identical"] >= 0.985 and x["iou"] >= 0.9995, res
        assert abs(st["ray_steps"] - s32["ray_steps"]) <= 1e-3 * s32["ray_steps"], (st, s32)


def test_x3_batch_frames_straddling_bound():
    """A 4-input network (the frame as 4th input): frames beyond X3_FRAME_BOUND (1024) take the
    fp32 MLP, the others the split -- per point, so a batch holding frames on both sides of the
    bound gives every frame the pixels of its own single-frame render."""
    rng = np.random.default_rng(12)
    dims = [4] + [32] * 8 + [1]
    K = [rng.normal(0, 0.3, size=(dims[i], dims[i + 1])).astype(np.float32) for i in range(len(dims) - 1)]
    K[0][3] *= 0.0005
    B = [rng.normal(0, 0.05, size=dims[i + 1]).astype(np.float32) for i in range(len(dims) - 1)]
    B[-1][0] = 0.2
    iv, nm = nr.camera(0, 0, 2)
    frames = [3, 1500, 1024, 1025, 7]
    with nr.Renderer(0) as r:
        r.load_mlp(dims, K, B).set_precision("fp32x3").set_static(nr.NR_COLOR_FACING, 4).set_scene("v1")
        singles = []
        for f in frames:
            r.set_view(iv, nm, f)
            singles.append(r.render(80, 64, 64)[0])
        imgs, _ = r.render_batch(80, 64, [(iv, nm, f) for f in frames], 64)
    assert all(np.array_equal(a, b) for a, b in zip(imgs, singles))
    assert any((s != 0).any() for s in singles)


def test_x3_three_input_net_past_frame_bound(chrome):
    """A 3-input network at frame 2000 (> X3_FRAME_BOUND): the frame is not an input of the
    network, so every point stays on the split -- the single-frame render (whose tracer passes the
    frame number to the MLP), the batched render and the oracle's restatement agree."""
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    iv, nm = nr.camera(20.0, 30.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision("fp32x3")
        r.set_view(iv, nm, 2000).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(96, 96, 64)
        imgs, _ = r.render_batch(96, 96, [(iv, nm, 2000), (iv, nm, 2000)], 64)
    pack = nr.pack_x3(dims, K, B)
    net = oracle.OracleNet(K, B, x3_pack=pack[:2])
    ref, rst = net.render(96, 96, iv, nm, frame=2000, color_type=1, matcap=chrome, max_steps=64, precision=4)
    assert (ref != 0).any()
    assert np.array_equal(img, ref) and st["ray_steps"] == rst["ray_steps"], (img != ref).sum()
    assert all(np.array_equal(b, ref) for b in imgs)
