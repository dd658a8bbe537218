"""The BASELINE.json configurations at their full sizes (C1-C5).

fp32 frames are compared with the C oracle bit for bit where the oracle finishes in
seconds (C1, C2, and C3's geometry/size/steps in fp32); at the reduced-precision
configs the checks are size-independent properties: shards of a frame re-assemble to
the full-frame render exactly, renders are deterministic, and the bf16/fp16 frame
covers the fp32 frame's silhouette (IoU > 0.97) with ray-step counts within 10%."""
import os

import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)
NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def setup(rend, nets, geom, prec, matcap, cam=(0.0, 0.0, 2.0)):
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision(prec)
    iv, nm = nr.camera(*cam)
    rend.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(matcap)
    return K, B, iv, nm


def iou(a, b):
    fa, fb = a != 0, b != 0
    return (fa & fb).sum() / max((fa | fb).sum(), 1)


@pytest.mark.parametrize("W,steps", [(256, 64), (1024, 128)])
def test_c1_c2_fp32_bitexact(rend, nets, chrome, W, steps):
    """C1 (256^2, 64 steps) and C2 (the bench frame: 1024^2, 128 steps), plane_1, Chrome."""
    K, B, iv, nm = setup(rend, nets, "plane_1", "fp32", chrome)
    img, st = rend.render(W, W, steps)
    ref, rst = oracle.OracleNet(K, B).render(W, W, iv, nm, color_type=1, matcap=chrome, max_steps=steps,
                                             nthreads=NTHREADS)
    assert np.array_equal(img, ref), int((img != ref).sum())
    for k in ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations"):
        assert st[k] == rst[k], (k, st, rst)


def test_c3_car1_2048(rend, nets, chrome):
    """C3: car_1 2048^2, 256 steps.  fp32 is bit-exact against the oracle; bf16 covers
    the fp32 silhouette and is deterministic."""
    K, B, iv, nm = setup(rend, nets, "car_1", "fp32", chrome)
    f32, s32 = rend.render(2048, 2048, 256)
    ref, rst = oracle.OracleNet(K, B).render(2048, 2048, iv, nm, color_type=1, matcap=chrome, max_steps=256,
                                             nthreads=NTHREADS)
    assert np.array_equal(f32, ref), int((f32 != ref).sum())
    assert s32["ray_steps"] == rst["ray_steps"]
    rend.set_precision("bf16")
    try:
        b1, sb = rend.render(2048, 2048, 256)
        b2, _ = rend.render(2048, 2048, 256)
    finally:
        rend.set_precision("fp32")
    assert np.array_equal(b1, b2)
    assert iou(b1, f32) > 0.97
    # bf16 SDF error (~1e-2) moves where grazing rays converge: step counts within 10%
    assert abs(sb["ray_steps"] - s32["ray_steps"]) / s32["ray_steps"] < 0.10


@pytest.mark.parametrize("band", [1, 8])
def test_c4_plane2_4096_shards(rend, nets, chrome, band):
    """C4: plane_2 4096^2 bf16, rows dealt round-robin to 8 shards (one per GPU) in bands of
    1 row (bench.py's layout) or 8; the 8 shard renders -- single-frame and through
    nr_render_batch, bench.py's call -- re-assemble to the single-launch frame exactly."""
    setup(rend, nets, "plane_2", "bf16", chrome)
    try:
        full, st = rend.render(4096, 4096, 128)
        iv, nm = nr.camera(0.0, 0.0, 2.0)
        shards, bshards, steps, bsteps = [], [], 0, 0
        for s in range(8):
            img, sst = rend.render_shard(4096, 4096, band, 8, s, 128)
            shards.append(img)
            steps += sst["ray_steps"]
            imgs, bst = rend.render_batch(4096, 4096, [(iv, nm, 0)] * 2, 128, band=band, nshards=8, shard=s)
            assert np.array_equal(imgs[0], img) and np.array_equal(imgs[1], img)
            bsteps += bst["ray_steps"]
        assert np.array_equal(nr.assemble_shards(shards, 4096, 4096, band, 8), full)
        assert steps == st["ray_steps"] and bsteps == 2 * st["ray_steps"]
        rend.set_precision("fp32")
        f32, s32 = rend.render(4096, 4096, 128)
    finally:
        rend.set_precision("fp32")
    assert iou(full, f32) > 0.97
    assert abs(st["ray_steps"] - s32["ray_steps"]) / s32["ray_steps"] < 0.10


@pytest.mark.parametrize("geom", ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"])
def test_c5_geometries_fp16_2048(rend, nets, chrome, geom):
    """C5: one geometry per GPU at 2048^2 with fp16 weights (the bundled 5 geometries;
    the bench's 8 replicas cycle through them): fp16 covers the fp32 silhouette."""
    setup(rend, nets, geom, "fp16", chrome, cam=(-20.0, 35.0, 2.0))
    try:
        h, sh = rend.render(2048, 2048, 128)
        rend.set_precision("fp32")
        f, sf = rend.render(2048, 2048, 128)
    finally:
        rend.set_precision("fp32")
    assert iou(h, f) > 0.97
    assert abs(sh["ray_steps"] - sf["ray_steps"]) / max(sf["ray_steps"], 1) < 0.10


def test_large_frame_8192(rend, nets, chrome):
    """An 8192^2 frame (64 Mpixel, beyond the configs): the persistent and wavefront
    schedules agree pixel for pixel and in every count, and the 3 row-band shards of
    one rank layout re-assemble to it (size-independent properties; the oracle would
    need minutes)."""
    setup(rend, nets, "plane_1", "fp32", chrome, cam=(-10.0, 25.0, 2.0))
    N = 8192
    a, sa = rend.set_schedule("persistent").render(N, N, 12)
    b, sb = rend.set_schedule("wavefront").render(N, N, 12)
    rend.set_schedule("persistent")
    assert sa["rays_hit"] > N * N // 4
    for k in ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations"):
        assert sa[k] == sb[k], (k, sa, sb)
    assert np.array_equal(a, b)
    shards = [rend.render_shard(N, N, 1, 3, s, 12)[0] for s in range(3)]
    assert np.array_equal(nr.assemble_shards(shards, N, N, 1, 3), a)
