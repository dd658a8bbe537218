"""GPU parity: libnr.so (HIP, gfx950) against the CPU oracle, through the C ABI.

FP32 is bit-exact by contract (DESIGN.md "numerics"); bf16/fp16 are tolerance
tests.  Pixel (W-1, H-1) needs no exclusion here: both sides fix quirk Q1.
"""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
from conftest import GEOMS

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def pts(n, seed=0, lo=-1.2, hi=1.2):
    return np.random.default_rng(seed).uniform(lo, hi, size=(n, 3)).astype(np.float32)


@pytest.mark.parametrize("geom", GEOMS)
def test_mlp_forward_bitexact(rend, nets, golden, geom):
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    X = golden["kat"]["X"]
    y_gpu = rend.mlp_forward(X)
    y_cpu = oracle.OracleNet(K, B).forward(X)
    assert np.array_equal(y_gpu.view(np.uint32), y_cpu.view(np.uint32)), \
        f"{(y_gpu != y_cpu).sum()} of {len(X)} differ, max {np.abs(y_gpu - y_cpu).max()}"


@pytest.mark.parametrize("n", [1, 31, 64, 65, 1000, 100003])
def test_mlp_forward_ragged(rend, nets, n):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    X = pts(n, seed=n)
    assert np.array_equal(rend.mlp_forward(X), oracle.OracleNet(K, B).forward(X))


def test_simpleinfer_batch_consistency(rend, nets):
    # simpleInfer.cpp:112-147: 1e6 identical zero inputs -> all outputs equal
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    Y = rend.mlp_forward(np.zeros((1000000, 3), np.float32))
    assert (Y == Y[0]).all()
    assert Y[0, 0] == oracle.OracleNet(K, B).forward(np.zeros((1, 3), np.float32))[0, 0]


@pytest.mark.parametrize("layer", range(9))
def test_layer_forward_bitexact(rend, nets, layer):
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B)
    A = np.random.default_rng(layer).uniform(-1, 1, size=(777, dims[layer])).astype(np.float32)
    Z = rend.layer_forward(layer, A)
    net1 = oracle.OracleNet([K[layer]], [B[layer]])
    ref = net1.forward(A)
    if layer != 8:
        ref = np.maximum(ref, 0)  # single-layer oracle net treats its only layer as last (linear)
    assert np.array_equal(Z, ref)


RENDER_CASES = [
    # W, H, scene, color, rx, ry, zoom, steps
    (128, 128, "v1", "matcap", 0.0, 0.0, 2.0, 128),
    (128, 96, "tanh", "matcap", -18.3, 150.7, 2.25, 256),
    (97, 61, "v1", "facing", 25.0, 40.0, 2.0, 64),
    (64, 64, "v1", "facing", 10.0, 300.0, 3.0, 6000),
    (1, 1, "v1", "facing", 0.0, 0.0, 2.0, 100),
    # the scenes sceneSDF comments out (volumeRender_kernel.cu:217-229)
    (96, 80, "subtract", "matcap", -15.0, 40.0, 2.0, 128),
    (64, 64, "cylinders", "facing", 20.0, 30.0, 2.0, 128),
    (96, 72, "displace", "matcap", 10.0, 200.0, 2.0, 128),
    (96, 72, "round", "facing", -25.0, 100.0, 2.25, 128),
]


@pytest.mark.parametrize("schedule", ["persistent", "wavefront", "layered"])
@pytest.mark.parametrize("W,H,scene,color,rx,ry,zoom,steps", RENDER_CASES)
def test_render_bitexact(rend, nets, chrome, W, H, scene, color, rx, ry, zoom, steps, schedule):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32").set_schedule(schedule)
    iv, nm = nr.camera(rx, ry, zoom)
    ct = nr.NR_COLOR_MATCAP if color == "matcap" else nr.NR_COLOR_FACING
    rend.set_view(iv, nm, 0).set_static(ct, 3).set_scene(scene).set_matcap(chrome)
    img, st = rend.render(W, H, steps)
    ref, rst = oracle.OracleNet(K, B).render(W, H, iv, nm, color_type=ct, scene=nr.NR_SCENE[scene],
                                             matcap=chrome if ct else None, max_steps=steps)
    diff = img != ref
    assert not diff.any(), f"{diff.sum()} pixels differ; gpu stats {st} oracle {rst}"
    for k in ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations"):
        assert st[k] == rst[k], (k, st, rst)
    rend.set_schedule("persistent")


@pytest.mark.parametrize("geom", ["plane_2", "car_1", "plane_3", "3a3d4a90a2db90b4203936772104a82d.obj"])
def test_render_geometries(rend, nets, chrome, geom):
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(-20.0, 35.0, 2.0)
    rend.set_view(iv, nm, 7).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
    img, st = rend.render(80, 72, 128)
    ref, rst = oracle.OracleNet(K, B).render(80, 72, iv, nm, frame=7, color_type=1, matcap=chrome, max_steps=128)
    assert np.array_equal(img, ref)
    assert st["ray_steps"] == rst["ray_steps"]


def test_render_empty_scene(rend, nets):
    # eye at (0, 0, 5) looking along +z, away from the bounding sphere: every ray misses
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B)
    iv = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, -1, 5], np.float32)
    nm = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, -1, 5, 0, 0, 0, 1], np.float32)
    rend.set_view(iv, nm).set_static(0, 3).set_scene("v1")
    img, st = rend.render(64, 48, 100)
    ref, rst = oracle.OracleNet(K, B).render(64, 48, iv, nm, max_steps=100)
    assert (img == 0).all() and (ref == 0).all()
    # the line through the eye still crosses the sphere behind it: those rays "hit" with
    # tnear, tfar < 0 and die on their first step (tfar <= 0), exactly as in the reference
    for k in ("rays_hit", "ray_steps", "rays_shaded", "iterations"):
        assert st[k] == rst[k], (k, st, rst)
    assert st["rays_shaded"] == 0


def test_render_zero_steps(rend, nets):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B)
    iv, nm = nr.camera(0, 0, 2)
    rend.set_view(iv, nm).set_static(0, 3).set_scene("v1")
    img, st = rend.render(32, 32, 0)
    assert (img == 0).all() and st["ray_steps"] == 0 and st["rays_hit"] == 32 * 32


@pytest.mark.parametrize("nshards,band", [(2, 8), (3, 5), (8, 8), (4, 1)])
def test_shards_assemble_to_frame(rend, nets, chrome, nshards, band):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(-10.0, 20.0, 2.0)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    W, H = 70, 83
    full, _ = rend.render(W, H, 128)
    shards = [rend.render_shard(W, H, band, nshards, s, 128)[0] for s in range(nshards)]
    assert sum(s.shape[0] for s in shards) == H
    assert np.array_equal(nr.assemble_shards(shards, W, H, band, nshards), full)


@pytest.mark.parametrize("nshards,band", [(2, 1), (4, 1), (8, 1), (2, 4)])
def test_stacked_assembly_device(rend, nets, chrome, nshards, band):
    """bench.py's N-rank collection on one device: each shard's n frames rendered by one
    nr_render_batch into a rank-major buffer (the layout one RCCL gather leaves on rank 0),
    then ONE device nr_assemble_shards of the n frames stacked as an (n*H)-row image (valid
    when H is a multiple of band * nshards) -- equal to the single-GPU frames."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")  # libnr's HIP runtime (by soname): device buffers without torch
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32").set_static(1, 3).set_scene("v1").set_matcap(chrome)
    W, H, n = 96, 64, 5
    assert H % (band * nshards) == 0
    cams = [(*nr.camera(-10.0, 30.0 * i, 2.0), 0) for i in range(n)]
    rows = H // nshards
    gather, frames = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(gather), ctypes.c_size_t(nshards * n * rows * W * 4)) == 0
    assert hip.hipMalloc(ctypes.byref(frames), ctypes.c_size_t(n * H * W * 4)) == 0
    try:
        for s in range(nshards):
            assert nr.shard_rows(H, band, nshards, s) == rows
            base = gather.value + s * n * rows * W * 4
            rend.render_batch_device([base + i * rows * W * 4 for i in range(n)], W, H, cams, 128, band, nshards, s)
        rend.assemble_device(gather.value, n * rows * W, frames.value, W, n * H, band, nshards)
        rend.synchronize()
        got = np.zeros((n, H, W), np.uint32)
        assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), frames, ctypes.c_size_t(got.nbytes), 2) == 0  # D2H
    finally:
        hip.hipFree(gather)
        hip.hipFree(frames)
    for i, (iv, nm, f) in enumerate(cams):
        rend.set_view(iv, nm, f)
        ref, _ = rend.render(W, H, 128)
        assert np.array_equal(got[i], ref), i
    rend.set_view(*nr.camera(0, 0, 2), 0)


@pytest.mark.parametrize("prec,tol", [("bf16", 0.05), ("fp16", 0.01)])
def test_mlp_lowp_tolerance(rend, nets, golden, prec, tol):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision(prec)
    X = golden["kat"]["X"]
    y = rend.mlp_forward(X)[:, 0]
    y64 = golden["kat"]["plane_1"]
    # tolerance relative to the output scale (SDF range of the bundled nets ~[-0.3, 1])
    assert np.abs(y - y64).max() < tol, np.abs(y - y64).max()
    rend.set_precision("fp32")


@pytest.mark.parametrize("schedule", ["persistent", "wavefront"])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_render_lowp_close(rend, nets, chrome, prec, schedule):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision(prec).set_schedule(schedule)
    iv, nm = nr.camera(0, 0, 2)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    img, st = rend.render(128, 128, 128)
    ref, rst = oracle.OracleNet(K, B).render(128, 128, iv, nm, color_type=1, matcap=chrome, max_steps=128)
    fg, fg_ref = img != 0, ref != 0
    iou = (fg & fg_ref).sum() / max((fg | fg_ref).sum(), 1)
    assert iou > 0.97, iou
    assert abs(st["ray_steps"] - rst["ray_steps"]) / rst["ray_steps"] < 0.05
    rend.set_precision("fp32").set_schedule("persistent")


def test_schedules_agree_1024(rend, nets, chrome):
    # full benchmark frame: persistent, wavefront and layered schedules give identical
    # pixels/stats
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(0, 0, 2)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    a, sa = rend.set_schedule("persistent").render(1024, 1024, 128)
    b, sb = rend.set_schedule("wavefront").render(1024, 1024, 128)
    c, sc = rend.set_schedule("layered").render(1024, 1024, 128)
    rend.set_schedule("persistent")
    assert np.array_equal(a, b) and np.array_equal(a, c)
    for k in ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations"):
        assert sa[k] == sb[k] == sc[k], (k, sa, sb, sc)


@pytest.mark.parametrize("W,H", [(200, 131), (1024, 1024)])
def test_temporal_order_same_pixels(rend, nets, chrome, W, H):
    # temporal block ordering changes only the order work is handed out
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(-15, 30, 2)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    a, sa = rend.render(W, H, 128)
    rend.set_temporal_order(True)
    b, sb = rend.render(W, H, 128)   # records costs, raster order
    c, sc = rend.render(W, H, 128)   # longest-first order from the previous frame
    rend.set_temporal_order(False)
    assert np.array_equal(a, b) and np.array_equal(a, c)
    assert sa["ray_steps"] == sb["ray_steps"] == sc["ray_steps"]


@pytest.mark.parametrize("mode", [1, 2])
def test_temporal_order_spin_same_pixels(rend, nets, chrome, mode):
    """The reference's --spin sequence (frame i at ry = i deg, frameNumber i; main.cpp:470-477)
    with the previous frame's block order, plain (1) and dilated over 3x3 blocks (2): every frame
    equals its plain render."""
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    rend.set_static(1, 3).set_scene("v1").set_matcap(chrome)
    plain = []
    for i in range(3):
        iv, nm = nr.camera(0, float(i), 2)
        rend.set_view(iv, nm, i)
        plain.append(rend.render(256, 192, 128))
    try:
        rend.set_temporal_order(mode)
        for i in range(3):
            iv, nm = nr.camera(0, float(i), 2)
            rend.set_view(iv, nm, i)
            img, st = rend.render(256, 192, 128)
            assert np.array_equal(img, plain[i][0]) and st["ray_steps"] == plain[i][1]["ray_steps"], (mode, i)
    finally:
        rend.set_temporal_order(False)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_temporal_order_batch_same_pixels(rend, nets, chrome, prec):
    """nr_render_batch with the temporal order: the first batch records its block costs, the
    next (and a sharded one after it, whose shape invalidates the order) hand the blocks out
    longest-first; pixels and ray-steps equal the plain batch."""
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision(prec)
    rend.set_static(1, 3).set_scene("v1").set_matcap(chrome)
    cams = [(*nr.camera(-20.0 + 10 * i, 40.0 * i, 2.0), i) for i in range(5)]
    try:
        a, sa = rend.render_batch(160, 120, cams, 128)
        rend.set_temporal_order(True)
        b, sb = rend.render_batch(160, 120, cams, 128)
        c, sc = rend.render_batch(160, 120, cams, 128)
        d, sd = rend.render_batch(160, 120, cams, 128, band=1, nshards=3, shard=1)
        rend.set_temporal_order(False)
        e, se = rend.render_batch(160, 120, cams, 128, band=1, nshards=3, shard=1)
        assert all(np.array_equal(x, y) and np.array_equal(x, z) for x, y, z in zip(a, b, c))
        assert sa["ray_steps"] == sb["ray_steps"] == sc["ray_steps"]
        assert all(np.array_equal(x, y) for x, y in zip(d, e)) and sd["ray_steps"] == se["ray_steps"]
    finally:
        rend.set_temporal_order(False).set_precision("fp32")


def test_render_deterministic(rend, nets, chrome):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(0, 0, 2)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    a, sa = rend.render(1024, 1024, 128)
    b, sb = rend.render(1024, 1024, 128)
    assert np.array_equal(a, b) and sa["ray_steps"] == sb["ray_steps"]


@pytest.mark.parametrize("W,H", [(200, 131), (1024, 1024)])
def test_schedule_knobs_same_pixels(rend, nets, chrome, W, H):
    # pixel spread, age hold (with issue priority) and occupancy only change which wave
    # marches which ray and when: pixels and statistics are identical
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(-15, 30, 2)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    with pytest.raises(nr.NRError):
        rend.set_pixel_spread(3)   # groups are powers of two
    with pytest.raises(nr.NRError):
        rend.set_pixel_spread(-2)  # -1 is "automatic"
    ref, sref = rend.set_pixel_spread(0).render(W, H, 128)
    try:
        for spread, bpc in [(16, 0), (64, 3), (1024, 1), (1, 0), (16, 3), (0, 2), (-1, 0)]:
            rend.set_pixel_spread(spread).set_occupancy(bpc)
            img, st = rend.render(W, H, 128)
            assert np.array_equal(img, ref), (spread, bpc)
            for k in ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations"):
                assert st[k] == sref[k], (k, spread, bpc)
        # rays per wave: explicit 64 / 32 / 16 (one tile: the fp32 stream, f32_hidden7_stream) and automatic (0: 32 for an fp32 launch of at most 2x
        # its waves' slots, this frame on 8 shards)
        rend.set_pixel_spread(-1).set_occupancy(0)
        for rays in (64, 32, 16, 0):
            rend.set_wave_rays(rays)
            img, st = rend.render(W, H, 128)
            assert np.array_equal(img, ref) and st["ray_steps"] == sref["ray_steps"], rays
            a8 = [rend.render_shard(W, H, 1, 8, k, 128)[0] for k in (0, 7)]
            rend.set_wave_rays(64)
            b8 = [rend.render_shard(W, H, 1, 8, k, 128)[0] for k in (0, 7)]
            assert all(np.array_equal(x, y) for x, y in zip(a8, b8)), rays
        with pytest.raises(nr.NRError):
            rend.set_wave_rays(65)
        with pytest.raises(nr.NRError):
            rend.set_wave_rays(-1)
    finally:
        rend.set_pixel_spread(-1).set_occupancy(0).set_wave_rays(0)


def test_iteration_map(rend, nets, chrome):
    # debug bit 3: each pixel holds the iterations its ray used (a converged ray counts
    # the colouring iteration too), so the map sums to ray-steps + shaded rays
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    iv, nm = nr.camera(0, 0, 2)
    rend.set_view(iv, nm).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    img, st = rend.render(256, 256, 128)
    rend.set_debug(8)
    try:
        m, st2 = rend.render(256, 256, 128)
    finally:
        rend.set_debug(0)
    assert st2["ray_steps"] == st["ray_steps"]
    assert int(m.astype(np.int64).sum()) == st["ray_steps"] + st["rays_shaded"]
    assert m.max() == st["iterations"] <= 128
    assert ((m > 0) | (img == 0)).all()


@pytest.mark.parametrize("schedule", ["persistent", "wavefront"])
@pytest.mark.parametrize("nshards,shard,n", [(1, 0, 5), (3, 1, 3), (1, 0, 40)])
def test_render_batch_matches_single_frames(rend, nets, chrome, nshards, shard, n, schedule):
    """nr_render_batch: frames with their own cameras and frame numbers, in one launch /
    one ray queue (40 frames: two), give each frame's single-frame pixels (persistent
    schedule) and summed stats."""
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32").set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
    rend.set_matcap(chrome)
    rng = np.random.default_rng(7)
    cams = []
    for i in range(n):
        iv, nm = nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0)
        cams.append((iv, nm, int(rng.integers(0, 360))))
    W, H = 96, 77
    rend.set_schedule(schedule)
    imgs, st = rend.render_batch(W, H, cams, 128, band=8, nshards=nshards, shard=shard)
    rend.set_schedule("persistent")
    tot = 0
    for (iv, nm, fr), img in zip(cams, imgs):
        rend.set_view(iv, nm, fr)
        ref, rst = rend.render_shard(W, H, 8, nshards, shard, 128)
        assert np.array_equal(img, ref)
        tot += rst["ray_steps"]
    assert st["ray_steps"] == tot
    rend.set_view(*nr.camera(0, 0, 2), 0)


@pytest.mark.parametrize("prec,spread", [("fp32", 0), ("fp32", 16), ("bf16", -1), ("fp16", -1)])
def test_render_batch_schedules_same_pixels(rend, nets, chrome, prec, spread):
    """Batched launches of >= 4 frames deal pixels block-major by default and, in bf16/fp16,
    take pixel-queue positions from wave-private pools and refill 8 slots at a time.  Each
    frame equals its single-frame render bit for bit, in every precision, on repeated
    launches.  (Round 1 saw the batched bf16/fp16 instance march a group of 16 rays
    differently from run to run: packed-FP32 VALU beside reduced-precision MFMAs, fixed by
    building without packed-FP32 ops -- DESIGN.md section 6, tools/pk_mfma_probe.hip.)"""
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
    rend.set_matcap(chrome)
    rng = np.random.default_rng(11)
    cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(6)]
    W, H = 160, 144
    try:
        refs, tot = [], 0
        for iv, nm, fr in cams:
            rend.set_view(iv, nm, fr)
            ref, rst = rend.render(W, H, 128)
            refs.append(ref)
            tot += rst["ray_steps"]
        rend.set_pixel_spread(spread)
        for trial in range(20 if prec != "fp32" else 3):
            imgs, st = rend.render_batch(W, H, cams, 128)
            ndiff = sum(int((img != ref).sum()) for img, ref in zip(imgs, refs))
            assert ndiff == 0, (trial, ndiff)
            assert st["ray_steps"] == tot, (trial, st["ray_steps"], tot)
    finally:
        rend.set_pixel_spread(-1).set_precision("fp32").set_view(*nr.camera(0, 0, 2), 0)


@pytest.mark.parametrize("schedule", ["persistent", "wavefront"])
def test_render_batch_animation_vs_oracle(rend, nets, chrome, schedule):
    """A batch of an animation (the sphere grid moves with the frame number) equals the
    oracle frame by frame."""
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32").set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
    rend.set_matcap(chrome)
    iv, nm = nr.camera(-15.0, 40.0, 2.0)
    cams = [(iv, nm, f) for f in (0, 90, 180)]
    W, H = 64, 64
    rend.set_schedule(schedule)
    imgs, _ = rend.render_batch(W, H, cams, 128)
    rend.set_schedule("persistent")
    for (iv_, nm_, f), img in zip(cams, imgs):
        ref, _ = oracle.OracleNet(K, B).render(W, H, iv_, nm_, frame=f, color_type=1, matcap=chrome, max_steps=128)
        assert np.array_equal(img, ref)


def test_batch_after_buffer_growth(rend, nets, chrome):
    """A batch, then a larger single frame (the ray queues grow), then the batch again:
    the per-frame staging survives the queue reallocation."""
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32").set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
    rend.set_matcap(chrome)
    cams = [(*nr.camera(0.0, 30.0 * i, 2.0), i) for i in range(3)]
    for schedule in ("persistent", "wavefront"):
        rend.set_schedule(schedule)
        a, _ = rend.render_batch(40, 30, cams, 64)
        rend.set_view(*nr.camera(0, 0, 2), 0)
        rend.render(1100 + (schedule == "wavefront") * 100, 1000, 16)
        b, _ = rend.render_batch(40, 30, cams, 64)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
    rend.set_schedule("persistent")
