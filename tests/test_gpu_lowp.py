"""bf16 clamped ReLU (nr_mlp16.h relu_clamp_bf16_x*): the ReLU folded into the conversion's
clamp bit on the power-of-two-scaled pack (nr_pack.cpp clamp_scales) gives the same values,
bit for bit, as cvt + v_pk_max_i16 on the same pack (nr_set_debug bit 9), in the MLP and in
every render path; inputs beyond LP_INPUT_BOUND take the v_pk_max form inside the kernel."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
from conftest import GEOMS

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)
NO_CLAMP = 1 << 9


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def both(rend, fn):
    """fn() with the clamped ReLU, then with v_pk_max_i16 (debug bit 9)."""
    rend.set_debug(0)
    a = fn()
    rend.set_debug(NO_CLAMP)
    try:
        b = fn()
    finally:
        rend.set_debug(0)
    return a, b


@pytest.mark.parametrize("geom", GEOMS)
def test_mlp_clamp_equals_pkmax(rend, nets, geom):
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision("bf16")
    rng = np.random.default_rng(3)
    X = rng.uniform(-1.5, 1.5, size=(50000, 3)).astype(np.float32)
    X[777] = (3e6, 0.0, 0.0)      # its 64-point chunk exceeds LP_INPUT_BOUND: v_pk_max form
    X[40000:40100] *= 1e5         # large but within the bound: clamped form, still exact
    a, b = both(rend, lambda: rend.mlp_forward(X))
    assert np.isfinite(a).all()
    assert np.array_equal(a, b), np.abs(a - b).max()
    rend.set_precision("fp32")


def test_mlp_clamp_close_to_fp32(rend, nets):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B)
    X = np.random.default_rng(4).uniform(-1.2, 1.2, size=(20000, 3)).astype(np.float32)
    y32 = rend.set_precision("fp32").mlp_forward(X)
    ybf = rend.set_precision("bf16").mlp_forward(X)
    err = np.abs(ybf - y32).max()
    assert err < 0.05, err
    rend.set_precision("fp32")


@pytest.mark.parametrize("schedule", ["persistent", "wavefront"])
def test_render_clamp_equals_pkmax(rend, nets, chrome, schedule):
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision("bf16").set_schedule(schedule)
    rend.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
    rng = np.random.default_rng(5)
    cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(5)]
    try:
        (ia, sa), (ib, sb) = both(rend, lambda: rend.render_batch(96, 80, cams, 128))
        assert all(np.array_equal(x, y) for x, y in zip(ia, ib))
        assert sa["ray_steps"] == sb["ray_steps"] and sa["rays_shaded"] == sb["rays_shaded"]
        rend.set_view(*cams[0])
        (fa, _), (fb, _) = both(rend, lambda: rend.render(96, 80, 128))
        assert np.array_equal(fa, fb) and np.array_equal(fa, ia[0])
    finally:
        rend.set_precision("fp32").set_schedule("persistent").set_view(*nr.camera(0, 0, 2), 0)


def test_animation_clamp_frame_bound(rend, chrome):
    """A 4-input network: frames within LP_INPUT_BOUND use the clamped form, a batch holding
    a frame number beyond it falls back for the whole launch; both equal the v_pk_max form."""
    rng = np.random.default_rng(6)
    dims = [4] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) * (1.0 / np.sqrt(dims[i]))).astype(np.float32) for i in range(9)]
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    B[-1][0] = 0.3
    rend.load_mlp(dims, K, B).set_precision("bf16").set_static(nr.NR_COLOR_FACING, 4).set_scene("v1")
    iv, nm = nr.camera(0, 0, 2)
    try:
        for frames in ([0, 1, 2, 3], [0, 5, 2_000_000, 3]):
            cams = [(iv, nm, f) for f in frames]
            (ia, sa), (ib, sb) = both(rend, lambda: rend.render_batch(64, 64, cams, 64))
            assert all(np.array_equal(x, y) for x, y in zip(ia, ib)), frames
            assert sa["ray_steps"] == sb["ray_steps"]
    finally:
        rend.set_precision("fp32").set_static(nr.NR_COLOR_MATCAP, 3).set_view(iv, nm, 0)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("debug", [0, NO_CLAMP])
def test_mlp_128_point_form_equals_64_point_form(rend, nets, prec, debug):
    """k_mlp16 runs bf16/fp16 on 128 points per wave (nr_mlp16.h mlp32_lowp_128: four 32-point
    tiles from two points per lane); a call of at most 64 points takes the 64-point form
    (mlp32_lowp_nt, the tracers' MLP).  Same arithmetic per point: every point's value is the
    same bit for bit, whichever tile, lane half and chunk carries it (ragged ends included)."""
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision(prec).set_debug(debug)
    try:
        X = np.random.default_rng(11).uniform(-1.3, 1.3, size=(64 * 24 + 37, 3)).astype(np.float32)
        X[5 * 64 + 9] = (2e6, 0.0, 0.0)  # beyond LP_INPUT_BOUND: this 128-point chunk takes the max form
        big = rend.mlp_forward(X)
        for c0 in range(0, len(X), 64):
            small = rend.mlp_forward(X[c0:c0 + 64])
            assert np.array_equal(big[c0:c0 + 64], small), (c0, np.abs(big[c0:c0 + 64] - small).max())
        # and 65..127-point calls: a 128-point chunk whose second set is ragged
        for n in (65, 100, 127):
            assert np.array_equal(rend.mlp_forward(X[:n]), big[:n]), n
    finally:
        rend.set_debug(0)
        rend.set_precision("fp32")


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_lowp_ragged_frames_schedules_agree(rend, nets, chrome, prec):
    """The bf16/fp16 persistent tracers generate rays in bulk into a per-wave LDS ring
    (nr_trace.hip, DENSE): tiny and ragged frames, 0/1/7 march steps, lane caps of 1-64 rays per
    wave and batched launches all give the wavefront schedule's pixels and ray-steps (a separate
    kernel path with the same per-ray arithmetic)."""
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
    rend.set_matcap(chrome)
    iv, nm = nr.camera(-10.0, 25.0, 2.0)
    cams = [(*nr.camera(-10.0 + 7 * i, 25.0 + 40 * i, 2.0), i) for i in range(5)]
    try:
        for W, H, steps in [(1, 1, 128), (3, 5, 128), (65, 1, 128), (1, 67, 128), (130, 3, 128),
                            (97, 61, 0), (97, 61, 1), (97, 61, 7), (200, 131, 128)]:
            rend.set_view(iv, nm, 0).set_schedule("wavefront")
            ref, sref = rend.render(W, H, steps)
            bref, bsref = rend.render_batch(W, H, cams, steps)
            rend.set_schedule("persistent")
            for rays in (64, 16, 5, 1):
                rend.set_wave_rays(rays).set_view(iv, nm, 0)
                img, st = rend.render(W, H, steps)
                assert np.array_equal(img, ref), (W, H, steps, rays)
                assert st["ray_steps"] == sref["ray_steps"] and st["rays_shaded"] == sref["rays_shaded"], (W, H, steps, rays)
                imgs, bst = rend.render_batch(W, H, cams, steps)
                assert all(np.array_equal(x, y) for x, y in zip(imgs, bref)), (W, H, steps, rays)
                assert bst["ray_steps"] == bsref["ray_steps"], (W, H, steps, rays)
    finally:
        rend.set_wave_rays(0).set_schedule("persistent").set_precision("fp32").set_view(*nr.camera(0, 0, 2), 0)
