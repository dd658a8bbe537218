"""The 16-bit MLP's software-pipelined instruction streams (nr_mlp16_asm.h, generated and
hazard-checked by tools/gen_mlp_asm.py) issue the same instructions on the same operands as the
builtin-compiled form, in a different order: every value must be identical, bit for bit, to the
builtin form (nr_set_debug bit 11) -- for bf16 with the clamped ReLU and with v_pk_max_i16
(bit 9), fp16, 3- and 4-input networks, ragged sizes and inputs beyond the clamp bound."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
from conftest import GEOMS

pytestmark = pytest.mark.gpu
NO_CLAMP = 1 << 9
NO_STREAM = 1 << 11


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


def stream_and_builtin(rend, fn, debug=0):
    rend.set_debug(debug)
    try:
        a = fn()
        rend.set_debug(debug | NO_STREAM)
        b = fn()
    finally:
        rend.set_debug(0)
    return a, b


@pytest.mark.parametrize("prec,debug", [("bf16", 0), ("bf16", NO_CLAMP), ("fp16", 0)])
@pytest.mark.parametrize("geom", GEOMS)
def test_mlp_stream_equals_builtin(rend, nets, geom, prec, debug):
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision(prec)
    rng = np.random.default_rng(21)
    X = rng.uniform(-1.5, 1.5, size=((1 << 18) + 77, 3)).astype(np.float32)
    X[1000:1064] *= 1e4
    X[5000] = (3e6, -1.0, 0.5)       # its chunk takes the max form (beyond LP_INPUT_BOUND)
    X[7000:7010] = 0.0
    X[7010] = (-0.0, 1e-30, -1e-30)
    try:
        a, b = stream_and_builtin(rend, lambda: rend.mlp_forward(X), debug)
        assert np.isfinite(a[np.isfinite(b)]).all()
        assert np.array_equal(a, b, equal_nan=True), (np.abs(a - b).max(), int((a != b).sum()))
    finally:
        rend.set_precision("fp32")


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_mlp_stream_four_inputs(rend, prec):
    """An animation network (x, y, z, frame): the 4th input rides in the input layer's operands."""
    rng = np.random.default_rng(22)
    dims = [4] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) / np.sqrt(dims[i])).astype(np.float32) for i in range(9)]
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    rend.load_mlp(dims, K, B).set_precision(prec)
    X = rng.uniform(-1.2, 1.2, size=(100_003, 4)).astype(np.float32)
    X[:, 3] = rng.integers(0, 400, size=len(X))
    try:
        a, b = stream_and_builtin(rend, lambda: rend.mlp_forward(X))
        assert np.array_equal(a, b), np.abs(a - b).max()
    finally:
        rend.set_precision("fp32")


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_mlp_stream_ragged(rend, nets, prec):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision(prec)
    X = np.random.default_rng(23).uniform(-1.2, 1.2, size=(4096, 3)).astype(np.float32)
    try:
        for n in (1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 4096):
            a, b = stream_and_builtin(rend, lambda: rend.mlp_forward(X[:n]))
            assert np.array_equal(a, b), n
    finally:
        rend.set_precision("fp32")


# ---- the tracer's march MLP (two 32-point tiles per wave: mlp7_x2_stream) -- whole frames

@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


@pytest.mark.parametrize("prec,debug", [("bf16", 0), ("bf16", NO_CLAMP), ("fp16", 0)])
@pytest.mark.parametrize("geom", ["plane_1", "car_1"])
def test_trace_stream_frames_identical(rend, chrome, geom, prec, debug):
    """One frame and a 6-frame batch (the batched instance) with the stream and with the builtin
    form: every pixel identical, and the same ray-step counts."""
    rend.load_h5(nr.geometry_path(geom)).set_precision(prec)
    rend.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
    cams = [nr.camera(5.0 * i, 30.0 * i, 2.0) + (i,) for i in range(6)]
    rend.set_view(*cams[1][:2], 0)
    try:
        (a, sa), (b, sb) = stream_and_builtin(rend, lambda: rend.render(384, 320, 128), debug)
        assert np.array_equal(a, b), int((a != b).sum())
        assert sa["ray_steps"] == sb["ray_steps"]
        (fa, _), (fb, _) = stream_and_builtin(rend, lambda: rend.render_batch(256, 256, cams, 96), debug)
        for i, (x, y) in enumerate(zip(fa, fb)):
            assert np.array_equal(x, y), (i, int((x != y).sum()))
    finally:
        rend.set_precision("fp32")


def test_trace_stream_animation_frames_identical(rend, chrome):
    """A 4-input network: the frame number rides in the stream's input operands."""
    rng = np.random.default_rng(24)
    dims = [4] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) / np.sqrt(dims[i])).astype(np.float32) for i in range(9)]
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    B[-1][:] = 0.3
    rend.load_mlp(dims, K, B).set_precision("bf16")
    rend.set_static(nr.NR_COLOR_FACING, 4).set_scene("v1")
    cams = [nr.camera(0.0, 10.0 * i, 2.0) + (7 * i,) for i in range(4)]
    try:
        (fa, sa), (fb, sb) = stream_and_builtin(rend, lambda: rend.render_batch(192, 160, cams, 64))
        for i, (x, y) in enumerate(zip(fa, fb)):
            assert np.array_equal(x, y), (i, int((x != y).sum()))
        assert sa["ray_steps"] == sb["ray_steps"]
    finally:
        rend.set_static(nr.NR_COLOR_MATCAP, 3).set_precision("fp32")


# ---- k_mlp16's per-CU chunk queue (one 12-wave workgroup per CU, chunks claimed through LDS)

CUQ = 1 << 12


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_mlp_cu_queue_equals_grid_stride(rend, nets, prec):
    """Every point evaluated exactly once by the CU-queue launch (ragged sizes, fewer chunks than
    CUs, a 4-input network below), the same values as the grid-stride launch (bit 12), and repeated
    launches stay right.  (Bit 12 selects the queue.)"""
    dims, K, B = nets["car_1"]
    rend.load_mlp(dims, K, B).set_precision(prec)
    rng = np.random.default_rng(25)
    try:
        for n in (1, 129, 128 * 777 + 5, (1 << 18) + 77, (1 << 20) + 64, 3_000_001):
            X = rng.uniform(-1.2, 1.2, size=(n, 3)).astype(np.float32)
            rend.set_debug(0)
            ref = rend.mlp_forward(X)
            rend.set_debug(CUQ)
            for rep in range(3):
                a = rend.mlp_forward(X)
                assert np.array_equal(a, ref), (n, rep, int((a != ref).sum()))
    finally:
        rend.set_debug(0)
        rend.set_precision("fp32")


# ---- the batched bf16/fp16 tracer with two ray groups per wave (k_trace2) against k_trace

TWO_GROUPS = 1 << 14   # flips the build's default tracer (k_trace) to k_trace2


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("geom,size,frames", [("car_1", 512, 6), ("plane_2", 384, 32), ("plane_1", 200, 3)])
def test_two_group_tracer_frames_identical(rend, chrome, geom, size, frames, prec):
    """Every pixel of a batch (several sizes, up to 32 frames, poses and frame numbers) identical
    between the two-group tracer (nr_set_debug bit 14) and the one-group k_trace, and the same
    ray-step and shaded-ray counts."""
    rend.load_h5(nr.geometry_path(geom)).set_precision(prec)
    rend.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
    cams = [nr.camera(7.0 * (i % 5), 23.0 * i, 2.0) + (i,) for i in range(frames)]
    try:
        rend.set_debug(0)
        a, sa = rend.render_batch(size, size, cams, 128)
        rend.set_debug(TWO_GROUPS)
        b, sb = rend.render_batch(size, size, cams, 128)
        for i, (x, y) in enumerate(zip(a, b)):
            assert np.array_equal(x, y), (i, int((x != y).sum()))
        assert sa["ray_steps"] == sb["ray_steps"] and sa["rays_shaded"] == sb["rays_shaded"], (sa, sb)
    finally:
        rend.set_debug(0)
        rend.set_precision("fp32")


def test_two_group_tracer_animation_and_facing(rend):
    """A 4-input network (the frame number rides in the 128-point MLP's inputs) with facing-ratio
    colouring (the ray direction regenerated from the pixel), batched: identical to k_trace."""
    rng = np.random.default_rng(26)
    dims = [4] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) / np.sqrt(dims[i])).astype(np.float32) for i in range(9)]
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    B[-1][:] = 0.2
    rend.load_mlp(dims, K, B).set_precision("bf16")
    rend.set_static(nr.NR_COLOR_FACING, 4).set_scene("v1")
    cams = [nr.camera(0.0, 11.0 * i, 2.0) + (5 * i,) for i in range(5)]
    try:
        rend.set_debug(0)
        a, sa = rend.render_batch(256, 192, cams, 96)
        rend.set_debug(TWO_GROUPS)
        b, sb = rend.render_batch(256, 192, cams, 96)
        for i, (x, y) in enumerate(zip(a, b)):
            assert np.array_equal(x, y), (i, int((x != y).sum()))
        assert sa["ray_steps"] == sb["ray_steps"]
    finally:
        rend.set_debug(0)
        rend.set_static(nr.NR_COLOR_MATCAP, 3).set_precision("fp32")
