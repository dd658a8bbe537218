"""fp32 clamped ReLU (nr_mlp16.h mlp16_fp32_nt<.., CL>): on the power-of-two-scaled fp32 pack
(nr_pack.cpp pack_fp32_16) the bias add and the ReLU are one v_add_f32 / v_fma_f32 with the
clamp bit.  The network output is the unscaled network's bit for bit, so every fp32 parity
test against the oracle covers it; these tests add the inputs beyond F32_INPUT_BOUND (the
kernel's add + max form on the same pack) and the A/B against that form (nr_set_debug
bit 9) on every render path."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
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
    """fn() with the clamped ReLU, then with add + max (debug bit 9)."""
    rend.set_debug(0)
    a = fn()
    rend.set_debug(NO_CLAMP)
    try:
        b = fn()
    finally:
        rend.set_debug(0)
    return a, b


@pytest.mark.parametrize("geom", GEOMS)
def test_mlp_clamp_bitexact_with_fallback(rend, nets, geom):
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    rng = np.random.default_rng(11)
    X = rng.uniform(-1.5, 1.5, size=(30000, 3)).astype(np.float32)
    X[777] = (3000.0, 0.0, 0.0)   # its 64-point chunk exceeds F32_INPUT_BOUND: add + max form
    X[20000:20100] *= 600.0        # large but within the bound: clamped form
    X[25000:25064] = 0.0           # zero inputs (the chains' +0 start)
    a, b = both(rend, lambda: rend.mlp_forward(X))
    ref = oracle.OracleNet(K, B).forward(X)
    assert np.array_equal(a, ref), np.abs(a - ref).max()
    assert np.array_equal(b, ref)


@pytest.mark.parametrize("schedule", ["persistent", "wavefront"])
def test_render_clamp_equals_max(rend, nets, chrome, schedule):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision("fp32").set_schedule(schedule)
    rend.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
    rng = np.random.default_rng(12)
    cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(4)]
    try:
        (ia, sa), (ib, sb) = both(rend, lambda: rend.render_batch(96, 80, cams, 128))
        assert all(np.array_equal(x, y) for x, y in zip(ia, ib))
        assert sa["ray_steps"] == sb["ray_steps"] and sa["rays_shaded"] == sb["rays_shaded"]
        rend.set_view(*cams[0])
        (fa, _), (fb, _) = both(rend, lambda: rend.render(96, 80, 128))
        assert np.array_equal(fa, fb) and np.array_equal(fa, ia[0])
        iv, nm, _ = cams[0]
        ref, _ = oracle.OracleNet(K, B).render(96, 80, iv, nm, color_type=1, matcap=chrome, max_steps=128)
        assert np.array_equal(fa, ref)
    finally:
        rend.set_schedule("persistent").set_view(*nr.camera(0, 0, 2), 0)


def test_animation_frame_beyond_bound(rend):
    """A 4-input network: a frame number beyond F32_INPUT_BOUND sends every wave to the
    add + max form; both frames bit-exact with the oracle."""
    rng = np.random.default_rng(13)
    dims = [4] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) * (1.0 / np.sqrt(dims[i]))).astype(np.float32) for i in range(9)]
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    B[-1][0] = 0.3
    rend.load_mlp(dims, K, B).set_precision("fp32").set_static(nr.NR_COLOR_FACING, 4).set_scene("v1")
    iv, nm = nr.camera(10.0, 20.0, 2.0)
    try:
        for frame in (7, 5000):
            rend.set_view(iv, nm, frame)
            img, _ = rend.render(64, 48, 64)
            ref, _ = oracle.OracleNet(K, B).render(64, 48, iv, nm, frame=frame, color_type=nr.NR_COLOR_FACING,
                                                   num_inputs=4, max_steps=64)
            assert np.array_equal(img, ref), frame
    finally:
        rend.set_static(nr.NR_COLOR_MATCAP, 3).set_view(*nr.camera(0, 0, 2), 0)


def test_unscalable_network_uses_max_form(rend):
    """A network whose interval bounds leave the scale range (first-layer weights ~1e27: the
    bound for inputs within +-1024 is past 2^100, so clamp_scales refuses it) keeps an
    unscaled pack and the add + max form on every wave: still the oracle's values bit for
    bit (all finite)."""
    rng = np.random.default_rng(14)
    dims = [3] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) / np.sqrt(dims[i])).astype(np.float32) for i in range(9)]
    K[0] = (K[0] * 1e27).astype(np.float32)
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    X = np.random.default_rng(15).uniform(-1.0, 1.0, size=(5000, 3)).astype(np.float32)
    X[100:164] = 1e-3
    y = rend.mlp_forward(X)
    ref = oracle.OracleNet(K, B).forward(X)
    assert np.isfinite(ref).all()
    assert np.array_equal(y, ref)


@pytest.mark.parametrize("geom", ["plane_1", "car_1"])
def test_tiny_inputs_stay_bitexact(rend, nets, geom):
    """ADVICE r2 / VERDICT r2 item 9: inputs near 1e-25 (and exact zeros, signed) reach the scaled
    pack's chains as tiny products; the layer-0 biases are nonzero, so every fmaf result stays
    normal in both the scaled and the unscaled evaluation, and the output is the oracle's."""
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision("fp32")
    rng = np.random.default_rng(21)
    X = (rng.uniform(-1, 1, size=(8192, 3)) * 10.0 ** rng.uniform(-30, -20, size=(8192, 3))).astype(np.float32)
    X[:64] = 0.0
    X[64:128] = -0.0
    X[128:192, 0] = np.float32(1e-38)   # subnormal-adjacent inputs
    a, b = both(rend, lambda: rend.mlp_forward(X))
    ref = oracle.OracleNet(K, B).forward(X)
    assert np.array_equal(a, ref) and np.array_equal(b, ref)


def test_tiny_weight_network_is_not_scaled(rend):
    """A network with a nonzero weight below 2^-60 (and a zero bias) could produce a chain result
    near f32's subnormal range: clamp_scales refuses to scale it (the add + max form on the
    unscaled pack), and inputs of 1e-30 through it stay the oracle's bit for bit."""
    rng = np.random.default_rng(22)
    dims = [3] + [32] * 8 + [1]
    K = [rng.uniform(-0.5, 0.5, size=(dims[i], dims[i + 1])).astype(np.float32) for i in range(len(dims) - 1)]
    B = [rng.uniform(-0.05, 0.05, size=dims[i + 1]).astype(np.float32) for i in range(len(dims) - 1)]
    K[0][:, 3] = np.float32(1e-25)
    B[0][3] = 0.0
    X = np.concatenate([rng.uniform(-1, 1, size=(2048, 3)), rng.uniform(-1, 1, size=(2048, 3)) * 1e-30]).astype(np.float32)
    rend.load_mlp(dims, K, B).set_precision("fp32")
    a, b = both(rend, lambda: rend.mlp_forward(X))
    ref = oracle.OracleNet(K, B).forward(X)
    assert np.array_equal(a, ref) and np.array_equal(b, ref)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_cancelling_bias_network(rend, prec):
    """the clamp margins must hold where a unit's bias cancels large products (the
    evaluation's rounding is relative to the terms, not to the small result): biases of -30 to
    -45 against weights of up to 4.  clamp_scales bounds with top + eps * sum|terms|; the clamped
    form equals the max form bit for bit (and fp32 equals the oracle)."""
    rng = np.random.default_rng(23)
    dims = [3] + [32] * 8 + [1]
    K = [rng.uniform(0.5, 4.0, size=(dims[i], dims[i + 1])).astype(np.float32) for i in range(len(dims) - 1)]
    K = [k * (1.0 / dims[i]) * np.where(rng.uniform(size=k.shape) < 0.9, 1, -1).astype(np.float32)
         for i, k in enumerate(K)]
    B = [np.full(dims[i + 1], -0.95, np.float32) * np.abs(K[i]).sum(0) * 1.5 for i in range(len(dims) - 1)]
    B[0] = rng.uniform(-45, -30, size=32).astype(np.float32)
    K[0] *= 30.0
    X = rng.uniform(-1.5, 1.5, size=(20000, 3)).astype(np.float32)
    rend.load_mlp(dims, K, B).set_precision(prec)
    try:
        a, b = both(rend, lambda: rend.mlp_forward(X))
        assert np.array_equal(a, b), np.abs(a - b).max()
        if prec == "fp32":
            assert np.array_equal(a, oracle.OracleNet(K, B).forward(X))
    finally:
        rend.set_precision("fp32")
