"""The 16-bit MLP's software-pipelined instruction streams (nr_mlp16_asm.h, generated and
hazard-checked by tools/gen_mlp_asm.py) issue the same instructions on the same operands as the
builtin-compiled form, in a different order: every value must be identical, bit for bit, to the
builtin form (nr_set_debug bit 11) -- for bf16 with the clamped ReLU and with v_pk_max_i16
(bit 9), fp16, 3- and 4-input networks, ragged sizes and inputs beyond the clamp bound.
Round 6: nr_set_debug bit 12 runs nr_mlp_forward's hidden layers on v_mfma_f32_16x16x32 (the
NR_S16_* streams on nr_pack.cpp's pack_lowp_s16 layout; measured slower than the default 32x32x16
stream, kept as the A/B form); both must equal the builtin form and the oracle's restatement."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
from conftest import GEOMS

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)
NO_CLAMP = 1 << 9
NO_STREAM = 1 << 11
S16 = 1 << 12


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


@pytest.mark.parametrize("prec,debug", [("bf16", 0), ("bf16", NO_CLAMP), ("fp16", 0), ("bf16", S16),
                                        ("bf16", S16 | NO_CLAMP), ("fp16", S16)])
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
@pytest.mark.parametrize("debug", [0, S16])
def test_mlp_stream_ragged(rend, nets, prec, debug):
    dims, K, B = nets["plane_1"]
    rend.load_mlp(dims, K, B).set_precision(prec)
    X = np.random.default_rng(23).uniform(-1.2, 1.2, size=(4096, 3)).astype(np.float32)
    try:
        for n in (1, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 4096):
            a, b = stream_and_builtin(rend, lambda: rend.mlp_forward(X[:n]), debug)
            assert np.array_equal(a, b), n
    finally:
        rend.set_precision("fp32")


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("debug", [0, S16])
@pytest.mark.parametrize("geom", GEOMS)
def test_mlp_forward_equals_oracle_restatement(rend, nets, geom, prec, debug):
    """nr_mlp_forward (k_mlp16: the 32x32x16 stream by default, the 16x16x32 one with bit 12)
    against the oracle's restatement of the GPU's 16-bit arithmetic (precision 1 / 2), bit for bit."""
    import oracle
    dims, K, B = nets[geom]
    rend.load_mlp(dims, K, B).set_precision(prec).set_debug(debug)
    X = np.random.default_rng(24).uniform(-1.2, 1.2, size=(16384 + 45, 3)).astype(np.float32)
    try:
        y = rend.mlp_forward(X)
    finally:
        rend.set_debug(0).set_precision("fp32")
    ref = oracle.OracleNet(K, B).forward(X, precision=1 if prec == "bf16" else 2, nthreads=16)
    assert np.array_equal(y, ref), int((y != ref).sum())
