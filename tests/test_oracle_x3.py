"""The oracle's fp32x3 emulation (nr_oracle.c mlp_point_gpu_x3), which pins the bf16/fp16 tracers'
normals since round 4 (nr_mlp16.h mlp16_x3_normal), checked on the CPU against the reference's
network evaluated exactly (tests/golden/mlp_kat.npz, fp64 over the h5py weights) and against the
oracle's own fp32 path where the split does not apply.  The pack is the library's (nr_pack_x3),
computed on the host -- no GPU call."""
import os

import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
from conftest import GEOMS


@pytest.mark.parametrize("geom", GEOMS)
def test_pack_x3_every_bundled_network(nets, geom):
    dims, K, B = nets[geom]
    a, f, ok = nr.pack_x3(dims, K, B)
    nh = len(dims) - 3  # hidden 32x32 layers
    assert ok, geom
    assert a.dtype == np.uint16 and f.dtype == np.float32
    # layer-0 operands (512) + 2048 per hidden layer (hi and residual, 2 k-steps); floats: the
    # scaled biases (32 per layer), the final weights, bias and the scales
    assert a.size == 512 + 2048 * nh, a.size
    assert f.size >= 32 + 32 * nh + 35, f.size


@pytest.mark.parametrize("geom", GEOMS)
def test_x3_emulation_within_fp32_class_band(golden, nets, geom):
    """The emulated fp32x3 MLP on the KAT points lands within the fp32x3 precision's own contract
    (tests/test_gpu_fp32x3.py test_x3_mlp_kat): max |y - fp64| <= 1e-5."""
    dims, K, B = nets[geom]
    X = golden["kat"]["X"]
    ref = golden["kat"][geom]
    net = oracle.OracleNet(K, B, x3_pack=nr.pack_x3(dims, K, B)[:2])
    y3 = net.forward(X, precision=4)[:, 0]
    y32 = net.forward(X, precision=0)[:, 0]
    e3 = np.abs(y3.astype(np.float64) - ref)
    e32 = np.abs(y32.astype(np.float64) - ref)
    assert e3.max() <= 1e-5, (e3.max(), e32.max())
    assert e3.mean() <= 5 * e32.mean() + 1e-9, (e3.mean(), e32.mean())
    assert not np.array_equal(y3, y32)  # the split path ran


def test_x3_emulation_falls_back_to_fp32_outside_bounds(nets):
    """Points with a coordinate beyond X3_INPUT_BOUND (4) take the fp32 MLP, bit-exact; points
    inside take the split -- per point, whatever else the batch holds."""
    dims, K, B = nets["plane_1"]
    rng = np.random.default_rng(3)
    X = rng.uniform(-1, 1, size=(256, 3)).astype(np.float32)
    X[::2, 1] *= 8.0  # every other point leaves the bounds where |y| > 4
    out = np.abs(X).max(axis=1) > 4.0
    assert out.any() and (~out).any()
    net = oracle.OracleNet(K, B, x3_pack=nr.pack_x3(dims, K, B)[:2])
    y3 = net.forward(X, precision=4)
    y32 = net.forward(X, precision=0)
    np.testing.assert_array_equal(y3[out], y32[out])
    assert not np.array_equal(y3[~out], y32[~out])
    # the same points alone give the same values (no batch dependence)
    np.testing.assert_array_equal(net.forward(X[~out], precision=4), y3[~out])


def test_x3_normals_in_the_bf16_render(nets):
    """A small bf16 oracle render with the x3 pack differs from the fp32-normal one only in its
    shading (same coverage, same ray-steps: the march does not use the normals)."""
    dims, K, B = nets["plane_1"]
    iv, nm = nr.camera(-18.8, 149.8, 2.27)
    a = oracle.OracleNet(K, B)
    b = oracle.OracleNet(K, B, x3_pack=nr.pack_x3(dims, K, B)[:2])
    ia, sa = a.render(48, 48, iv, nm, precision=1, max_steps=200)
    ib, sb = b.render(48, 48, iv, nm, precision=1, max_steps=200)
    assert sa["ray_steps"] == sb["ray_steps"] and sa["rays_hit"] == sb["rays_hit"] > 100
    assert sa["shade_evals"] == sb["shade_evals"]
    assert not np.array_equal(ia, ib)


@pytest.mark.parametrize("geom", ["plane_1", "car_1"])
def test_mfma_fast_path_equals_generic(nets, geom):
    """The restatement's decoded-operand fast path (nr_oracle.c mfma_fast) and its generic form
    (mfma_sum_e on doubles) are the same arithmetic: bf16, fp16 and fp32x3 outputs bit for bit."""
    dims, K, B = nets[geom]
    X = np.random.default_rng(5).uniform(-1.3, 1.3, size=(384, 3)).astype(np.float32)
    net = oracle.OracleNet(K, B, x3_pack=nr.pack_x3(dims, K, B)[:2])
    try:
        fast = {p: net.forward(X, precision=p, nthreads=1) for p in (1, 2, 4)}
        oracle.set_mfma_model(3, -1)
        slow = {p: net.forward(X, precision=p, nthreads=1) for p in (1, 2, 4)}
    finally:
        oracle.set_mfma_model(3, 26)
    for p in (1, 2, 4):
        np.testing.assert_array_equal(fast[p], slow[p])


def _from16(u, prec):
    if prec == "f16":
        return u.view(np.float16).astype(np.float64)
    return (u.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


@pytest.mark.parametrize("prec,emin", [("f16", -14), ("bf16", -126)])
def test_mfma_model_against_measured_hardware(golden_dir, prec, emin):
    """The oracle's model of one v_mfma_f32_32x32x16_{f16,bf16} output (nr_oracle.c mfma_sum_e,
    both its generic and fast forms) against outputs measured on gfx950 (tests/golden/mfma_*.npz,
    made by tests/golden/make_mfma_golden.py from tools/mfma_cases.py and tools/mfma_model.py
    runs): the 167 hand-built dot products and 10,240 random outputs over five kinds of operand
    distribution, every one bit for bit."""
    z = np.load(os.path.join(golden_dir, f"mfma_{prec}.npz"))
    for i in range(len(z["hand_d"])):
        for fast in (0, 1):
            r = oracle.mfma_sum(z["hand_c"][i], z["hand_a"][i], z["hand_b"][i], emin, fast)
            assert np.float32(r) == z["hand_d"][i], (i, fast, r, float(z["hand_d"][i]))
    for kind in ("cancel", "generic", "residual", "tiny", "x3_like"):
        A, B = _from16(z[kind + "_A"], prec), _from16(z[kind + "_B"], prec)
        C, D = z[kind + "_C"], z[kind + "_D"]
        bad = 0
        for m in range(A.shape[0]):
            for r in range(32):
                for c in range(32):
                    v = oracle.mfma_sum(C[m, r, c], A[m, r], B[m, :, c], emin, (r + c) & 1)
                    bad += np.float32(v) != D[m, r, c]
        assert bad == 0, (kind, bad)


def test_pack_x3_rejects_non_fused_shapes():
    """nr_pack_x3 takes [3|4, 32, ..., 32, 1] only; any other shape is NR_E_INVALID with a message
    (the library's error convention), not a crash."""
    rng = np.random.default_rng(2)
    dims = [3, 48, 1]
    K = [rng.standard_normal((3, 48)).astype(np.float32), rng.standard_normal((48, 1)).astype(np.float32)]
    B = [np.zeros(48, np.float32), np.zeros(1, np.float32)]
    with pytest.raises(Exception) as e:
        nr.pack_x3(dims, K, B)
    assert "fused" in str(e.value) or "invalid" in str(e.value).lower()


def test_x3_oracle_pack_lifecycle(nets):
    """The oracle's decoded x3 operands follow the pack it is handed: two networks alternating in
    one process give each its own values (or_set_x3_pack re-decodes on every call)."""
    X = np.random.default_rng(8).uniform(-1, 1, size=(64, 3)).astype(np.float32)
    outs = {}
    for g in ("plane_1", "car_1", "plane_1"):
        dims, K, B = nets[g]
        y = oracle.OracleNet(K, B, x3_pack=nr.pack_x3(dims, K, B)[:2]).forward(X, precision=4)
        if g in outs:
            np.testing.assert_array_equal(outs[g], y)
        outs[g] = y
    assert not np.array_equal(outs["plane_1"], outs["car_1"])
