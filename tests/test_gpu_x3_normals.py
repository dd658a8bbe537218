"""The bf16/fp16 tracers' normals in fp32x3 (round 4; nr_mlp16.h mlp16_x3_normal): the four
tetrahedron samples of every coloured ray (surfaceNormal, volumeRender_kernel.cu:361-377) go
through the fp32x3 split of the library's x3 pack instead of the fp32 MLP; a point outside the
pack's input bounds (|x|, |y|, |z| > 4, or a 4-input network's frame > 1024) takes the fp32 MLP.
nr_set_debug bit 15 selects the fp32 normals (the r3 behaviour) for A/B.  Checked here:
  * the march is untouched: same ray-steps, coverage and shaded rays with either normal form;
  * persistent and wavefront schedules, single-frame and batched launches give the same pixels
    in both forms (each path carries the same per-point rule);
  * each form is bit-exact with the oracle restating the same normals (oracle.OracleNet with or
    without x3_pack; the matrix core's summation as nr_oracle.c mfma_sum_e models it);
  * the fallback: a 4-input network whose frames are beyond X3_FRAME_BOUND gives the fp32-normal
    frame bit for bit; a batch mixing in- and out-of-bound frames gives each its own form."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
from conftest import compare_frames

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)
FP32_NORMALS = 1 << 15
PREC = {"bf16": 1, "fp16": 2}


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_x3_normals_against_their_emulation(rend, nets, chrome, prec):
    dims, K, B = nets["car_1"]
    pack = nr.pack_x3(dims, K, B)
    assert pack[2]
    iv, nm = nr.camera(-10.0, 25.0, 2.0)
    rend.load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
    rend.set_matcap(chrome).set_view(iv, nm, 0)
    W = H = 160
    try:
        a, sa = rend.render(W, H, 128)
        aw, saw = rend.set_schedule("wavefront").render(W, H, 128)
        rend.set_schedule("persistent").set_debug(FP32_NORMALS)
        b, sb = rend.render(W, H, 128)
        bw, sbw = rend.set_schedule("wavefront").render(W, H, 128)
    finally:
        rend.set_debug(0).set_schedule("persistent").set_precision("fp32")
    assert np.array_equal(a, aw) and np.array_equal(b, bw)
    for k in ("ray_steps", "rays_hit", "rays_shaded", "shade_evals"):
        assert sa[k] == sb[k] == saw[k] == sbw[k], (k, sa, sb)
    assert np.array_equal(a != 0, b != 0)
    assert not np.array_equal(a, b)
    kw = dict(color_type=1, matcap=chrome, max_steps=128, nthreads=16, precision=PREC[prec])
    ea, _ = oracle.OracleNet(K, B, x3_pack=pack[:2]).render(W, H, iv, nm, **kw)
    eb, _ = oracle.OracleNet(K, B).render(W, H, iv, nm, **kw)
    # each form bit-exact with the oracle restating it (nr_oracle.c mfma_sum_e / mlp_point_gpu_x3)
    assert np.array_equal(a, ea), compare_frames(a, ea)
    assert np.array_equal(b, eb), compare_frames(b, eb)


def _net4(seed=41, scale=1.4):
    """a [4, 32 x 8, 1] network whose x3 and fp32 normals give visibly different texels (checked
    on the oracle: 3,982 of 4,096 pixels at 64^2)"""
    rng = np.random.default_rng(seed)
    dims = [4] + [32] * 8 + [1]
    K = [(rng.standard_normal((dims[i], dims[i + 1])) * (scale / np.sqrt(dims[i]))).astype(np.float32) for i in range(9)]
    B = [(rng.standard_normal(dims[i + 1]) * 0.05).astype(np.float32) for i in range(9)]
    B[-1][0] = 0.3
    return dims, K, B


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_x3_normals_frame_bound_fallback(rend, chrome, prec):
    dims, K, B = _net4()
    assert nr.pack_x3(dims, K, B)[2]
    rend.load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 4).set_scene("v1")
    rend.set_matcap(chrome)
    iv, nm = nr.camera(0, 0, 2)
    frames = [0, 5, 2000, 3]  # 2000 > X3_FRAME_BOUND: that frame's normals in fp32
    cams = [(iv, nm, f) for f in frames]
    try:
        ia, sa = rend.render_batch(64, 64, cams, 64)
        rend.set_debug(FP32_NORMALS)
        ib, sb = rend.render_batch(64, 64, cams, 64)
        rend.set_view(iv, nm, 2000)
        fb, _ = rend.render(64, 64, 64)
        rend.set_debug(0)
        fa, _ = rend.render(64, 64, 64)
    finally:
        rend.set_debug(0).set_precision("fp32").set_static(nr.NR_COLOR_MATCAP, 3).set_view(iv, nm, 0)
    assert sa["ray_steps"] == sb["ray_steps"]
    assert np.array_equal(ia[2], ib[2]) and np.array_equal(fa, fb) and np.array_equal(fa, ia[2])
    assert sum(not np.array_equal(x, y) for x, y in zip(ia, ib)) >= 1
    # the oracle with the x3 pack restates the same per-point rule
    pack = nr.pack_x3(dims, K, B)
    net = oracle.OracleNet(K, B, x3_pack=pack[:2])
    for f, img in zip(frames, ia):
        ref, _ = net.render(64, 64, iv, nm, frame=f, color_type=1, matcap=chrome, num_inputs=4, max_steps=64,
                            precision=PREC[prec])
        assert np.array_equal(img, ref), (f, compare_frames(img, ref))
