"""Randomized cross-checks of the persistent tracer over the shapes and knobs it supports
(fixed seeds, small frames): every case exercises a different mix of frame size (ragged,
tiny), march-step cap, camera and frame number, scene, colouring, row-band sharding,
rays per wave, pixel spread and batching.

  fp32: the persistent render equals the C oracle's (volumeRender_kernel.cu:608-692 restated,
        oracle/nr_oracle.c) bit for bit, and each frame of a batch equals its single render;
  bf16 / fp16 / fp32x3: the persistent render equals the wavefront schedule's (a separate
        kernel path with the same per-ray arithmetic), and batches equal single renders.
Schedules and knobs only change which wave marches which ray and when, never a pixel."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)
SCENES = ["v1", "tanh", "subtract", "cylinders", "displace", "round"]


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def case(seed):
    rng = np.random.default_rng(seed)
    W, H = int(rng.integers(1, 161)), int(rng.integers(1, 121))
    steps = int(rng.choice([0, 1, 5, 64, 128, 256], p=[0.04, 0.04, 0.07, 0.3, 0.35, 0.2]))
    return dict(W=W, H=H, steps=steps, rx=float(rng.uniform(-40, 40)),
                ry=float(rng.uniform(0, 360)), zoom=float(rng.uniform(1.6, 2.6)), frame=int(rng.integers(0, 360)),
                scene=SCENES[int(rng.integers(0, len(SCENES)))], color=int(rng.integers(0, 2)),
                nshards=int(rng.choice([1, 2, 3, 8])), band=int(rng.choice([1, 3, 8])),
                rays=int(rng.choice([0, 7, 32, 64])), spread=int(rng.choice([-1, 0, 16])),
                geom=["plane_1", "car_1", "plane_2"][int(rng.integers(0, 3))])


def setup(rend, nets, chrome, c, prec):
    dims, K, B = nets[c["geom"]]
    rend.load_mlp(dims, K, B).set_precision(prec).set_static(c["color"], 3).set_scene(c["scene"])
    rend.set_matcap(chrome).set_wave_rays(c["rays"]).set_pixel_spread(c["spread"])
    iv, nm = nr.camera(c["rx"], c["ry"], c["zoom"])
    rend.set_view(iv, nm, c["frame"])
    return K, B, iv, nm


def reset(rend):
    rend.set_wave_rays(0).set_pixel_spread(-1).set_schedule("persistent").set_precision("fp32")
    rend.set_view(*nr.camera(0, 0, 2), 0)


def batch_cams(c, n=3):
    return [(*nr.camera(c["rx"] + 5 * i, c["ry"] + 30 * i, c["zoom"]), c["frame"] + i) for i in range(n)]


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_fp32_vs_oracle(rend, nets, chrome, seed):
    c = case(seed)
    try:
        K, B, iv, nm = setup(rend, nets, chrome, c, "fp32")
        img, st = rend.render(c["W"], c["H"], c["steps"])
        ref, rst = oracle.OracleNet(K, B).render(c["W"], c["H"], iv, nm, frame=c["frame"], color_type=c["color"],
                                                 scene=nr.NR_SCENE[c["scene"]], matcap=chrome, max_steps=c["steps"],
                                                 nthreads=8)
        assert np.array_equal(img, ref), (c, int((img != ref).sum()))
        assert st["ray_steps"] == rst["ray_steps"], c
        # the same frame as row-band shards, and a batch of poses against single renders
        shard = c["nshards"] - 1
        sh, _ = rend.render_shard(c["W"], c["H"], c["band"], c["nshards"], shard, c["steps"])
        rows = [y for y in range(c["H"]) if (y // c["band"]) % c["nshards"] == shard]
        assert np.array_equal(sh.reshape(-1, c["W"])[: len(rows)], img[rows]), c
        cams = batch_cams(c)
        imgs, _ = rend.render_batch(c["W"], c["H"], cams, c["steps"])
        for (iv2, nm2, f2), b in zip(cams, imgs):
            rend.set_view(iv2, nm2, f2)
            s1, _ = rend.render(c["W"], c["H"], c["steps"])
            assert np.array_equal(b, s1), c
    finally:
        reset(rend)


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32x3"])
@pytest.mark.parametrize("seed", range(100, 108))
def test_fuzz_lowp_schedules_agree(rend, nets, chrome, prec, seed):
    c = case(seed)
    try:
        setup(rend, nets, chrome, c, prec)
        a, sa = rend.set_schedule("persistent").render(c["W"], c["H"], c["steps"])
        b, sb = rend.set_schedule("wavefront").render(c["W"], c["H"], c["steps"])
        assert np.array_equal(a, b), (c, int((a != b).sum()))
        assert sa["ray_steps"] == sb["ray_steps"], c
        rend.set_schedule("persistent")
        cams = batch_cams(c, 5)
        imgs, _ = rend.render_batch(c["W"], c["H"], cams, c["steps"])
        for (iv2, nm2, f2), bi in zip(cams, imgs):
            rend.set_view(iv2, nm2, f2)
            s1, _ = rend.render(c["W"], c["H"], c["steps"])
            assert np.array_equal(bi, s1), c
    finally:
        reset(rend)
