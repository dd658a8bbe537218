"""The BASELINE.json reduced-precision configurations (C3-C5) at their full sizes on the SHIPPED
default path: bf16 / fp16 with the endgame on (NR_ENDGAME_DEFAULT; test_gpu_configs.py covers the
pure 16-bit march).  Size-independent properties: renders are deterministic,
the persistent and wavefront schedules give the same frame and counts, the 8 shards of C4
re-assemble to the single-launch frame, and the frame covers the fp32 frame (bit-exact with the
oracle: test_gpu_configs.py) with the endgame's fixed coverage targets -- IoU >= 0.99 on C3 / C4,
>= 0.98 on C5 (the crops' targets, test_gpu_lowp_contract.py EG_TARGETS).  The endgame's own
bit-exactness against the oracle restatement is test_gpu_endgame.py's (crops)."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr

pytestmark = pytest.mark.gpu


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
    return iv, nm


def iou(a, b):
    fa, fb = a != 0, b != 0
    return (fa & fb).sum() / max((fa | fb).sum(), 1)


def fp32_frame(rend, W, steps):
    rend.set_precision("fp32")
    return rend.render(W, W, steps)[0]


COUNTS = ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations", "endgame_evals", "endgame_switches")


def test_c3_bf16_default(rend, nets, chrome):
    """C3: car_1 2048^2, 256 steps, bf16 at the default endgame: deterministic, persistent ==
    wavefront, IoU >= 0.99 against the fp32 frame."""
    setup(rend, nets, "car_1", "bf16", chrome)
    try:
        a, sa = rend.set_schedule("persistent").render(2048, 2048, 256)
        a2, _ = rend.render(2048, 2048, 256)
        b, sb = rend.set_schedule("wavefront").render(2048, 2048, 256)
    finally:
        rend.set_schedule("persistent")
    assert sa["endgame_switches"] > 0 and sa["endgame_evals"] > 0
    assert np.array_equal(a, a2)
    assert np.array_equal(a, b), int((a != b).sum())
    for k in COUNTS:
        assert sa[k] == sb[k], (k, sa, sb)
    f32 = fp32_frame(rend, 2048, 256)
    v = iou(a, f32)
    print(f"C3 default: IoU {v:.5f}, identical to fp32 {np.mean(a == f32):.4f}")
    assert v >= 0.99


def test_c4_bf16_default_shards(rend, nets, chrome):
    """C4: plane_2 4096^2 bf16 at the default endgame, 8 one-row-band shards (bench.py's layout),
    single-frame and batched: they re-assemble to the single-launch frame exactly; IoU >= 0.99."""
    iv, nm = setup(rend, nets, "plane_2", "bf16", chrome)
    full, st = rend.render(4096, 4096, 128)
    assert st["endgame_switches"] > 0
    shards, steps, fine = [], 0, 0
    for s in range(8):
        img, sst = rend.render_shard(4096, 4096, 1, 8, s, 128)
        shards.append(img)
        steps += sst["ray_steps"]
        fine += sst["endgame_evals"]
        imgs, _ = rend.render_batch(4096, 4096, [(iv, nm, 0)] * 2, 128, band=1, nshards=8, shard=s)
        assert np.array_equal(imgs[0], img) and np.array_equal(imgs[1], img)
    assert np.array_equal(nr.assemble_shards(shards, 4096, 4096, 1, 8), full)
    assert steps == st["ray_steps"] and fine == st["endgame_evals"]
    f32 = fp32_frame(rend, 4096, 128)
    v = iou(full, f32)
    print(f"C4 default: IoU {v:.5f}, identical to fp32 {np.mean(full == f32):.4f}")
    assert v >= 0.99


@pytest.mark.parametrize("geom", ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"])
def test_c5_fp16_default(rend, nets, chrome, geom):
    """C5: the 5 geometries at 2048^2, fp16 at the default endgame: deterministic, IoU >= 0.98
    against the fp32 frame."""
    setup(rend, nets, geom, "fp16", chrome, cam=(-20.0, 35.0, 2.0))
    h, sh = rend.render(2048, 2048, 128)
    h2, sh2 = rend.render(2048, 2048, 128)
    assert np.array_equal(h, h2) and all(sh[k] == sh2[k] for k in COUNTS)
    f32 = fp32_frame(rend, 2048, 128)
    v = iou(h, f32)
    print(f"C5 {geom[:8]} default: IoU {v:.5f}, identical to fp32 {np.mean(h == f32):.4f}")
    assert v >= 0.98
