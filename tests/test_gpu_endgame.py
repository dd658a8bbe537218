"""The reduced-precision endgame (round 5; nr_set_endgame, k_trace's EG instances):
a bf16 / fp16 ray whose 16-bit MLP output falls below tau re-evaluates that point in fp32x3 and
takes every later step of its march in fp32x3 (the per-point rule of the fp32x3 normals: the split
within the x3 pack's input bounds, the fp32 MLP outside), so the convergence test
(volumeRender_kernel.cu:474 `tstep < 1e-6`), the background test and the hit point are decided at
fp32-class precision while the bulk stays 16-bit.

Contract: BIT-EXACT against the oracle's restatement (oracle/nr_oracle.c or_set_endgame: the same
switch rule over the bit-exact bf16 / fp16 / fp32x3 arithmetic) -- every pixel, the ray-step count
(every march evaluation, the switch iteration's two included) and the number of fp32x3
evaluations -- over geometries, cameras, both 16-bit precisions, thresholds, scenes, step caps,
ragged sizes, batches and a 4-input network with frames on both sides of the x3 pack's frame
bound.  The quality it buys against the exact-MLP frame is asserted in test_gpu_lowp_contract.py."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle

pytestmark = pytest.mark.gpu
PREC = {"bf16": 1, "fp16": 2}


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def _oracle(geom_or_net, K=None, B=None):
    if K is None:
        dims, K, B = nr.read_keras_h5(nr.geometry_path(geom_or_net))
    else:
        dims = geom_or_net
    pack = nr.pack_x3(dims, K, B)
    assert pack[2], "the network's x3 pack must be valid for the endgame"
    return oracle.OracleNet(K, B, x3_pack=pack[:2])


def _check(img, st, ref, rst):
    assert (ref != 0).any()
    assert np.array_equal(img, ref), int((img != ref).sum())
    assert st["ray_steps"] == rst["ray_steps"], (st, rst)
    assert st["endgame_evals"] == rst["endgame_evals"] > 0, (st, rst)
    # the rays handed off (round 6): each one's switch point is counted twice in ray_steps
    assert st["endgame_switches"] == rst["endgame_switches"] > 0, (st, rst)
    assert st["endgame_switches"] <= st["endgame_evals"]
    assert st["rays_shaded"] == rst["rays_shaded"], (st, rst)


@pytest.mark.parametrize("geom,prec", [("plane_1", "bf16"), ("car_1", "bf16"), ("plane_3", "fp16"), ("plane_2", "fp16")])
@pytest.mark.parametrize("tau", [nr.NR_ENDGAME_DEFAULT, 0.02])
def test_endgame_frames_bitexact(chrome, geom, prec, tau):
    net = _oracle(geom)
    for cam in ((0.0, 0.0, 2.0), (25.0, 140.0, 2.6)):
        iv, nm = nr.camera(*cam)
        with nr.Renderer(0) as r:
            r.load_h5(nr.geometry_path(geom)).set_precision(prec).set_endgame(tau)
            r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
            img, st = r.render(160, 144, 128)
        ref, rst = net.render(160, 144, iv, nm, color_type=1, matcap=chrome, max_steps=128, nthreads=16,
                              precision=PREC[prec], endgame=tau)
        _check(img, st, ref, rst)


def test_endgame_default_on_and_off(chrome):
    """nr_set_endgame(0) is the pure 16-bit march (the round-4 contract); the default threshold
    is NR_ENDGAME_DEFAULT."""
    net = _oracle("car_1")
    iv, nm = nr.camera(10.0, 30.0, 2.2)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("car_1")).set_precision("bf16")
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        dflt, sd = r.render(128, 128, 96)
        r.set_endgame(0)
        pure, sp = r.render(128, 128, 96)
    kw = dict(color_type=1, matcap=chrome, max_steps=96, nthreads=16, precision=1)
    ref_eg, _ = net.render(128, 128, iv, nm, endgame=nr.NR_ENDGAME_DEFAULT, **kw)
    ref_pure, rp = net.render(128, 128, iv, nm, **kw)
    assert np.array_equal(dflt, ref_eg) and sd["endgame_evals"] > 0
    assert np.array_equal(pure, ref_pure) and sp["endgame_evals"] == 0 and sp["ray_steps"] == rp["ray_steps"]
    assert sp["endgame_switches"] == 0 and sd["endgame_switches"] > 0
    assert not np.array_equal(dflt, pure)


@pytest.mark.parametrize("scene", ["tanh", "subtract", "displace"])
def test_endgame_scenes(chrome, scene):
    net = _oracle("plane_1")
    iv, nm = nr.camera(-15.0, 60.0, 2.0)
    sid = nr.NR_SCENE[scene]
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision("bf16")
        r.set_view(iv, nm, 3).set_static(nr.NR_COLOR_FACING, 3).set_scene(scene)
        img, st = r.render(128, 112, 128)
    ref, rst = net.render(128, 112, iv, nm, frame=3, color_type=0, scene=sid, max_steps=128, nthreads=16,
                          precision=1, endgame=nr.NR_ENDGAME_DEFAULT)
    _check(img, st, ref, rst)


@pytest.mark.parametrize("W,H,steps", [(1, 1, 64), (7, 301, 128), (96, 96, 1), (96, 96, 5), (96, 96, 0)])
def test_endgame_sizes_and_caps(chrome, W, H, steps):
    net = _oracle("car_1")
    iv, nm = nr.camera(0.0, 0.0, 2.0) if W > 1 else nr.camera(0.0, 0.0, 0.01)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("car_1")).set_precision("fp16")
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(W, H, steps)
    ref, rst = net.render(W, H, iv, nm, color_type=1, matcap=chrome, max_steps=steps, nthreads=16, precision=2,
                          endgame=nr.NR_ENDGAME_DEFAULT)
    assert np.array_equal(img, ref), int((img != ref).sum())
    assert st["ray_steps"] == rst["ray_steps"] and st["endgame_evals"] == rst.get("endgame_evals", 0)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_endgame_batch_equals_single_frames(chrome, prec):
    """A batch (every frame's rays share the waves and their fine queues) equals the single-frame
    renders and the oracle, frame by frame."""
    net = _oracle("plane_2")
    cams = [nr.camera(7.0 * i, 41.0 * i, 2.0 + 0.1 * i) + (i,) for i in range(5)]
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_2")).set_precision(prec)
        r.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        imgs, bst = r.render_batch(144, 128, cams, 128)
        singles = []
        for iv, nm, f in cams:
            r.set_view(iv, nm, f)
            singles.append(r.render(144, 128, 128))
    tot_steps = tot_eg = tot_sw = 0
    for (iv, nm, f), img, (one, st) in zip(cams, imgs, singles):
        ref, rst = net.render(144, 128, iv, nm, frame=f, color_type=1, matcap=chrome, max_steps=128, nthreads=16,
                              precision=PREC[prec], endgame=nr.NR_ENDGAME_DEFAULT)
        assert np.array_equal(img, ref) and np.array_equal(one, ref), (f, int((img != ref).sum()))
        assert st["ray_steps"] == rst["ray_steps"] and st["endgame_evals"] == rst["endgame_evals"]
        assert st["endgame_switches"] == rst["endgame_switches"]
        tot_steps += rst["ray_steps"]
        tot_eg += rst["endgame_evals"]
        tot_sw += rst["endgame_switches"]
    assert bst["ray_steps"] == tot_steps and bst["endgame_evals"] == tot_eg and bst["endgame_switches"] == tot_sw


def test_endgame_four_input_network_frame_bound():
    """A 4-input network (the frame as 4th input): frames within the x3 pack's frame bound finish
    in the split, frames beyond it (1500) in the fp32 MLP -- per point, in a batch too."""
    rng = np.random.default_rng(31)
    dims = [4] + [32] * 8 + [1]
    K = [rng.normal(0, 0.3, size=(dims[i], dims[i + 1])).astype(np.float32) for i in range(len(dims) - 1)]
    K[0][3] *= 0.0005
    B = [rng.normal(0, 0.05, size=dims[i + 1]).astype(np.float32) for i in range(len(dims) - 1)]
    B[-1][0] = 0.2
    net = _oracle(dims, K, B)
    iv, nm = nr.camera(0.0, 20.0, 2.0)
    frames = [3, 1500, 1024, 7]
    with nr.Renderer(0) as r:
        r.load_mlp(dims, K, B).set_precision("bf16").set_endgame(0.01)
        r.set_static(nr.NR_COLOR_FACING, 4).set_scene("v1")
        imgs, _ = r.render_batch(96, 80, [(iv, nm, f) for f in frames], 96)
    for f, img in zip(frames, imgs):
        ref, _ = net.render(96, 80, iv, nm, frame=f, color_type=0, num_inputs=4, max_steps=96, nthreads=16,
                            precision=1, endgame=0.01)
        assert np.array_equal(img, ref), (f, int((img != ref).sum()))
    assert any((i != 0).any() for i in imgs)


@pytest.mark.parametrize("extra", [2, 5])
def test_endgame_deep_networks(chrome, extra):
    """Deeper fused networks (plane_1 with `extra` identity hidden layers inserted: 9 and 12 hidden
    layers, the same function): the endgame's 12-wave workgroups hold both packs in LDS only up to
    ~9 hidden layers; deeper networks take the 4-wave instances that read the fp32x3 pack from
    global memory (nr_trace.hip launch_trace_k).  Both bit-exact with the oracle's restatement."""
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    K, B = list(K), list(B)
    for _ in range(extra):
        K.insert(4, np.eye(32, dtype=np.float32))
        B.insert(4, np.zeros(32, dtype=np.float32))
    dims = [3] + [32] * (len(K) - 1) + [1]
    net = _oracle(dims, K, B)
    iv, nm = nr.camera(-15.0, 30.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_mlp(dims, K, B).set_precision("bf16")
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(112, 96, 96)
        # a batch of the same frame twice (the batched instance of the same form)
        imgs, bst = r.render_batch(112, 96, [(iv, nm, 0)] * 2, 96)
    ref, rst = net.render(112, 96, iv, nm, color_type=1, matcap=chrome, max_steps=96, nthreads=16, precision=1,
                          endgame=nr.NR_ENDGAME_DEFAULT)
    _check(img, st, ref, rst)
    assert all(np.array_equal(x, ref) for x in imgs) and bst["endgame_evals"] == 2 * rst["endgame_evals"]


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("tau", [0.0, nr.NR_ENDGAME_DEFAULT])
def test_sixteen_ray_waves_bitexact(chrome, prec, tau):
    """Waves capped at 16 rays (nr_set_wave_rays 16: every march MLP on one 32-point tile with points
    16-31 idle, the shape of a launch's tail) bit-exact with the oracle's restatement, pure march and
    endgame.  (Round 6 ran these waves on one 16-point tile of v_mfma_f32_16x16x32, bit-exact, and
    removed that form again: profiles/r6_s16_tail_mlp.txt.)"""
    net = _oracle("car_1")
    iv, nm = nr.camera(-12.0, 40.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("car_1")).set_precision(prec).set_endgame(tau).set_wave_rays(16)
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(120, 104, 128)
    ref, rst = net.render(120, 104, iv, nm, color_type=1, matcap=chrome, max_steps=128, nthreads=16,
                          precision=PREC[prec], endgame=tau)
    assert (ref != 0).any()
    assert np.array_equal(img, ref), int((img != ref).sum())
    assert st["ray_steps"] == rst["ray_steps"] and st["endgame_evals"] == rst.get("endgame_evals", 0)


def test_endgame_off_for_fp32_normals(chrome):
    """Bit 15 (fp32 normals) marches in pure 16-bit (no fp32x3 pass), on both schedules."""
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision("bf16")
        iv, nm = nr.camera(0.0, 0.0, 2.0)
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        r.set_debug(1 << 15)
        _, st = r.render(96, 96, 64)
        assert st["endgame_evals"] == 0
        r.set_schedule("wavefront")
        _, st = r.render(96, 96, 64)
        assert st["endgame_evals"] == 0


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_endgame_wavefront_equals_persistent(chrome, prec):
    """Round 6: the wavefront schedule's endgame (a fine queue per iteration, k_march16 modes 1 / 2)
    gives the persistent tracer's frames, ray-step, fp32x3-evaluation and switch counts -- single
    frames and a batch, against the oracle too."""
    net = _oracle("car_1")
    cams = [nr.camera(5.0 * i - 10.0, 37.0 * i + 20.0, 2.2) + (i,) for i in range(3)]
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("car_1")).set_precision(prec)
        r.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        pers = []
        for iv, nm, f in cams:
            r.set_view(iv, nm, f)
            pers.append(r.render(136, 120, 128))
        pb, pbs = r.render_batch(136, 120, cams, 128)
        r.set_schedule("wavefront")
        wave = []
        for iv, nm, f in cams:
            r.set_view(iv, nm, f)
            wave.append(r.render(136, 120, 128))
        wb, wbs = r.render_batch(136, 120, cams, 128)
    for (iv, nm, f), (a, sa), (b, sb), c, d in zip(cams, pers, wave, pb, wb):
        ref, rst = net.render(136, 120, iv, nm, frame=f, color_type=1, matcap=chrome, max_steps=128, nthreads=16,
                              precision=PREC[prec], endgame=nr.NR_ENDGAME_DEFAULT)
        assert np.array_equal(b, ref) and np.array_equal(a, ref) and np.array_equal(d, ref) and np.array_equal(c, ref)
        for k in ("ray_steps", "endgame_evals", "endgame_switches", "rays_shaded"):
            assert sa[k] == sb[k] == rst[k], (k, sa[k], sb[k], rst[k])
    for k in ("ray_steps", "endgame_evals", "endgame_switches"):
        assert pbs[k] == wbs[k] > 0, (k, pbs[k], wbs[k])


def test_endgame_rejects_bad_threshold():
    with nr.Renderer(0) as r:
        for bad in (-1.0, float("nan"), float("inf")):
            with pytest.raises(nr.NRError):
                r.set_endgame(bad)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_schedule_pixel_contract(chrome, prec):
    """The documented per-schedule rule for 16-bit frames (neural_render.h, nr_set_schedule): at
    default settings persistent = wavefront = the endgame frame, with nr_set_endgame(0) both = the
    pure 16-bit march, layered = the fp32 frame; each against the oracle."""
    net = _oracle("plane_1")
    iv, nm = nr.camera(-12.0, 35.0, 2.1)
    kw = dict(color_type=1, matcap=chrome, max_steps=128, nthreads=16)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision(prec)
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        pers, _ = r.render(128, 120, 128)
        r.set_schedule("wavefront")
        wave, _ = r.render(128, 120, 128)
        r.set_schedule("layered")
        lay, _ = r.render(128, 120, 128)
        r.set_schedule("persistent").set_endgame(0)
        pure, _ = r.render(128, 120, 128)
        r.set_schedule("wavefront")
        wpure, _ = r.render(128, 120, 128)
    ref_eg, _ = net.render(128, 120, iv, nm, precision=PREC[prec], endgame=nr.NR_ENDGAME_DEFAULT, **kw)
    ref_pure, _ = net.render(128, 120, iv, nm, precision=PREC[prec], **kw)
    ref_f32, _ = net.render(128, 120, iv, nm, precision=0, **kw)
    assert np.array_equal(pers, ref_eg) and np.array_equal(wave, ref_eg)
    assert np.array_equal(pure, ref_pure) and np.array_equal(wpure, ref_pure)
    assert np.array_equal(lay, ref_f32)
