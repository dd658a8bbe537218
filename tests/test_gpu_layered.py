"""GPU parity of the layered schedule (NR_SCHED_LAYERED): networks of any dense shape.

The reference renders whatever layer list NeuralNetwork::load builds
(neuralNetwork.cpp:85-151, one CUTLASS GEMM per layer per iteration,
denseLayer.cu:229-278).  libnr takes [3|4, 32, ..., 32, 1] on its fused kernels and
every other shape on the layered schedule; both are fp32 bit-exact against the oracle,
whose MLP is shape-generic (oracle/nr_oracle.c mlp_point).

Two kinds of network are used:
  * exact re-shapes of a bundled geometry (zero-padded hidden units, inserted identity
    layers): the ascending-k fmaf chain gives bit-identical SDFs, so the frame must equal
    the fused kernels' frame of the original network as well as the oracle's;
  * seeded random networks (no bundled model has another shape): parity with the
    oracle on the same weights ("parity unpinned" against the reference itself, which
    cannot run here -- SURVEY.md 8c).
"""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle

pytestmark = pytest.mark.gpu
PURE_16BIT = True  # the pure 16-bit march (conftest.py pure_16bit)

STATS = ("ray_steps", "shade_evals", "rays_hit", "rays_shaded", "iterations")


@pytest.fixture(scope="module")
def rend():
    r = nr.Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def widen(K, B, w):
    """Zero-pad every hidden layer to width w (same function, same fmaf chains)."""
    K2, B2 = [], []
    n = len(K)
    for l, (k, b) in enumerate(zip(K, B)):
        i, o = k.shape
        ii = i if l == 0 else w
        oo = o if l == n - 1 else w
        kk = np.zeros((ii, oo), np.float32)
        kk[:i, :o] = k
        bb = np.zeros(oo, np.float32)
        bb[:o] = b
        K2.append(kk)
        B2.append(bb)
    return K2, B2


def insert_identity(K, B, after, w):
    """Insert 32 -> w -> 32 identity layers (ReLU of non-negative inputs is exact)."""
    up = np.zeros((32, w), np.float32)
    up[np.arange(32), np.arange(32)] = 1.0
    down = np.zeros((w, 32), np.float32)
    down[np.arange(32), np.arange(32)] = 1.0
    K2 = K[:after + 1] + [up, down] + K[after + 1:]
    B2 = B[:after + 1] + [np.zeros(w, np.float32), np.zeros(32, np.float32)] + B[after + 1:]
    return K2, B2


def random_net(dims, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    K = [(rng.standard_normal((i, o)) * scale / np.sqrt(i)).astype(np.float32) for i, o in zip(dims[:-1], dims[1:])]
    B = [(rng.standard_normal(o) * 0.1).astype(np.float32) for o in dims[1:]]
    return K, B


def load(rend, K, B):
    dims = [K[0].shape[0]] + [k.shape[1] for k in K]
    rend.load_mlp(dims, K, B)
    return dims


def render_both(rend, K, B, W, H, steps, cam=(0.0, 0.0, 2.0), frame=0, color=1, scene="v1", ninputs=3,
                matcap=None):
    iv, nm = nr.camera(*cam)
    rend.set_view(iv, nm, frame).set_static(color, ninputs).set_scene(scene)
    if matcap is not None:
        rend.set_matcap(matcap)
    img, st = rend.render(W, H, steps)
    ref, rst = oracle.OracleNet(K, B).render(W, H, iv, nm, frame=frame, color_type=color, num_inputs=ninputs,
                                             scene=nr.NR_SCENE[scene], matcap=matcap if color else None,
                                             max_steps=steps)
    return img, st, ref, rst


def assert_same(img, st, ref, rst):
    d = img != ref
    assert not d.any(), f"{d.sum()} pixels differ; gpu {st} oracle {rst}"
    for k in STATS:
        assert st[k] == rst[k], (k, st, rst)


@pytest.mark.parametrize("how", ["widen48", "widen40", "identity64"])
def test_reshaped_plane_matches_fused_and_oracle(rend, nets, chrome, how):
    dims, K, B = nets["plane_1"]
    rend.set_precision("fp32").set_schedule("persistent")
    if how == "widen48":
        K2, B2 = widen(K, B, 48)
    elif how == "widen40":
        K2, B2 = widen(K, B, 40)
    else:
        K2, B2 = insert_identity(K, B, 3, 64)
    # the original network on the fused kernels
    rend.load_mlp(dims, K, B)
    iv, nm = nr.camera(-18.3, 150.7, 2.25)
    rend.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    fused, sf = rend.render(96, 80, 128)
    # the reshaped network: not a fused shape, so layered whatever the schedule says
    load(rend, K2, B2)
    img, st, ref, rst = render_both(rend, K2, B2, 96, 80, 128, cam=(-18.3, 150.7, 2.25), matcap=chrome)
    assert_same(img, st, ref, rst)
    assert np.array_equal(img, fused)
    for k in STATS:
        assert st[k] == sf[k], (k, st, sf)


@pytest.mark.parametrize("dims,seed,scene,color", [
    ([3, 16, 16, 1], 1, "v1", 0),
    ([3, 16, 16, 1], 2, "tanh", 1),
    ([3, 64, 48, 24, 1], 3, "tanh", 1),
    ([3, 1], 4, "v1", 0),
    ([3, 128, 128, 128, 1], 5, "tanh", 0),
    ([3, 20, 17, 30, 1], 6, "v1", 1),
])
def test_random_networks_vs_oracle(rend, chrome, dims, seed, scene, color):
    K, B = random_net(dims, seed)
    load(rend, K, B)
    img, st, ref, rst = render_both(rend, K, B, 72, 56, 96, cam=(-20.0, 35.0, 2.0), color=color, scene=scene,
                                    matcap=chrome)
    assert_same(img, st, ref, rst)
    assert st["ray_steps"] > 0


def test_animation_network_four_inputs(rend, chrome):
    """numInputs = 4 (main.cpp:619-621): the frame number is the 4th network input."""
    K, B = random_net([4, 24, 24, 1], 11)
    load(rend, K, B)
    for frame in (0, 45, 300):
        img, st, ref, rst = render_both(rend, K, B, 64, 48, 96, cam=(10.0, 60.0, 2.0), frame=frame, ninputs=4,
                                        matcap=chrome, scene="tanh")
        assert_same(img, st, ref, rst)


@pytest.mark.parametrize("schedule", ["persistent", "wavefront"])
@pytest.mark.parametrize("scene", ["v1", "tanh"])
def test_fused_four_input_network(rend, chrome, schedule, scene):
    """A [4, 32 x 8, 1] network (numInputs = 4, main.cpp:619-621; the frame number is the 4th
    input, kernel.cu:524-545) takes the FUSED march kernels (k_trace's and k_march16's
    4-input layer 0): single frames and one nr_render_batch of three frames equal the
    oracle frame by frame (seeded random weights: parity unpinned against the reference)."""
    K, B = random_net([4] + [32] * 8 + [1], 41, scale=1.4)
    load(rend, K, B)  # [4, 32, ..., 32, 1]: a fused shape (nr_pack.cpp fused_shape_ok)
    rend.set_schedule(schedule)
    try:
        iv, nm = nr.camera(-12.0, 70.0, 2.0)
        rend.set_static(nr.NR_COLOR_MATCAP, 4).set_scene(scene).set_matcap(chrome)
        refs = []
        for frame in (0, 45, 300):
            rend.set_view(iv, nm, frame)
            img, st = rend.render(72, 56, 96)
            ref, rst = oracle.OracleNet(K, B).render(72, 56, iv, nm, frame=frame, color_type=1, num_inputs=4,
                                                     scene=nr.NR_SCENE[scene], matcap=chrome, max_steps=96)
            assert_same(img, st, ref, rst)
            assert rst["rays_hit"] > 0
            refs.append((ref, rst))
        imgs, bst = rend.render_batch(72, 56, [(iv, nm, f) for f in (0, 45, 300)], 96)
        for img, (ref, rst) in zip(imgs, refs):
            assert np.array_equal(img, ref)
        assert bst["ray_steps"] == sum(r[1]["ray_steps"] for r in refs)
    finally:
        rend.set_schedule("persistent").set_static(nr.NR_COLOR_MATCAP, 3)


@pytest.mark.parametrize("chunk", [64, 1000, 4096])
def test_layer_chunks(rend, chrome, chunk):
    """Bounded layer scratch: the same frame in chunks of 64 / 1000 / 4096 points."""
    K, B = random_net([3, 96, 96, 1], 21)
    load(rend, K, B)
    rend.set_layer_chunk(chunk)
    try:
        img, st, ref, rst = render_both(rend, K, B, 50, 45, 64, cam=(5.0, 200.0, 2.0), matcap=chrome)
    finally:
        rend.set_layer_chunk(0)
    assert_same(img, st, ref, rst)


def test_graph_replay_across_frames(rend, nets, chrome):
    """The captured graph is reused for a new camera / frame number / output: each frame
    still equals the oracle (per-frame arguments live in device memory)."""
    dims, K, B = nets["car_1"]
    K2, B2 = widen(K, B, 36)
    load(rend, K2, B2)
    rng = np.random.default_rng(5)
    for i in range(3):
        cam = (float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0)
        fr = int(rng.integers(0, 360))
        img, st, ref, rst = render_both(rend, K2, B2, 64, 64, 128, cam=cam, frame=fr, matcap=chrome)
        assert_same(img, st, ref, rst)


def test_long_cap_direct_launches(rend, chrome):
    """max_steps > 1024 is issued launch by launch instead of as a graph."""
    K, B = random_net([3, 20, 1], 8)
    load(rend, K, B)
    img, st, ref, rst = render_both(rend, K, B, 24, 20, 1500, cam=(0.0, 0.0, 2.0), color=0)
    assert_same(img, st, ref, rst)


def test_layered_shards_and_batch(rend, nets, chrome):
    dims, K, B = nets["plane_1"]
    K2, B2 = widen(K, B, 33)
    load(rend, K2, B2)
    iv, nm = nr.camera(-10.0, 20.0, 2.0)
    rend.set_view(iv, nm, 0).set_static(1, 3).set_scene("v1").set_matcap(chrome)
    W, H = 70, 83
    full, _ = rend.render(W, H, 128)
    shards = [rend.render_shard(W, H, 8, 3, s, 128)[0] for s in range(3)]
    assert np.array_equal(nr.assemble_shards(shards, W, H, 8, 3), full)
    cams = [(iv, nm, 0), (*nr.camera(15.0, 100.0, 2.0), 30)]
    imgs, _ = rend.render_batch(W, H, cams, 128)
    assert np.array_equal(imgs[0], full)
    ref, _ = oracle.OracleNet(K2, B2).render(W, H, cams[1][0], cams[1][1], frame=30, color_type=1, matcap=chrome,
                                             max_steps=128)
    assert np.array_equal(imgs[1], ref)


@pytest.mark.parametrize("dims,n", [([3, 1024, 1], 40000), ([3, 48, 48, 48, 2], 5000), ([4, 7, 1], 1),
                                    ([3, 70, 33, 130, 17, 1], 3001), ([5, 64, 64, 3], 999)])
def test_generic_mlp_forward_chunked(rend, dims, n):
    K, B = random_net(dims, 31)
    load(rend, K, B)
    X = np.random.default_rng(2).uniform(-1, 1, size=(n, dims[0])).astype(np.float32)
    assert np.array_equal(rend.mlp_forward(X), oracle.OracleNet(K, B).forward(X))


def test_two_output_network_refused(rend):
    K, B = random_net([3, 8, 2], 1)
    load(rend, K, B)
    rend.set_static(0, 3)
    with pytest.raises(RuntimeError, match="one output"):
        rend.render(8, 8, 10)


def test_direct_launches_equal_graph(rend, nets, chrome):
    """Debug bit 8 (launch by launch, no hipGraph) renders the same frame."""
    dims, K, B = nets["plane_3"]
    K2, B2 = widen(K, B, 44)
    load(rend, K2, B2)
    iv, nm = nr.camera(12.0, 250.0, 2.0)
    rend.set_view(iv, nm, 5).set_static(1, 3).set_scene("tanh").set_matcap(chrome)
    a, sa = rend.render(90, 70, 128)
    rend.set_debug(256)
    try:
        b, sb = rend.render(90, 70, 128)
    finally:
        rend.set_debug(0)
    assert np.array_equal(a, b)
    for k in STATS:
        assert sa[k] == sb[k], (k, sa, sb)
