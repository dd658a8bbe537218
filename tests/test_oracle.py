"""CPU tests: the oracle against the reference's own artefacts, and the kernel-form
restructurings against the reference forms.

Golden fixtures (tests/golden/, made by make_golden.py from /root/reference):
  weights_h5py.npz  the five .h5 files read by h5py (independent HDF5 implementation)
  mlp_kat.npz       fp64 numpy MLP outputs (ReLU hidden, linear last layer)
  silhouettes.npz   foreground masks of the reference renders neuralGeometries/*.h5.ppm
"""
import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
from conftest import GEOMS, REF_CAMERAS


@pytest.mark.parametrize("geom", GEOMS)
def test_hdf5_reader_matches_h5py(nets, golden, geom):
    # NeuralNetwork::load (neuralNetwork.cpp:85-151): groups in HDF5 name order
    dims, K, B = nets[geom]
    w = golden["weights"]
    order = [str(x) for x in w[f"{geom}/__order__"]]
    assert order == sorted(order)
    assert len(K) == len(order) == 9
    assert dims == [3] + [32] * 8 + [1]
    for i, name in enumerate(order):
        assert np.array_equal(K[i], w[f"{geom}/{name}/kernel:0"]), name
        assert np.array_equal(B[i], w[f"{geom}/{name}/bias:0"]), name
    assert sum(k.size for k in K) + sum(b.size for b in B) == 7553


@pytest.mark.parametrize("geom", GEOMS)
def test_oracle_mlp_vs_fp64(nets, golden, geom):
    dims, K, B = nets[geom]
    X = golden["kat"]["X"]
    y = oracle.OracleNet(K, B).forward(X)[:, 0].astype(np.float64)
    ref = golden["kat"][geom]
    # fp32 fmaf chains over K <= 32: |err| is a few ulp of the partial-sum magnitudes
    assert np.abs(y - ref).max() < 5e-6
    # the simpleInfer points (simpleInfer.cpp:81-126) are the last two rows
    assert np.abs(y[-2:] - ref[-2:]).max() < 5e-6


def test_oracle_batch_consistency(nets):
    # simpleInfer batchTest (simpleInfer.cpp:112-147): identical inputs -> identical outputs
    dims, K, B = nets["plane_1"]
    Y = oracle.OracleNet(K, B).forward(np.zeros((50000, 3), np.float32), nthreads=4)
    assert (Y == Y[0]).all()


def test_oracle_lowp_close(nets, golden):
    dims, K, B = nets["plane_1"]
    X = golden["kat"]["X"]
    net = oracle.OracleNet(K, B)
    ref = golden["kat"]["plane_1"]
    for prec, tol in [(1, 0.05), (2, 0.01)]:
        assert np.abs(net.forward(X, precision=prec)[:, 0] - ref).max() < tol


def _sil(golden, name):
    s = golden["sil"]
    shape = tuple(s[f"{name}/shape"])
    return np.unpackbits(s[name])[: shape[0] * shape[1]].reshape(shape).astype(bool)


@pytest.mark.parametrize("name,res,min_iou", [("plane_1", 256, 0.999), ("car_1", 128, 0.999)])
def test_oracle_silhouette_vs_reference_render(nets, golden, name, res, min_iou):
    """The reference's own renders (neuralGeometries/<g>.h5.ppm, 1024^2) pin coverage:
    the pure-neural scene (sceneSDF -> tanh(nSDF), volumeRender_kernel.cu:229) at the
    camera recovered for them (conftest.REF_CAMERAS: 0.9993 / 0.9995 at these sizes).  Pixel (x, y) of a res^2 render is the
    same ray as pixel (x*k, y*k) of the 1024^2 golden (u = x/W*2-1 has no half-pixel
    offset), so the golden is subsampled, not resized."""
    gold = _sil(golden, name)
    k = gold.shape[0] // res
    gold = gold[::k, ::k]
    iv, nm = nr.camera(*REF_CAMERAS[name])
    dims, K, B = nets[name]
    img, st = oracle.OracleNet(K, B).render(res, res, iv, nm, color_type=0, scene=1, max_steps=6000)
    fg = img != 0
    iou = (fg & gold).sum() / (fg | gold).sum()
    assert iou >= min_iou, iou


def test_plane2_reference_render_is_black(golden):
    # plane_2.h5.ppm is all zeros, so it pins nothing
    assert int(golden["sil"]["plane_2/count"]) == 0


def test_tanh_restatement_close_to_libm():
    xs = np.concatenate([np.linspace(-12, 12, 20001), np.geomspace(1e-12, 10, 2000), -np.geomspace(1e-12, 10, 2000)])
    xs = xs.astype(np.float32)
    got = np.array([oracle.tanh_f(x) for x in xs], np.float32)
    ref = np.tanh(xs.astype(np.float64)).astype(np.float32)
    ulps = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1


def test_smooth_union_kernel_form_bit_exact():
    """nr_device.h evaluates sdfOpSmoothUnion (volumeRender_kernel.cu:144-149) without the
    f64 division when |d2-d1| >= k; bit-identical to the reference form."""
    rng = np.random.default_rng(3)
    n = 2_000_000
    d1 = rng.standard_normal(n).astype(np.float32) * rng.choice([1e-4, 1e-2, 1.0], n).astype(np.float32)
    d2 = d1 + (rng.standard_normal(n) * rng.choice([1e-3, 1e-2, 1e-1], n)).astype(np.float32)
    k = np.float32(0.01)
    edge = np.concatenate([d1[:1000] + k, d1[:1000] - k, np.nextafter(d1[:1000] + k, 0), np.zeros(4)]).astype(np.float32)
    d1 = np.concatenate([d1, d1[:1000], d1[:1000], d1[:1000], [0.0, -0.0, 0.0, -0.0]]).astype(np.float32)
    d2 = np.concatenate([d2, edge[:3000], [0.0, 0.0, -0.0, -0.0]]).astype(np.float32)
    # signed zeros, infinities, NaN and huge values on either side (the fmaf forms of the
    # saturated cases must keep the reference's signs and NaN/inf behaviour)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e38, -1e38, 1e-45, -1e-45, 0.01, -0.01], np.float32)
    a, b = np.meshgrid(sp, sp)
    d1 = np.concatenate([d1, a.ravel()]).astype(np.float32)
    d2 = np.concatenate([d2, b.ravel()]).astype(np.float32)
    ref, ker = oracle.smooth_union_pair(d1, d2, 0.01)
    same = (ref.view(np.uint32) == ker.view(np.uint32)) | (np.isnan(ref) & np.isnan(ker))
    assert same.all(), (d1[~same][:5], d2[~same][:5], ref[~same][:5], ker[~same][:5])


def test_scene_x0_f32_add_equals_f64_form():
    """nr_device.h many_sphere forms the first sphere column's x as p.x + 0.5f; the reference's
    cP.x = p.x + 0.5 (volumeRender_kernel.cu:186) promotes to f64 and stores to f32.  Equal bit
    for bit on floats of every exponent, signed zeros, subnormals, infinities and NaN."""
    rng = np.random.default_rng(21)
    bits = rng.integers(0, 2 ** 32, 4_000_000, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    near = (rng.uniform(-1, 1, 1_000_000) * 2.0 ** rng.integers(-40, 3, 1_000_000)).astype(np.float32)
    sp = np.array([0.0, -0.0, 0.5, -0.5, -0.25, 2 ** -30, -2 ** -30, 2 ** -31, 1e-45, -1e-45, np.inf, -np.inf,
                   np.nan, 16777216.0, -16777217.0, 3.4e38, -3.4e38], np.float32)
    x = np.concatenate([x, near, sp])
    with np.errstate(invalid="ignore", over="ignore"):
        ref = (x.astype(np.float64) + 0.5).astype(np.float32)
        ker = x + np.float32(0.5)
    same = (ref.view(np.uint32) == ker.view(np.uint32)) | (np.isnan(ref) & np.isnan(ker))
    assert same.all(), x[~same][:5]


def test_scene_far_screen_implies_union_test():
    """nr_device.h many_sphere skips a sphere (adds +0 to the running union s) when its squared
    distance q >= max(T, 0)^2, T = (nsdf + 0.11f) + (|nsdf| + 0.2f) 2^-16 in f32.  Sampled at and
    just above the threshold, over surface values across scales, signed zeros and the T <= 0
    edge: the reference's sdfOpSmoothUnion(s, sqrtf(q) - 0.1f, 0.01) (volumeRender_kernel.cu:
    144-149, :189) equals s + 0 for s = nsdf, s below it, and s above it by far more than a
    union's rounding (the running union never exceeds nsdf but for that)."""
    rng = np.random.default_rng(12)
    n = 400_000
    f = np.float32
    X = np.concatenate([rng.uniform(-1.5, 2.5, n), rng.uniform(-0.12, -0.10, n // 4),
                        rng.standard_normal(n // 4) * rng.choice([1e-6, 1e-3, 1e2, 1e6], n // 4),
                        [0.0, -0.0, -0.11, -0.1100001, 1e-30, -1e-30]]).astype(f)
    T = ((np.abs(X) + f(0.2)).astype(np.float64) * 2.0 ** -16 + (X + f(0.11)).astype(np.float64)).astype(f)  # fmaf
    T2 = np.where(T < 0, f(0), T).astype(f) ** 2
    qs = [T2, np.nextafter(T2, f(np.inf)), np.nextafter(np.nextafter(T2, f(np.inf)), f(np.inf)),
          (T2 * f(1.0 + 2 ** -20)).astype(f), (T2 * rng.uniform(1, 4, T2.size)).astype(f),
          np.full_like(T2, 0.0), np.full_like(T2, 1e-30)]
    for q in qs:
        far = q >= T2
        d = (np.sqrt(q) - f(0.1)).astype(f)
        for s in (X, (X - np.abs(X) * f(2 ** -10) - f(1e-4)).astype(f), (X + (np.abs(X) + f(0.01)) * f(2 ** -21)).astype(f)):
            ref, _ = oracle.smooth_union_pair(s[far], d[far], 0.01)
            want = (s[far] + f(0.0)).astype(f)
            same = ref.view(np.uint32) == want.view(np.uint32)
            assert same.all(), (X[far][~same][:5], q[far][~same][:5], s[far][~same][:5])


def test_smooth_subtraction_kernel_form_bit_exact():
    """nr_device.h evaluates sdfOpSmoothSubtraction (volumeRender_kernel.cu:137-142) without
    the f64 division when |d1+d2| >= k (h exactly 0 or 1); bit-identical to the reference
    form, signed zeros, infinities and NaN included."""
    rng = np.random.default_rng(4)
    n = 2_000_000
    d1 = rng.standard_normal(n).astype(np.float32) * rng.choice([1e-4, 1e-2, 1.0], n).astype(np.float32)
    d2 = -d1 + (rng.standard_normal(n) * rng.choice([1e-3, 1e-2, 1e-1], n)).astype(np.float32)
    k = np.float32(0.01)
    e = d1[:1000]
    edge = np.concatenate([k - e, -k - e, np.nextafter(k - e, 0), np.nextafter(-k - e, 0)]).astype(np.float32)
    d1 = np.concatenate([d1, e, e, e, e]).astype(np.float32)
    d2 = np.concatenate([d2, edge]).astype(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e38, -1e38, 1e-45, -1e-45, 0.01, -0.01, 0.005], np.float32)
    a, b = np.meshgrid(sp, sp)
    d1 = np.concatenate([d1, a.ravel()]).astype(np.float32)
    d2 = np.concatenate([d2, b.ravel()]).astype(np.float32)
    ref, ker = oracle.smooth_sub_pair(d1, d2, 0.01)
    same = (ref.view(np.uint32) == ker.view(np.uint32)) | (np.isnan(ref) & np.isnan(ker))
    assert same.all(), (d1[~same][:5], d2[~same][:5], ref[~same][:5], ker[~same][:5])


def test_many_cylinder_kernel_form_bit_exact():
    """manyCylinderCut (volumeRender_kernel.cu:157-174) walked as 15 rows x 20 columns, as the
    kernel evaluates it; points near the cylinder shells take the smooth-subtraction slow path."""
    rng = np.random.default_rng(6)
    n = 60_000
    p = rng.uniform(-1.3, 1.3, size=(n, 3)).astype(np.float32)
    # near the axes: x = -0.88 + 0.1 i + 0.02..., y = -0.38 + 0.1 j + 0.02
    i = rng.integers(0, 20, n // 2)
    j = rng.integers(0, 15, n // 2)
    ang = rng.uniform(0, 2 * np.pi, n // 2)
    rad = 0.02 + rng.normal(0, 0.01, n // 2)
    p[: n // 2, 0] = (-0.9 + 0.1 * i + 0.02 + rad * np.cos(ang)).astype(np.float32)
    p[: n // 2, 1] = (0.5 - 0.1 - 0.1 * j + 0.02 + rad * np.sin(ang)).astype(np.float32)
    nsdf = rng.normal(0, 0.3, n).astype(np.float32)
    ref, ker = oracle.cylinders_pair(p, nsdf)
    same = (ref.view(np.uint32) == ker.view(np.uint32)) | (np.isnan(ref) & np.isnan(ker))
    assert same.all(), (p[~same][:3], ref[~same][:3], ker[~same][:3])
    assert (ref != nsdf).mean() > 0.05  # the cylinders actually cut


def test_sin_restatement_close_to_libm():
    """nr_sin_f (the sin of sdfOpDisplace, :103-110, built from IEEE double operations on CPU
    and GPU alike) is within 1 ulp of the correctly rounded sin on the scene's range."""
    xs = np.concatenate([np.linspace(-8, 8, 40001), np.geomspace(1e-9, 8, 3000), -np.geomspace(1e-9, 8, 3000),
                         [0.0, -0.0]]).astype(np.float32)
    got = np.array([oracle.sin_f(x) for x in xs], np.float32)
    ref = np.sin(xs.astype(np.float64)).astype(np.float32)
    ulps = np.abs(got.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1
    assert np.isnan(oracle.sin_f(float("inf"))) and np.isnan(oracle.sin_f(float("nan")))


@pytest.mark.parametrize("frame", [0, 7, 359])
def test_many_sphere_kernel_form_bit_exact(frame):
    """manySphere (volumeRender_kernel.cu:176-196) with the sphere-grid coordinates hoisted
    out of the loop, as the kernel evaluates it."""
    rng = np.random.default_rng(frame)
    n = 400_000
    p = rng.uniform(-1.3, 1.3, size=(n, 3)).astype(np.float32)
    # concentrate some points near the sphere shells (centres x in {-0.5,-0.1,0.3}, y in
    # {0.2,-0.2,-0.6}, z = 0.7 - frame*1.4/360) so the smooth-union slow path is taken
    c = np.stack(np.meshgrid([-0.5, -0.1, 0.3], [-0.6, -0.2, 0.2], indexing="ij"), -1).reshape(-1, 2)
    sel = rng.integers(0, 9, n // 2)
    dirs = rng.standard_normal((n // 2, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    cz = 0.7 - frame * 2 * 0.7 / 360
    centre = np.stack([c[sel, 0], c[sel, 1], np.full(n // 2, cz)], -1)
    p[: n // 2] = (centre + dirs * (0.1 + rng.normal(0, 0.01, (n // 2, 1)))).astype(np.float32)
    nsdf = rng.normal(0, 0.3, n).astype(np.float32)
    ref, ker = oracle.many_sphere_pair(p, nsdf, frame)
    assert np.array_equal(ref.view(np.uint32), ker.view(np.uint32))


@pytest.mark.parametrize("frame", [0, 17])
def test_many_sphere_far_test_bit_exact(frame):
    """The kernel decides 'sphere farther than s + k' from |cP|^2 without the sqrt
    (nr_device.h many_sphere); points placed on shells of radius s + 0.1111 (+- tiny to
    +- 1e-3) around the 9 sphere centres probe that threshold."""
    rng = np.random.default_rng(5 + frame)
    n = 1_000_000
    c = np.stack(np.meshgrid([-0.5, -0.1, 0.3], [-0.6, -0.2, 0.2], indexing="ij"), -1).reshape(-1, 2)
    cz = 0.7 - frame * 2 * 0.7 / 360
    sel = rng.integers(0, 9, n)
    dirs = rng.standard_normal((n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    s = np.concatenate([rng.normal(0, 0.3, n // 2), rng.uniform(-0.2, 3, n - n // 2)]).astype(np.float32)
    s[:8] = [0.0, -0.0, -0.1111, -0.2, 999.0, 1e4, np.inf, np.nan]
    rad = np.abs(s.astype(np.float64) + 0.1111 + rng.normal(0, 1e-6, n) * rng.choice([0, 1, 1e2, 1e3], n))
    rad = np.nan_to_num(rad, nan=0.5, posinf=0.5)
    centre = np.stack([c[sel, 0], c[sel, 1], np.full(n, cz)], -1)
    p = (centre + dirs * rad[:, None]).astype(np.float32)
    ref, ker = oracle.many_sphere_pair(p, s, frame)
    assert np.array_equal(ref.view(np.uint32), ker.view(np.uint32))


def test_intersect_sphere_f32_division_bit_exact():
    """The kernels' ray generation (nr_trace.hip gen_ray, nr_kernels.hip k_init_f) takes
    each root of intersectSphere (volumeRender_kernel.cu:199-215) as one f32 division
    where the reference divides in f64 and rounds: innocuous double rounding (53 >= 2*24+2)
    makes them bit-identical.  Checked on eye rays of random cameras (the renderer's
    distribution), on random origins/directions over many magnitudes, and on edge cases."""
    rng = np.random.default_rng(11)
    n = 2_000_000
    # camera-like rays: origin at distance ~zoom, unit-ish directions through the sphere
    zoom = rng.uniform(0.5, 6.0, n)
    o = rng.standard_normal((n, 3))
    o *= (zoom / np.linalg.norm(o, axis=1))[:, None]
    d = -o / zoom[:, None] + rng.normal(0, 0.4, (n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # arbitrary magnitudes (denormal-ish to huge), unnormalised directions
    m = n // 2
    o2 = rng.standard_normal((m, 3)) * 10.0 ** rng.uniform(-20, 18, (m, 1))
    d2 = rng.standard_normal((m, 3)) * 10.0 ** rng.uniform(-20, 18, (m, 1))
    edge_o = np.array([[0, 0, 2], [0, 0, 1.2], [0, 0, 0], [1.2, 0, 0], [0, 0, -2], [1e30, 0, 0], [0, 1.2, 1e-30]])
    edge_d = np.array([[0, 0, -1], [0, 0, -1], [0, 0, 1], [0, 1, 0], [0, 0, 0], [-1, 0, 0], [0, -1e-20, 0]])
    O = np.concatenate([o, o2, edge_o]).astype(np.float32)
    D = np.concatenate([d, d2, edge_d]).astype(np.float32)
    ref, ker = oracle.intersect_pair(O, D, 1.2)
    assert ref[:, 0].sum() > n // 2  # most camera rays hit
    assert np.array_equal(ref.view(np.uint32), ker.view(np.uint32))
