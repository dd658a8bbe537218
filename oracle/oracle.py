"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  See nr_oracle.c for what it
restates and how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# OR_LIBRARY: another build of the same source (tools/contract_drift.py: -ffp-contract=fast)
SO = os.environ.get("OR_LIBRARY") or os.path.join(HERE, "_build", "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = ctypes.CDLL(SO)
        P = ctypes.c_void_p
        I = ctypes.c_int
        L.or_mlp_forward.restype = I
        L.or_mlp_forward.argtypes = [I, P, P, P, ctypes.c_long, I, P, I, I]
        L.or_render.restype = I
        L.or_render.argtypes = [I, P, P, P, P, I, I, I, I, P, I, I, I, I, I, P, P, I]
        L.or_render_ex.restype = I
        L.or_render_ex.argtypes = [I, P, P, P, P, I, I, I, I, P, I, I, I, I, I, P, P, I, I, I, I]
        L.or_scene_sdf.restype = ctypes.c_float
        L.or_scene_sdf.argtypes = [ctypes.c_float] * 4 + [I, I]
        L.nr_tanh_f.restype = ctypes.c_float
        L.nr_tanh_f.argtypes = [ctypes.c_float]
        L.or_batch_smooth_union.restype = None
        L.or_batch_smooth_union.argtypes = [P, P, ctypes.c_long, ctypes.c_float, P, P]
        L.or_batch_many_sphere.restype = None
        L.or_batch_many_sphere.argtypes = [P, P, ctypes.c_long, I, P, P]
        L.nr_sin_f.restype = ctypes.c_float
        L.nr_sin_f.argtypes = [ctypes.c_float]
        L.or_batch_smooth_sub.restype = None
        L.or_batch_smooth_sub.argtypes = [P, P, ctypes.c_long, ctypes.c_float, P, P]
        L.or_batch_cylinders.restype = None
        L.or_batch_cylinders.argtypes = [P, P, ctypes.c_long, P, P]
        L.or_batch_intersect.restype = None
        L.or_batch_intersect.argtypes = [P, P, ctypes.c_long, ctypes.c_float, P, P]
        L.or_set_x3_pack.restype = None
        L.or_set_x3_pack.argtypes = [P, P, I, I]
        L.or_set_mfma_model.restype = None
        L.or_set_mfma_model.argtypes = [I, I]
        L.or_set_dot2_model.restype = None
        L.or_set_dot2_model.argtypes = [I]
        L.or_mfma_sum.restype = ctypes.c_float
        L.or_mfma_sum.argtypes = [ctypes.c_float, P, P, I, I]
        L.or_trace_mfma.restype = None
        L.or_trace_mfma.argtypes = [P, ctypes.c_long]
        L.or_trace_count.restype = ctypes.c_long
        L.or_trace_count.argtypes = []
        L.or_set_endgame.restype = None
        L.or_set_endgame.argtypes = [ctypes.c_float]
        L.or_endgame_evals.restype = ctypes.c_longlong
        L.or_endgame_evals.argtypes = []
        L.or_endgame_switches.restype = ctypes.c_longlong
        L.or_endgame_switches.argtypes = []
        _lib = L
    return _lib


def pack_params(kernels, biases):
    """Keras kernels (in, out) -> the oracle's out-major W[out][in] + bias per layer
    (DenseLayer::initializeWeights, denseLayer.cu:217-227)."""
    parts = []
    dims = [kernels[0].shape[0]]
    for K, b in zip(kernels, biases):
        K = np.asarray(K, np.float32)
        parts.append(np.ascontiguousarray(K.T).reshape(-1))
        parts.append(np.asarray(b, np.float32).reshape(-1))
        dims.append(K.shape[1])
    return np.array(dims, np.int32), np.concatenate(parts).astype(np.float32)


class OracleNet:
    def __init__(self, kernels, biases, x3_pack=None):
        """x3_pack = (a_ops uint16, floats float32) from the library's nr_pack_x3 (the fp32x3 pack):
        precision 4 evaluates with the fp32x3 emulation (nr_oracle.c mlp_point_gpu_x3), and
        precision-1/2 renders take their normals from it, as the bf16/fp16 tracers do.  None: fp32
        normals."""
        self.dims, self.params = pack_params(kernels, biases)
        self.nlayers = len(kernels)
        self.x3 = None
        if x3_pack is not None:
            self.x3 = (np.ascontiguousarray(x3_pack[0], np.uint16), np.ascontiguousarray(x3_pack[1], np.float32))

    def _x3_on(self):
        if self.x3 is None:
            lib().or_set_x3_pack(None, None, 0, 0)
        else:
            lib().or_set_x3_pack(self.x3[0].ctypes.data, self.x3[1].ctypes.data, self.nlayers - 2, int(self.dims[0]))

    def forward(self, X, precision=0, nthreads=0):
        X = np.ascontiguousarray(X, np.float32)
        n = X.shape[0]
        Y = np.zeros((n, int(self.dims[-1])), np.float32)
        self._x3_on()
        rc = lib().or_mlp_forward(self.nlayers, self.dims.ctypes.data, self.params.ctypes.data, X.ctypes.data, n,
                                  X.shape[1], Y.ctypes.data, precision, nthreads)
        assert rc == 0, rc
        return Y

    def render(self, W, H, inv_view, normal, frame=0, color_type=0, num_inputs=3, scene=0, matcap=None,
               max_steps=6000, nthreads=0, precision=0, rows=None, endgame=0.0):
        """precision 1/2: the GPU's bf16/fp16 MLP arithmetic (nr_oracle.c mlp_point_gpu_lowp) for
        the marching points; the normals in fp32x3 when the net holds an x3 pack (as the bf16/fp16
        tracers compute them), else fp32.  rows=(y0, y1): render only those rows of the frame.
        endgame > 0 (precision 1/2, a net with an x3 pack): a ray whose 16-bit MLP output falls below
        it is re-evaluated and marched from then on in fp32x3 (nr_oracle.c or_set_endgame); the
        stats then carry "endgame_evals", the fp32x3 march evaluations."""
        y0, y1 = rows if rows is not None else (0, H)
        out = np.zeros((y1 - y0, W), np.uint32)
        stats = np.zeros(5, np.int64)
        iv = np.ascontiguousarray(inv_view, np.float32)
        nm = np.ascontiguousarray(normal, np.float32)
        if matcap is not None:
            mc = np.ascontiguousarray(matcap, np.uint32)
            mp, mw, mh = mc.ctypes.data, mc.shape[1], mc.shape[0]
        else:
            mc, mp, mw, mh = None, None, 0, 0
        self._x3_on()
        lib().or_set_endgame(float(endgame))
        rc = lib().or_render_ex(self.nlayers, self.dims.ctypes.data, self.params.ctypes.data, iv.ctypes.data,
                                nm.ctypes.data, frame, color_type, num_inputs, scene, mp, mw, mh, W, H, max_steps,
                                out.ctypes.data, stats.ctypes.data, nthreads, precision, y0, y1)
        assert rc == 0, rc
        keys = ["ray_steps", "shade_evals", "iterations", "rays_hit", "rays_shaded"]
        st = dict(zip(keys, (int(v) for v in stats)))
        if endgame > 0:
            st["endgame_evals"] = int(lib().or_endgame_evals())
            st["endgame_switches"] = int(lib().or_endgame_switches())
        lib().or_set_endgame(0.0)
        return out, st


def set_mfma_model(model, w=26):
    """The emulations' model of one 16-bit MFMA output (nr_oracle.c mfma_sum): 0 exact sum rounded
    once, 1 two groups of 8 each rounded, 2 groups of 8 aligned and cut w bits below their
    largest product.  For fitting (tools/fit_emulation.py); process-wide."""
    lib().or_set_mfma_model(int(model), int(w))


def mfma_sum(acc, a, b, emin, fast=1):
    """One v_mfma_f32_32x32x16_{f16,bf16} output as the restatement computes it (nr_oracle.c
    mfma_sum / mfma_fast): acc + sum a[k] b[k], k = 0..15, 16-bit operand values as floats;
    emin -14 (fp16) or -126 (bf16)."""
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return float(lib().or_mfma_sum(float(acc), a.ctypes.data, b.ctypes.data, int(emin), int(fast)))


def scene_sdf(p, nsdf, scene=0, frame=0):
    return lib().or_scene_sdf(float(p[0]), float(p[1]), float(p[2]), float(nsdf), scene, frame)


def tanh_f(x):
    return lib().nr_tanh_f(float(x))


def sin_f(x):
    return lib().nr_sin_f(float(x))


def smooth_sub_pair(d1, d2, k=0.01):
    """(reference form, kernel form) of sdfOpSmoothSubtraction over arrays (bitwise comparable)."""
    d1 = np.ascontiguousarray(d1, np.float32)
    d2 = np.ascontiguousarray(d2, np.float32)
    ref, ker = np.empty_like(d1), np.empty_like(d1)
    lib().or_batch_smooth_sub(d1.ctypes.data, d2.ctypes.data, d1.size, k, ref.ctypes.data, ker.ctypes.data)
    return ref, ker


def cylinders_pair(p, nsdf):
    """(reference form, kernel form) of manyCylinderCut over points (bitwise comparable)."""
    p = np.ascontiguousarray(p, np.float32)
    nsdf = np.ascontiguousarray(nsdf, np.float32)
    ref, ker = np.empty_like(nsdf), np.empty_like(nsdf)
    lib().or_batch_cylinders(p.ctypes.data, nsdf.ctypes.data, nsdf.size, ref.ctypes.data, ker.ctypes.data)
    return ref, ker


def smooth_union_pair(d1, d2, k=0.01):
    """(reference form, kernel form) of sdfOpSmoothUnion over arrays (bitwise comparable)."""
    d1 = np.ascontiguousarray(d1, np.float32)
    d2 = np.ascontiguousarray(d2, np.float32)
    ref = np.zeros_like(d1)
    ker = np.zeros_like(d1)
    lib().or_batch_smooth_union(d1.ctypes.data, d2.ctypes.data, d1.size, k, ref.ctypes.data, ker.ctypes.data)
    return ref, ker


def many_sphere_pair(p, nsdf, frame=0):
    p = np.ascontiguousarray(p, np.float32)
    nsdf = np.ascontiguousarray(nsdf, np.float32)
    ref = np.zeros_like(nsdf)
    ker = np.zeros_like(nsdf)
    lib().or_batch_many_sphere(p.ctypes.data, nsdf.ctypes.data, nsdf.size, frame, ref.ctypes.data, ker.ctypes.data)
    return ref, ker


def intersect_pair(o, d, r=1.2):
    """(reference form, kernel form) of intersectSphere: [hit, tnear, tfar] per ray."""
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    ref = np.zeros_like(o)
    ker = np.zeros_like(o)
    lib().or_batch_intersect(o.ctypes.data, d.ctypes.data, o.shape[0], r, ref.ctypes.data, ker.ctypes.data)
    return ref, ker
