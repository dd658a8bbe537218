"""CPU feasibility check ("give fp16 a cheaper ReLU than v_pk_max_i16"): the fp16
MLP with the ReLU folded into v_cvt_pk_f16_f32's clamp needs every activation scaled below 1.  Round 3
scaled by one interval pass over inputs within +-2^20 and lost coverage (fp16 subnormals).  Here the
scales come from sub-box interval bounds over xyz within +-B (the fp32x3 pack's method, nr_pack.cpp
box_tops, restated in numpy), and the oracle's fp16 restatement (precision 2) renders C5 crops with
the scaled network -- the values the GPU would compute from such a pack (the clamp equals max(., 0)
once every activation is below 1) -- against the exact-MLP frame, beside the unscaled fp16 network.
usage: python tools/fp16_clamp_explore.py [--rows 48] [--bound 4] [--margin 1]"""
import argparse
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import cudaneuralrender_amd as nr  # noqa: E402
import oracle  # noqa: E402
from conftest import GEOMS, compare_frames  # noqa: E402


def box_tops(dims, K, B, xb, m=16):
    """max over m^3 sub-boxes of |xyz| <= xb of each ReLU layer's interval top (double)."""
    g = np.linspace(-xb, xb, m + 1)
    ix = np.stack(np.meshgrid(np.arange(m), np.arange(m), np.arange(m), indexing="ij"), -1).reshape(-1, 3)
    lo = g[ix]
    hi = g[ix + 1]
    tops = []
    for l in range(len(dims) - 2):
        W = np.asarray(K[l], np.float64).reshape(dims[l], dims[l + 1])
        b = np.asarray(B[l], np.float64)
        Wp, Wn = np.maximum(W, 0), np.minimum(W, 0)
        a = b + lo @ Wp + hi @ Wn
        c = b + hi @ Wp + lo @ Wn
        lo, hi = np.maximum(a, 0), np.maximum(c, 0)
        tops.append(float(hi.max()))
    return tops


def scaled(dims, K, B, tops, margin):
    e = [int(math.ceil(math.log2(t))) + margin if t > 0 else 0 for t in tops]
    nl = len(K)
    K2, B2 = [], []
    for l in range(nl):
        sw = (e[l - 1] if l > 0 else 0) - (e[l] if l < nl - 1 else 0)
        sb = -e[l] if l < nl - 1 else 0
        K2.append((np.asarray(K[l], np.float64) * 2.0 ** sw).astype(np.float32))
        B2.append((np.asarray(B[l], np.float64) * 2.0 ** sb).astype(np.float32))
    return K2, B2, e


ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=48)
ap.add_argument("--bound", type=float, default=4.0)
ap.add_argument("--margin", type=int, default=1)
ap.add_argument("--threads", type=int, default=8)
ap.add_argument("--geoms", default=",".join(GEOMS))
a = ap.parse_args()
chrome = nr.load_png(nr.matcap_path("Chrome"))
iv, nm = nr.camera(0.0, 0.0, 2.0)
for geom in a.geoms.split(","):
    dims, K, B = nr.read_keras_h5(nr.geometry_path(geom))
    pack = nr.pack_x3(dims, K, B)
    tops = box_tops(dims, K, B, a.bound)
    K2, B2, e = scaled(dims, K, B, tops, a.margin)
    net = oracle.OracleNet(K, B, x3_pack=pack[:2])
    net2 = oracle.OracleNet(K2, B2, x3_pack=pack[:2])
    mid = 1024
    kw = dict(color_type=1, matcap=chrome, max_steps=128, nthreads=a.threads, rows=(mid - a.rows // 2, mid + a.rows // 2))
    exact, _ = net.render(2048, 2048, iv, nm, precision=3, **kw)
    f16, _ = net.render(2048, 2048, iv, nm, precision=2, **kw)
    f16s, _ = net2.render(2048, 2048, iv, nm, precision=2, **kw)
    # the largest scaled activation the march actually meets is below 1 by construction (hard bound)
    r0, r1 = compare_frames(f16, exact), compare_frames(f16s, exact)
    print(json.dumps({"geometry": geom[:10], "scales_e": e, "tops": [round(t, 3) for t in tops],
                      "fp16_vs_exact": {"identical": round(r0["identical"], 4), "iou": round(r0["iou"], 5)},
                      "fp16_scaled_vs_exact": {"identical": round(r1["identical"], 4), "iou": round(r1["iou"], 5)}}),
          flush=True)
