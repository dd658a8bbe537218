"""Refines the camera recovered for a reference render by maximising the
silhouette IoU of the CPU oracle's pure-neural render (sceneSDF -> tanh(nSDF),
volumeRender_kernel.cu:229) against the render's foreground mask (tests/golden/silhouettes.npz):
Nelder-Mead over (rx, ry, zoom[, tx, ty]) of updateViewMatrices (main.cpp:207-222).

    python tools/camera_fit.py NAME RX RY ZOOM [TX TY] [--res 256]

Results (tests/test_gpu_golden.py uses them): plane_1 (-18.3, 150.7, 2.25) -> (-18.8021, 149.7984,
2.2702), IoU 0.966 -> 0.9993 at 256^2; car_1 stays near 0.88 (profiles/r3_shading_search.txt)."""
import argparse
import os
import sys

import numpy as np
from scipy.optimize import minimize

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cudaneuralrender_amd as nr  # noqa: E402
import oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("name")
ap.add_argument("p", type=float, nargs="+")
ap.add_argument("--res", type=int, default=256)
ap.add_argument("--maxfev", type=int, default=120)
a = ap.parse_args()
g = np.load(os.path.join(REPO, "tests", "golden", "silhouettes.npz"))
shape = tuple(g[f"{a.name}/shape"])
gold = np.unpackbits(g[a.name])[: shape[0] * shape[1]].reshape(shape).astype(bool)
k = shape[0] // a.res
gs = gold[::k, ::k]
dims, K, B = nr.read_keras_h5(nr.geometry_path(a.name))
net = oracle.OracleNet(K, B)


def iou(p):
    iv, nm = nr.camera(*p)
    img, _ = net.render(a.res, a.res, iv, nm, color_type=0, scene=1, max_steps=6000, nthreads=8)
    fg = img != 0
    return (fg & gs).sum() / (fg | gs).sum()


p0 = np.array(a.p, float)
steps = [0.5, 0.5, 0.03, 0.03, 0.03][: len(p0)]
simplex = [p0] + [p0 + np.eye(len(p0))[i] * steps[i] for i in range(len(p0))]
print(a.name, a.res, "start", p0, round(iou(p0), 5), flush=True)
r = minimize(lambda p: -iou(p), p0, method="Nelder-Mead",
             options=dict(xatol=0.005, fatol=1e-5, maxfev=a.maxfev, initial_simplex=simplex))
print(a.name, a.res, "refined", r.x.round(4), round(-r.fun, 5))
