"""fp32x3 exploration on the GPU box: MLP error against the fp64 KAT, pixel agreement of
fp32x3 frames with the fp32 oracle next to the band an exact (fp64) MLP gives, and
single / batched frame times against fp32.  Prints JSON lines; no asserts."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cudaneuralrender_amd as nr  # noqa: E402
import oracle  # noqa: E402

GEOMS = ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]
kat = np.load(os.path.join(REPO, "tests", "golden", "mlp_kat.npz"))
chrome = nr.load_png(nr.matcap_path("Chrome"))


def channels(img):
    return np.stack([(img >> (8 * c)) & 0xff for c in range(4)], -1).astype(np.int32)


def compare(a, b):
    fa, fb = a != 0, b != 0
    both = fa & fb
    d = np.abs(channels(a) - channels(b))[both][:, :3]
    return {"identical": round(float((a == b).mean()), 5), "iou": round(float(both.sum() / max((fa | fb).sum(), 1)), 6),
            "mean_abs": round(float(d.mean()) if len(d) else 0.0, 4)}


for g in GEOMS:
    dims, K, B = nr.read_keras_h5(nr.geometry_path(g))
    X = kat["X"]
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path(g)).set_precision("fp32x3")
        y3 = r.mlp_forward(X)[:, 0]
    y32 = oracle.OracleNet(K, B).forward(X)[:, 0]
    ref = kat[g]
    print(json.dumps({"kat": g, "x3_max": float(np.abs(y3 - ref).max()), "x3_mean": float(np.abs(y3 - ref).mean()),
                      "f32_max": float(np.abs(y32 - ref).max()), "f32_mean": float(np.abs(y32 - ref).mean())}), flush=True)

CASES = [("C2", "plane_1", 1024, 128, None, 0, 0), ("C2-oblique", "plane_1", 1024, 128, None, -20, 150),
         ("C3", "car_1", 2048, 256, (896, 1152), 0, 0), ("C4", "plane_2", 4096, 128, (1984, 2112), 0, 0)]
CASES += [("C5", g, 2048, 128, (960, 1088), 0, 0) for g in GEOMS]
for name, g, size, steps, rows, rx, ry in CASES:
    dims, K, B = nr.read_keras_h5(nr.geometry_path(g))
    iv, nm = nr.camera(rx, ry, 2.0)
    out = {}
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path(g)).set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
        r.set_matcap(chrome)
        for prec in ("fp32", "fp32x3"):
            r.set_precision(prec)
            img, st = r.render(size, size, steps)
            t = []
            for _ in range(3):
                _, s2 = r.render(size, size, steps)
                t.append(s2["ms_total"])
            imgs, bst = r.render_batch(size, size, [(iv, nm, 0)] * 8, steps)
            out[prec] = (img, st, min(t), bst["ms_total"] / 8)
    y0, y1 = rows if rows else (0, size)
    net = oracle.OracleNet(K, B)
    kw = dict(color_type=1, matcap=chrome, max_steps=steps, nthreads=16, rows=(y0, y1))
    t0 = time.time()
    f32, _ = net.render(size, size, iv, nm, precision=0, **kw)
    f64, _ = net.render(size, size, iv, nm, precision=3, **kw)
    res = {"case": name, "geom": g, "size": size, "rows": [y0, y1],
           "fp32_gpu_eq_oracle": bool(np.array_equal(out["fp32"][0][y0:y1], f32)),
           "x3_vs_fp32_oracle": compare(out["fp32x3"][0][y0:y1], f32),
           "fp64march_vs_fp32_oracle": compare(f64, f32),
           "x3_vs_fp64march": compare(out["fp32x3"][0][y0:y1], f64),
           "ray_steps": [out["fp32"][1]["ray_steps"], out["fp32x3"][1]["ray_steps"]],
           "ms_single": [round(out["fp32"][2], 3), round(out["fp32x3"][2], 3)],
           "ms_batch8": [round(out["fp32"][3], 3), round(out["fp32x3"][3], 3)],
           "oracle_s": round(time.time() - t0, 1)}
    print(json.dumps(res), flush=True)
