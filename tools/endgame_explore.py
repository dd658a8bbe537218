"""CPU exploration of the reduced-precision endgame (oracle or_set_endgame):
for thresholds tau, the oracle's bf16 / fp16 render with the fp32x3 endgame against the exact-MLP
frame (identical pixels, coverage IoU, mean |delta|) and the share of march evaluations that run
in fp32x3.  Row crops of the BASELINE C3-C5 frames (fewer rows than the GPU tests' crops).
usage: python tools/endgame_explore.py [--rows N] [--taus 0,0.005,0.01,...] [--configs C3,C4,C5]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import cudaneuralrender_amd as nr  # noqa: E402
import oracle  # noqa: E402
from conftest import GEOMS, compare_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=32)
ap.add_argument("--taus", default="0,0.002,0.005,0.01,0.02,0.05")
ap.add_argument("--configs", default="C3,C4,C5")
ap.add_argument("--threads", type=int, default=8)
a = ap.parse_args()
CFG = {"C3": [("car_1", 2048, 256, 1)], "C4": [("plane_2", 4096, 128, 1)],
       "C5": [(g, 2048, 128, 2) for g in GEOMS]}
chrome = nr.load_png(nr.matcap_path("Chrome"))
iv, nm = nr.camera(0.0, 0.0, 2.0)
for c in a.configs.split(","):
    for geom, size, steps, prec in CFG[c]:
        dims, K, B = nr.read_keras_h5(nr.geometry_path(geom))
        pack = nr.pack_x3(dims, K, B)
        net = oracle.OracleNet(K, B, x3_pack=pack[:2])
        mid = size // 2
        rows = (mid - a.rows // 2, mid + a.rows // 2)
        kw = dict(color_type=1, matcap=chrome, max_steps=steps, nthreads=a.threads, rows=rows)
        exact, _ = net.render(size, size, iv, nm, precision=3, **kw)
        f32, _ = net.render(size, size, iv, nm, precision=0, **kw)
        x3, sx3 = net.render(size, size, iv, nm, precision=4, **kw)
        base = {"config": c, "geometry": geom[:10], "rows": rows, "fp32_vs_exact": compare_frames(f32, exact)["identical"],
                "x3_vs_exact": compare_frames(x3, exact)["identical"], "x3_iou": compare_frames(x3, exact)["iou"]}
        print(json.dumps(base), flush=True)
        for tau in (float(t) for t in a.taus.split(",")):
            img, st = net.render(size, size, iv, nm, precision=prec, endgame=tau, **kw)
            r = compare_frames(img, exact)
            print(json.dumps({"config": c, "geometry": geom[:10], "tau": tau, "identical": round(r["identical"], 4),
                              "iou": round(r["iou"], 5), "mean_abs": max(r["mean_abs"][:3]),
                              "ray_steps": st["ray_steps"], "fine_share": round(st.get("endgame_evals", 0) / max(st["ray_steps"], 1), 4)}),
                  flush=True)
