"""Diagnostic for a build with -DNR_DBG_WCOUNT=2 (each pixel's top byte = 1 + the lane that
marched its ray): repeated batched renders against single-frame renders of the same build;
prints the marching lanes of the pixels that differ (GPU box).
    NR_LIBRARY=build/lt/libnr.so python tools/lowp_lanes.py PREC TRIALS"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dims, K, B = nr.read_keras_h5(nr.geometry_path("car_1"))
r = nr.Renderer(0).load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
r.set_matcap(nr.load_png(nr.matcap_path("Chrome")))
W, H = 160, 144
rng = np.random.default_rng(11)
cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(6)]
ref = []
for iv, nm, fr in cams:
    r.set_view(iv, nm, fr)
    ref.append(r.render(W, H, 128)[0] & 0xFFFFFF)
n = 0
for t in range(trials):
    imgs = r.render_batch(W, H, cams, 128)[0]
    for f, (im, rf) in enumerate(zip(imgs, ref)):
        d = np.argwhere((im & 0xFFFFFF) != rf)
        if len(d) and n < 12:
            n += 1
            lanes = sorted(set(((im[d[:, 0], d[:, 1]] >> 24).astype(int) - 1).tolist()))
            print(f"trial {t} frame {f}: {len(d)} px, marching lanes {lanes}", flush=True)
print("done")
