"""fp32 drift from floating-point contraction.  The CPU oracle is built twice:
-ffp-contract=off (the parity contract shared with the HIP kernels) and -ffp-contract=fast on
an FMA target (x86-64-v3), which fuses a*b+c wherever the source has it -- what nvcc's default
--fmad=true does to the reference's dot()/length() (helper_math.h), sdfOpSmoothUnion
(volumeRender_kernel.cu:145-149), intersectSphere and the colour arithmetic.  Both render the
same frames; their difference is the expected pixel drift of this repo's (bit-exact to the
contraction-free restatement) fp32 frames against the real reference binary.

    python tools/contract_drift.py [--size 1024] [--steps 128]      (CPU only)
prints one JSON object per frame: identical-pixel fraction, coverage IoU, mean / max |delta|
per channel over pixels both cover, ray-steps of both builds."""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--steps", type=int, default=128)
ap.add_argument("--geoms", default="plane_1,car_1")
ap.add_argument("--render-to", default="", help=argparse.SUPPRESS)  # child mode
a = ap.parse_args()
FRAMES = [(g, cam) for g in a.geoms.split(",") for cam in [(0.0, 0.0, 2.0), (-18.3, 150.7, 2.25)]]


def render_all(outdir):
    import cudaneuralrender_amd as nr
    import oracle
    mc = nr.load_png(nr.matcap_path("Chrome"))
    for i, (g, (rx, ry, zoom)) in enumerate(FRAMES):
        dims, K, B = nr.read_keras_h5(nr.geometry_path(g))
        iv, nm = nr.camera(rx, ry, zoom)
        img, st = oracle.OracleNet(K, B).render(a.size, a.size, iv, nm, color_type=1, matcap=mc, max_steps=a.steps)
        np.save(os.path.join(outdir, f"f{i}.npy"), img)
        np.save(os.path.join(outdir, f"s{i}.npy"), np.array([st["ray_steps"]], np.int64))


def channels(img):
    return np.stack([(img >> (8 * c)) & 0xff for c in range(4)], -1).astype(np.int32)


if a.render_to:
    render_all(a.render_to)
    sys.exit(0)

subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all", "fma"], check=True)
with tempfile.TemporaryDirectory() as tmp:
    dirs = {}
    for tag, so in [("off", "liboracle.so"), ("fast", "liboracle_fma.so")]:
        d = os.path.join(tmp, tag)
        os.makedirs(d)
        env = dict(os.environ, OR_LIBRARY=os.path.join(REPO, "oracle", "_build", so))
        subprocess.run([sys.executable, __file__, "--size", str(a.size), "--steps", str(a.steps), "--geoms", a.geoms,
                        "--render-to", d], env=env, check=True)
        dirs[tag] = d
    for i, (g, cam) in enumerate(FRAMES):
        x, y = (np.load(os.path.join(dirs[t], f"f{i}.npy")) for t in ("off", "fast"))
        sx, sy = (int(np.load(os.path.join(dirs[t], f"s{i}.npy"))[0]) for t in ("off", "fast"))
        fx, fy = x != 0, y != 0
        both = fx & fy
        d = np.abs(channels(x) - channels(y))[both]
        print(json.dumps({"geometry": g, "camera": cam, "size": a.size, "steps": a.steps,
                          "identical": round(float((x == y).mean()), 6),
                          "iou": round(float(both.sum() / max((fx | fy).sum(), 1)), 6),
                          "mean_abs_rgba": [round(float(v), 4) for v in d.mean(0)],
                          "max_abs_rgba": [int(v) for v in d.max(0)],
                          "ray_steps_off": sx, "ray_steps_fast": sy}), flush=True)
