"""Diagnostic: where do batched reduced-precision renders differ from single-frame renders?
Iteration maps (nr_set_debug itmap) of repeated batched launches against the single-frame
map: frame, pixel block, queue position within the frame and the iteration counts (GPU box)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dims, K, B = nr.read_keras_h5(nr.geometry_path("car_1"))
r = nr.Renderer(0).load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
r.set_matcap(nr.load_png(nr.matcap_path("Chrome")))
W, H = 160, 144
rng = np.random.default_rng(11)
cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(6)]
mode = sys.argv[3] if len(sys.argv) > 3 else "itmap"
if mode == "itmap":
    r.set_debug(8)
ref = []
for iv, nm, fr in cams:
    r.set_view(iv, nm, fr)
    ref.append(r.render(W, H, 128)[0])
nbad = 0
for trial in range(trials):
    imgs = r.render_batch(W, H, cams, 128)[0]
    for f, (im, rf) in enumerate(zip(imgs, ref)):
        d = np.argwhere(im != rf)
        if not len(d):
            continue
        nbad += 1
        if nbad > 12:
            continue
        ys, xs = d[:, 0], d[:, 1]
        blk = sorted(set(((ys // 8) * (W // 8) + xs // 8).tolist()))
        pq = sorted(set(((ys % 8) * 8 + xs % 8).tolist()))
        vals = im[ys, xs]
        same_pos = [g for g in range(len(ref)) if np.array_equal(ref[g][ys, xs], vals)]
        shifted = []
        for g in range(len(ref)):
            for dy in range(-16, 17):
                for dx in range(-16, 17):
                    yy, xx = ys + dy, xs + dx
                    if (dy or dx or g != f) and yy.min() >= 0 and xx.min() >= 0 and yy.max() < H and xx.max() < W \
                            and np.array_equal(ref[g][yy, xx], vals):
                        shifted.append((g, dy, dx))
        print(f"  matches single render of frames {same_pos} at the same pixels; shifted matches {shifted[:6]}")
        print(f"trial {trial} frame {f}: {len(d)} px, blocks {blk}, in-block positions {pq[:20]}, "
              f"values batch {im[ys, xs][:16].tolist()} single {rf[ys, xs][:16].tolist()}", flush=True)
print(prec, trials, "trials,", nbad, "differing frames")
