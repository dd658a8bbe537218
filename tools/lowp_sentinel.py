"""Diagnostic: repeated batched renders into device images pre-filled with a sentinel; counts
pixels never written and pixels that differ from the single-frame render, and repeats the
single-frame renders (GPU box).
    python tools/lowp_sentinel.py PREC TRIALS [BATCH_OCCUPANCY [SINGLE_OCCUPANCY [FRAMES [WxH]]]]
(occupancy: workgroups per CU of the persistent grid, nr_set_occupancy; 0 = automatic)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 12
occ_b = int(sys.argv[3]) if len(sys.argv) > 3 else 0
occ_s = int(sys.argv[4]) if len(sys.argv) > 4 else 0
ncams = int(sys.argv[5]) if len(sys.argv) > 5 else 6
W, H = (int(v) for v in sys.argv[6].split("x")) if len(sys.argv) > 6 else (160, 144)
dims, K, B = nr.read_keras_h5(nr.geometry_path("car_1"))
r = nr.Renderer(0).load_mlp(dims, K, B).set_precision(prec).set_static(int(os.environ.get("NR_COLOR", nr.NR_COLOR_MATCAP)), 3).set_scene("v1")
r.set_matcap(nr.load_png(nr.matcap_path("Chrome")))
rng = np.random.default_rng(11)
cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(ncams)]
ref, tot = [], np.zeros(3, np.int64)
for iv, nm, fr in cams:
    r.set_view(iv, nm, fr)
    img, s1 = r.render(W, H, 128)
    ref.append(img)
    tot += [s1["ray_steps"], s1["rays_hit"], s1["rays_shaded"]]
print("single-frame totals (ray steps, hit, shaded):", tot.tolist())
SENT = 0x5EED5EED
res = []
r.set_occupancy(occ_b)
for trial in range(trials):
    outs = [torch.full((H, W), SENT, dtype=torch.int64, device="cuda:0").to(torch.int32) for _ in cams]
    torch.cuda.synchronize()
    st = r.render_batch_device([o.data_ptr() for o in outs], W, H, cams, 128, with_stats=True)
    torch.cuda.synchronize()
    imgs = [o.cpu().numpy().view(np.uint32) for o in outs]
    unwritten = sum(int((im == SENT).sum()) for im in imgs)
    diff = sum(int((im != rf).sum()) for im, rf in zip(imgs, ref))
    res.append((unwritten, diff, st["ray_steps"], st["rays_hit"], st["rays_shaded"]))
r.set_occupancy(occ_s)
sd = []
for trial in range(max(1, trials // 3)):
    n = 0
    for (iv, nm, fr), rf in zip(cams, ref):
        r.set_view(iv, nm, fr)
        n += int((r.render(W, H, 128)[0] != rf).sum())
    sd.append(n)
r.set_occupancy(0)
print(prec, f"occupancy {occ_s}: single-frame re-renders, differing pixels per trial:", sd)
bad = [x for x in res if x[0] or x[1]]
print(prec, f"occupancy {occ_b}:", len(res), "batched trials,", len(bad),
      "differing (unwritten, differing, ray steps, hit, shaded):", bad[:8], flush=True)
