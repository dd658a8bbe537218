"""Diagnostic for a build with -DNR_DBG_WCOUNT=1 (every pixel write is an atomicAdd of
0x01000000 | low 24 bits): batched renders into zeroed device images; each pixel's top
byte is the number of times it was written, which must be exactly 1 (GPU box).
    NR_LIBRARY=build/wc/libnr.so python tools/lowp_wcount.py PREC TRIALS"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cudaneuralrender_amd as nr  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dims, K, B = nr.read_keras_h5(nr.geometry_path("car_1"))
r = nr.Renderer(0).load_mlp(dims, K, B).set_precision(prec).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1")
r.set_matcap(nr.load_png(nr.matcap_path("Chrome")))
W, H = 160, 144
rng = np.random.default_rng(11)
cams = [(*nr.camera(float(rng.uniform(-30, 30)), float(rng.uniform(0, 360)), 2.0), 0) for _ in range(6)]
nbad = 0
for trial in range(trials):
    outs = [torch.zeros((H, W), dtype=torch.int32, device="cuda:0") for _ in cams]
    torch.cuda.synchronize()
    st = r.render_batch_device([o.data_ptr() for o in outs], W, H, cams, 128, with_stats=True)
    torch.cuda.synchronize()
    for f, o in enumerate(outs):
        cnt = o.cpu().numpy().view(np.uint32) >> 24
        bad = np.argwhere(cnt != 1)
        if len(bad):
            nbad += 1
            ys, xs = bad[:, 0], bad[:, 1]
            print(f"trial {trial} frame {f}: {len(bad)} px written {sorted(set(cnt[ys, xs].tolist()))} times; "
                  f"blocks {sorted(set(((ys // 8) * (W // 8) + xs // 8).tolist()))[:8]}, "
                  f"in-block {sorted(set(((ys % 8) * 8 + xs % 8).tolist()))[:20]}", flush=True)
print(prec, trials, "trials,", nbad, "frames with a pixel not written exactly once")
