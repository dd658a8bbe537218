import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import cudaneuralrender_amd as nr
out = torch.zeros(1024*1024, dtype=torch.int32, device="cuda")
for pst, take in [(0,16),(16,16),(32,16),(32,4),(128,16)]:
    r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
    r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(nr.load_png(nr.matcap_path("Chrome")))
    r.set_cost_probe(pst, take)
    for _ in range(3): r.render_device(out.data_ptr(), 1024, 1024, 128)
    r.set_profiling(True)
    for _ in range(10): r.render_device(out.data_ptr(), 1024, 1024, 128)
    print(pst, take, r.prof_collect(), flush=True)
    del r
