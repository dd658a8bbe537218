import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
import cudaneuralrender_amd as nr
mat = nr.load_png(nr.matcap_path("Chrome"))
def mk():
    r = nr.Renderer(0).load_h5(nr.geometry_path("plane_1"))
    r.set_camera(0, 0, 2).set_static(1, 3).set_scene("v1").set_matcap(mat)
    return r
for depth in [1, 2, 3]:
    rs = [mk() for _ in range(depth)]
    outs = [torch.zeros(1024 * 1024, dtype=torch.int32, device="cuda") for _ in range(depth)]
    for i in range(6):
        rs[i % depth].render_device(outs[i % depth].data_ptr(), 1024, 1024, 128)
    for r in rs: r.synchronize()
    K = 30
    t0 = time.perf_counter()
    for i in range(K):
        rs[i % depth].render_device(outs[i % depth].data_ptr(), 1024, 1024, 128)
    for r in rs: r.synchronize()
    dt = time.perf_counter() - t0
    print(f"depth {depth}: {dt / K * 1e3:.3f} ms/frame  {14825508 * K / dt / 1e6:.1f} Mray-steps/s")
    for r in rs: r.close()
