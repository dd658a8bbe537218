import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnr.so on cuda:0)")


GEOMS = ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]

# Cameras (rx, ry, zoom) of the reference's own renders neuralGeometries/<g>.h5.ppm, refined from
# SURVEY.md App. A's (plane_1 (-18.3, 150.7, 2.25), car_1 (-79, 229, 3.05): the mirror-image view)
# by maximising the silhouette IoU of the oracle's render (tools/camera_fit.py, a coarse grid for
# car_1 first): at 1024^2 the oracle's foreground differs from the reference render's in 40 of
# 47,890 pixels (plane_1, IoU 0.99917) and 16 of 128,484 (car_1, IoU 0.99988).
REF_CAMERAS = {"plane_1": (-18.8021, 149.7984, 2.2702), "car_1": (80.0, 140.0, 3.1)}


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(REPO, "tests", "golden")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(REPO, "tests", "golden")
    return {
        "weights": np.load(os.path.join(d, "weights_h5py.npz")),
        "kat": np.load(os.path.join(d, "mlp_kat.npz")),
        "sil": np.load(os.path.join(d, "silhouettes.npz")),
    }


@pytest.fixture(scope="session")
def nets():
    """(dims, kernels, biases) for every bundled geometry, read by libnr's HDF5 reader."""
    import cudaneuralrender_amd as nr
    return {g: nr.read_keras_h5(nr.geometry_path(g)) for g in GEOMS}


def channels(img):
    """uint32 RGBA (a<<24|b<<16|g<<8|r) -> [..., 4] int channels"""
    import numpy as np
    return np.stack([(img >> (8 * c)) & 0xff for c in range(4)], -1).astype(np.int32)


def compare_frames(gpu, ref):
    """Identical-pixel fraction, coverage IoU and per-channel mean / max |delta| over the pixels
    both frames cover."""
    import numpy as np
    fg, fr = gpu != 0, ref != 0
    both = fg & fr
    d = np.abs(channels(gpu) - channels(ref))[both] if both.any() else np.zeros((0, 4), np.int32)
    return {"identical": float((gpu == ref).mean()),
            "iou": float(both.sum() / max((fg | fr).sum(), 1)),
            "mean_abs": [round(float(v), 4) for v in (d.mean(0) if len(d) else np.zeros(4))],
            "max_abs": [int(v) for v in (d.max(0) if len(d) else np.zeros(4))]}


@pytest.fixture(scope="module", autouse=True)
def pure_16bit(request):
    """Modules that set PURE_16BIT = True test the pure bf16 / fp16 march (the round-4 contract
    against the oracle's precision-1/2 restatement, and the schedules against each other): every
    Renderer they create starts with nr_set_endgame(ctx, 0) instead of the library's default
    threshold (NR_ENDGAME_DEFAULT; the endgame's own contract: test_gpu_endgame.py,
    test_gpu_lowp_contract.py)."""
    if not getattr(request.module, "PURE_16BIT", False):
        yield
        return
    import cudaneuralrender_amd as nr
    init = nr.Renderer.__init__

    def init_pure(self, *a, **kw):
        init(self, *a, **kw)
        self.set_endgame(0.0)

    nr.Renderer.__init__ = init_pure
    try:
        yield
    finally:
        nr.Renderer.__init__ = init
