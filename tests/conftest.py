import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnr.so on cuda:0)")


GEOMS = ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]


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
