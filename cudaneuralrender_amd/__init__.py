"""MI355X-native neural-SDF sphere tracer (drop-in for daviesthomas/cudaNeuralRender's
render_kernel + NeuralNetwork::forward hot path).

Compute lives in ``lib/libnr.so`` (HIP, gfx950) behind the C ABI of
``include/neural_render.h``; this package is the Python host side.
"""
import os

from ._lib import LIB_PATH, NR_ENDGAME_DEFAULT, NR_PRECISION, NR_SCENE, NR_SCHEDULE, NRError, lib  # noqa: F401
from .renderer import (NR_COLOR_FACING, NR_COLOR_MATCAP, Group, Renderer, assemble_shards, camera,  # noqa: F401
                       load_png, pack_x3, read_keras_h5, save_png, save_ppm, shard_rows, batch_frames_per_launch,
                       group_layout)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
DATA_DIR = os.path.join(REPO_DIR, "data")


def geometry_path(name):
    """Path of a bundled neuralGeometries/<name>.h5 (copied from the reference as data)."""
    return os.path.join(DATA_DIR, "neuralGeometries", name if name.endswith(".h5") else name + ".h5")


def matcap_path(name):
    return os.path.join(DATA_DIR, "matcaps", name if name.endswith(".png") else name + ".png")
