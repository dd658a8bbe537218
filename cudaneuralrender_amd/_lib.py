"""ctypes binding of libnr.so (C ABI: include/neural_render.h).

The shared library is built in-tree (``make -C cudaneuralrender_amd/csrc``, or
``__graft_entry__.build()``) into ``cudaneuralrender_amd/lib/libnr.so``.  There is
no fallback: if the library is missing, importing the compute API raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# NR_LIBRARY: an alternative build of the same ABI (A/B experiments under tools/)
LIB_PATH = os.environ.get("NR_LIBRARY") or os.path.join(_HERE, "lib", "libnr.so")

NR_OK = 0
NR_PRECISION = {"fp32": 0, "bf16": 1, "fp16": 2, "fp32x3": 3}
NR_SCENE = {"v1": 0, "tanh": 1, "subtract": 2, "cylinders": 3, "displace": 4, "round": 5}
NR_COLOR_FACING, NR_COLOR_MATCAP = 0, 1
NR_HOST, NR_DEVICE = 0, 1
NR_SCHEDULE = {"persistent": 0, "wavefront": 1, "layered": 2}
NR_GROUP_COPY, NR_GROUP_ASYNC = 1, 2
NR_ENDGAME_DEFAULT = 0.001  # include/neural_render.h: the bf16/fp16 endgame threshold by default

# every symbol include/neural_render.h declares
EXPORTS = [
    "nr_create", "nr_destroy", "nr_last_error", "nr_abi_version", "nr_set_stream", "nr_synchronize",
    "nr_load_h5", "nr_load_mlp", "nr_mlp_info", "nr_set_precision", "nr_set_view", "nr_set_static",
    "nr_set_scene", "nr_set_matcap", "nr_render", "nr_render_shard", "nr_render_batch", "nr_shard_rows",
    "nr_assemble_shards", "nr_mlp_forward", "nr_layer_forward", "nr_camera", "nr_camera_ex", "nr_h5_read_keras",
    "nr_png_load", "nr_png_save", "nr_ppm_save", "nr_free", "nr_set_profiling", "nr_prof_collect",
    "nr_set_poll_interval", "nr_set_schedule", "nr_set_debug", "nr_debug_stamps",
    "nr_set_occupancy", "nr_set_temporal_order", "nr_dense_forward", "nr_set_pixel_spread", "nr_set_cost_probe", "nr_set_wave_rays", "nr_set_queue_shards", "nr_set_layer_chunk", "nr_batch_frames_per_launch",
    "nr_h5_open", "nr_h5_close", "nr_h5_root", "nr_h5_object_type", "nr_h5_num_members", "nr_h5_member",
    "nr_h5_dims", "nr_h5_read_f32",
    "nr_group_create", "nr_group_destroy", "nr_group_size", "nr_group_render_batch", "nr_pack_x3",
    "nr_set_endgame", "nr_group_create_ex", "nr_group_synchronize", "nr_group_layout",
]


class NRStats(ctypes.Structure):
    _fields_ = [
        ("ray_steps", ctypes.c_uint64),
        ("shade_evals", ctypes.c_uint64),
        ("rays_hit", ctypes.c_uint64),
        ("rays_shaded", ctypes.c_uint64),
        ("iterations", ctypes.c_int32),
        ("launches", ctypes.c_int32),
        ("ms_total", ctypes.c_float),
        ("endgame_evals", ctypes.c_uint64),
        ("endgame_switches", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class NRFrame(ctypes.Structure):
    """nr_frame: one frame of nr_render_batch."""
    _fields_ = [
        ("inv_view", ctypes.c_float * 12),
        ("normal", ctypes.c_float * 16),
        ("frame", ctypes.c_int),
        ("out", ctypes.c_void_p),
    ]


class NRKernelProf(ctypes.Structure):
    _fields_ = [
        ("march_ms", ctypes.c_double),
        ("shade_ms", ctypes.c_double),
        ("init_ms", ctypes.c_double),
        ("march_launches", ctypes.c_uint64),
        ("shade_launches", ctypes.c_uint64),
        ("init_launches", ctypes.c_uint64),
        ("renders", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class NRError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[nr error {code}] {msg}")
        self.code = code


_lib = None


def lib():
    """Load libnr.so (once).  Raises if the HIP extension has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libnr.so not built: {LIB_PATH} missing (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, I, F, L64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_long
    FP = ctypes.POINTER(ctypes.c_float)
    IP = ctypes.POINTER(ctypes.c_int)
    sig = {
        "nr_create": (I, [I, ctypes.POINTER(P)]),
        "nr_destroy": (I, [P]),
        "nr_last_error": (ctypes.c_char_p, [P]),
        "nr_abi_version": (I, []),
        "nr_set_stream": (I, [P, P, I]),
        "nr_synchronize": (I, [P]),
        "nr_load_h5": (I, [P, ctypes.c_char_p]),
        "nr_load_mlp": (I, [P, I, IP, ctypes.POINTER(FP), ctypes.POINTER(FP)]),
        "nr_pack_x3": (I, [I, IP, ctypes.POINTER(FP), ctypes.POINTER(FP), P, ctypes.c_long, P, ctypes.c_long,
                           ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long), IP]),
        "nr_mlp_info": (I, [P, IP, IP, IP, IP]),
        "nr_set_precision": (I, [P, I]),
        "nr_set_view": (I, [P, FP, FP, I]),
        "nr_set_static": (I, [P, I, I]),
        "nr_set_scene": (I, [P, I]),
        "nr_set_matcap": (I, [P, P, I, I]),
        "nr_render": (I, [P, P, I, I, I, I, ctypes.POINTER(NRStats)]),
        "nr_render_shard": (I, [P, P, I, I, I, I, I, I, I, ctypes.POINTER(NRStats)]),
        "nr_render_batch": (I, [P, ctypes.POINTER(NRFrame), I, I, I, I, I, I, I, I, ctypes.POINTER(NRStats)]),
        "nr_group_create": (I, [ctypes.POINTER(P), I, ctypes.POINTER(P)]),
        "nr_group_destroy": (I, [P]),
        "nr_group_create_ex": (I, [ctypes.POINTER(P), I, I, ctypes.POINTER(P)]),
        "nr_group_synchronize": (I, [P]),
        "nr_group_layout": (I, [I, I, I, I, I, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
        "nr_group_size": (I, [P]),
        "nr_group_render_batch": (I, [P, ctypes.POINTER(NRFrame), I, I, I, I, I, I, ctypes.POINTER(NRStats)]),
        "nr_shard_rows": (I, [I, I, I, I]),
        "nr_batch_frames_per_launch": (I, [I, I, I, I, I, I, I]),
        "nr_assemble_shards": (I, [P, P, ctypes.c_size_t, P, I, I, I, I, I]),
        "nr_mlp_forward": (I, [P, P, P, L64, I]),
        "nr_layer_forward": (I, [P, I, P, P, L64, I]),
        "nr_camera": (I, [F, F, F, F, F, FP, FP]),
        "nr_camera_ex": (I, [F, F, F, F, F, I, FP, FP]),
        "nr_h5_read_keras": (I, [ctypes.c_char_p, I, IP, IP, FP, ctypes.c_size_t]),
        "nr_h5_open": (I, [ctypes.c_char_p, ctypes.POINTER(P)]),
        "nr_h5_close": (None, [P]),
        "nr_h5_root": (I, [P, ctypes.POINTER(ctypes.c_uint64)]),
        "nr_h5_object_type": (I, [P, ctypes.c_uint64, IP]),
        "nr_h5_num_members": (I, [P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_size_t)]),
        "nr_h5_member": (I, [P, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                             ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint64)]),
        "nr_h5_dims": (I, [P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), I, IP]),
        "nr_h5_read_f32": (I, [P, ctypes.c_uint64, FP, ctypes.c_size_t]),
        "nr_png_load": (I, [ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)), IP, IP]),
        "nr_png_save": (I, [ctypes.c_char_p, P, I, I, I]),
        "nr_ppm_save": (I, [ctypes.c_char_p, P, I, I]),
        "nr_free": (None, [P]),
        "nr_set_profiling": (I, [P, I]),
        "nr_prof_collect": (I, [P, ctypes.POINTER(NRKernelProf)]),
        "nr_set_poll_interval": (I, [P, I]),
        "nr_set_schedule": (I, [P, I]),
        "nr_set_debug": (I, [P, I]),
        "nr_set_endgame": (I, [P, F]),
        "nr_set_occupancy": (I, [P, I]),
        "nr_set_pixel_spread": (I, [P, I]),
        "nr_set_cost_probe": (I, [P, I, I]),
        "nr_set_wave_rays": (I, [P, I]),
        "nr_set_queue_shards": (I, [P, I]),
        "nr_set_layer_chunk": (I, [P, ctypes.c_long]),
        "nr_set_temporal_order": (I, [P, I]),
        "nr_dense_forward": (I, [P, P, P, I, I, I, P, P, L64, I]),
        "nr_debug_stamps": (I, [P, P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc, ctx=None):
    if rc != NR_OK:
        msg = lib().nr_last_error(ctx)
        raise NRError(rc, msg.decode() if msg else "")
    return rc
