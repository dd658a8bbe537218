"""Python host side of the renderer: a thin object wrapper over the C ABI.

Mirrors the reference's host flow (src/main.cpp:636-678 -> generateSingleImage
:404-468): load the network (NeuralNetwork::load), optionally a matcap
(Image::loadPNG), copyStaticSettings, updateViewMatrices + copyViewMatrices, then
render_kernel.  All compute runs in libnr.so on the GPU.
"""
import ctypes

import numpy as np

from ._lib import (NR_COLOR_FACING, NR_COLOR_MATCAP, NR_DEVICE, NR_GROUP_ASYNC, NR_GROUP_COPY, NR_HOST, NR_PRECISION,
                   NR_SCENE, NR_SCHEDULE, NRFrame, NRKernelProf, NRStats, check, lib)

_FP = ctypes.POINTER(ctypes.c_float)


def _fptr(a):
    return a.ctypes.data_as(_FP)


CAMERA_MODES = {"f64": 0, "eigen": 1}


def camera(rx=0.0, ry=0.0, zoom=2.0, tx=0.0, ty=0.0, mode="f64"):
    """updateViewMatrices (main.cpp:207-222): returns (inv_view[12], normal[16]) float32.

    ``zoom`` is the value of the reference's ``-z`` flag (default 2): the eye sits at
    R * (tx, ty, zoom)... i.e. viewTranslation = (tx, ty, -zoom).  ``mode`` "f64": double
    arithmetic rounded once (nr_camera); "eigen": the reference's float Eigen expression restated
    (nr_camera_ex NR_CAMERA_EIGEN)."""
    iv = np.zeros(12, np.float32)
    nm = np.zeros(16, np.float32)
    check(lib().nr_camera_ex(rx, ry, zoom, tx, ty, CAMERA_MODES[mode], _fptr(iv), _fptr(nm)))
    return iv, nm


def read_keras_h5(path):
    """NeuralNetwork::load's reader (neuralNetwork.cpp:85-151) without a device:
    returns (dims, [kernel (in, out)], [bias (out,)])."""
    L = lib()
    nl = ctypes.c_int(0)
    check(L.nr_h5_read_keras(path.encode(), 0, ctypes.byref(nl), None, None, 0))
    dims = (ctypes.c_int * (nl.value + 1))()
    check(L.nr_h5_read_keras(path.encode(), nl.value, ctypes.byref(nl), dims, None, 0))
    dims = list(dims)
    total = sum(dims[i] * dims[i + 1] + dims[i + 1] for i in range(nl.value))
    buf = np.zeros(total, np.float32)
    check(L.nr_h5_read_keras(path.encode(), nl.value, ctypes.byref(nl), None, _fptr(buf), total))
    kernels, biases, off = [], [], 0
    for i in range(nl.value):
        n = dims[i] * dims[i + 1]
        kernels.append(buf[off:off + n].reshape(dims[i], dims[i + 1]).copy())
        off += n
        biases.append(buf[off:off + dims[i + 1]].copy())
        off += dims[i + 1]
    return dims, kernels, biases


def load_png(path):
    """Image::loadPNG (image.cu:36-65): (h, w) uint32 packed a<<24|b<<16|g<<8|r."""
    L = lib()
    p = ctypes.POINTER(ctypes.c_uint32)()
    w, h = ctypes.c_int(0), ctypes.c_int(0)
    check(L.nr_png_load(path.encode(), ctypes.byref(p), ctypes.byref(w), ctypes.byref(h)))
    try:
        arr = np.ctypeslib.as_array(p, shape=(h.value * w.value,)).copy().reshape(h.value, w.value)
    finally:
        L.nr_free(ctypes.cast(p, ctypes.c_void_p))
    return arr


def save_png(path, img, flip=True):
    """Image::savePNG (image.cu:67-110); flip=True is the reference's 180-degree rotation."""
    img = np.ascontiguousarray(img, dtype=np.uint32)
    check(lib().nr_png_save(path.encode(), img.ctypes.data, img.shape[1], img.shape[0], int(flip)))


def save_ppm(path, img):
    img = np.ascontiguousarray(img, dtype=np.uint32)
    check(lib().nr_ppm_save(path.encode(), img.ctypes.data, img.shape[1], img.shape[0]))


def pack_x3(dims, kernels, biases):
    """The library's fp32x3 pack of a fused-shape network (nr_pack_x3; host only): (a_ops uint16,
    floats float32, ok).  For the test oracle's emulation of the fp32x3 MLP (the bf16/fp16 tracers'
    normals)."""
    L = lib()
    nl = len(kernels)
    d = (ctypes.c_int * (nl + 1))(*dims)
    ks = [np.ascontiguousarray(k, np.float32) for k in kernels]
    bs = [np.ascontiguousarray(b, np.float32) for b in biases]
    kp = (_FP * nl)(*[_fptr(k) for k in ks])
    bp = (_FP * nl)(*[_fptr(b) for b in bs])
    na, nf, ok = ctypes.c_long(0), ctypes.c_long(0), ctypes.c_int(0)
    check(L.nr_pack_x3(nl, d, kp, bp, None, 0, None, 0, ctypes.byref(na), ctypes.byref(nf), ctypes.byref(ok)))
    a = np.zeros(na.value, np.uint16)
    f = np.zeros(nf.value, np.float32)
    check(L.nr_pack_x3(nl, d, kp, bp, a.ctypes.data, na.value, f.ctypes.data, nf.value, ctypes.byref(na),
                       ctypes.byref(nf), ctypes.byref(ok)))
    return a, f, ok.value


def shard_rows(H, band, nshards, shard):
    return lib().nr_shard_rows(H, band, nshards, shard)


def group_layout(W, H, band, n, nframes):
    """nr_group_layout: (shard_px, per_rank) of nr_group_render_batch's gather buffer."""
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    check(lib().nr_group_layout(W, H, band, n, nframes, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def batch_frames_per_launch(W, H, band, nshards, shard, nframes, queue_shards=8):
    """Frames nr_render_batch puts in one k_trace launch (0: the shard overflows the
    32-bit pixel queue even for one frame)."""
    return lib().nr_batch_frames_per_launch(W, H, band, nshards, shard, nframes, queue_shards)


def assemble_shards(shards, W, H, band, nshards):
    """Host re-interleave of gathered shards (list or stacked array, each padded to a
    common stride) into the full frame."""
    stride = max(shard_rows(H, band, nshards, s) for s in range(nshards)) * W
    buf = np.zeros((nshards, stride), np.uint32)
    for s, sh in enumerate(shards):
        a = np.asarray(sh, np.uint32).reshape(-1)
        buf[s, :a.size] = a
    out = np.zeros((H, W), np.uint32)
    check(lib().nr_assemble_shards(None, buf.ctypes.data, stride, out.ctypes.data, W, H, band, nshards, NR_HOST))
    return out


class Renderer:
    """One renderer context per GPU (nr_ctx)."""

    def __init__(self, device=0):
        self._L = lib()
        self._ctx = ctypes.c_void_p()
        check(self._L.nr_create(device, ctypes.byref(self._ctx)))
        self.device = device

    # -- lifecycle
    def close(self):
        if self._ctx:
            self._L.nr_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc):
        return check(rc, self._ctx)

    # -- network
    def load_h5(self, path):
        self._chk(self._L.nr_load_h5(self._ctx, path.encode()))
        return self

    def load_mlp(self, dims, kernels, biases):
        nl = len(kernels)
        d = (ctypes.c_int * (nl + 1))(*dims)
        ks = [np.ascontiguousarray(k, np.float32) for k in kernels]
        bs = [np.ascontiguousarray(b, np.float32) for b in biases]
        kp = (_FP * nl)(*[_fptr(k) for k in ks])
        bp = (_FP * nl)(*[_fptr(b) for b in bs])
        self._chk(self._L.nr_load_mlp(self._ctx, nl, d, kp, bp))
        return self

    def mlp_info(self):
        nl, nw, nb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        dims = (ctypes.c_int * 64)()
        self._chk(self._L.nr_mlp_info(self._ctx, ctypes.byref(nl), dims, ctypes.byref(nw), ctypes.byref(nb)))
        return {"nlayers": nl.value, "dims": list(dims[:nl.value + 1]), "weights": nw.value, "biases": nb.value}

    def set_precision(self, precision):
        self._chk(self._L.nr_set_precision(self._ctx, NR_PRECISION[precision] if isinstance(precision, str) else precision))
        return self

    # -- settings
    def set_view(self, inv_view, normal, frame=0):
        iv = np.ascontiguousarray(inv_view, np.float32).reshape(12)
        nm = np.ascontiguousarray(normal, np.float32).reshape(16)
        self._chk(self._L.nr_set_view(self._ctx, _fptr(iv), _fptr(nm), int(frame)))
        return self

    def set_camera(self, rx=0.0, ry=0.0, zoom=2.0, frame=0):
        iv, nm = camera(rx, ry, zoom)
        return self.set_view(iv, nm, frame)

    def set_static(self, color_type=NR_COLOR_FACING, num_inputs=3):
        self._chk(self._L.nr_set_static(self._ctx, int(color_type), int(num_inputs)))
        return self

    def set_scene(self, scene):
        self._chk(self._L.nr_set_scene(self._ctx, NR_SCENE[scene] if isinstance(scene, str) else int(scene)))
        return self

    def set_matcap(self, rgba):
        m = np.ascontiguousarray(rgba, np.uint32)
        self._chk(self._L.nr_set_matcap(self._ctx, m.ctypes.data, m.shape[1], m.shape[0]))
        return self

    def set_stream(self, stream_ptr=None, own=False):
        """Issue work on `stream_ptr` (a hipStream_t as int; 0/None = HIP's null stream,
        e.g. torch.cuda.current_stream().cuda_stream), or on the private stream (own=True)."""
        self._chk(self._L.nr_set_stream(self._ctx, ctypes.c_void_p(stream_ptr) if stream_ptr else None, int(own)))
        return self

    def set_profiling(self, on=True):
        self._chk(self._L.nr_set_profiling(self._ctx, int(on)))

    def prof_collect(self):
        p = NRKernelProf()
        self._chk(self._L.nr_prof_collect(self._ctx, ctypes.byref(p)))
        return p.as_dict()

    def set_schedule(self, schedule):
        """"persistent" (one k_trace launch per frame, default), "wavefront" (one
        k_march launch per iteration) or "layered" (one dense-layer launch per layer per
        iteration, replayed as a hipGraph; networks of other shapes always use it)."""
        self._chk(self._L.nr_set_schedule(self._ctx, NR_SCHEDULE[schedule] if isinstance(schedule, str) else schedule))
        return self

    def set_occupancy(self, blocks_per_cu):
        self._chk(self._L.nr_set_occupancy(self._ctx, int(blocks_per_cu)))
        return self

    def set_pixel_spread(self, group_blocks):
        """Persistent schedule: deal each group of `group_blocks` 8x8 blocks pixel-major
        (0 = block-major; -1 = automatic, the default: 16 for one-frame launches, 0 for
        nr_render_batch launches of 4 or more frames)."""
        self._chk(self._L.nr_set_pixel_spread(self._ctx, int(group_blocks)))
        return self

    def set_cost_probe(self, max_steps, rays_per_wave=16):
        """Persistent schedule: probe each 8x8 block's centre ray (capped at max_steps
        iterations) before the frame and dispense blocks longest-first (0 = off)."""
        self._chk(self._L.nr_set_cost_probe(self._ctx, int(max_steps), int(rays_per_wave)))
        return self

    def set_wave_rays(self, rays):
        """Persistent schedule: at most `rays` (1-64) rays per wave at once; 0 = automatic (the
        default: 64, or 32 for an fp32 launch whose pixels fill at most 2x its waves' slots)."""
        self._chk(self._L.nr_set_wave_rays(self._ctx, int(rays)))
        return self

    def set_queue_shards(self, n):
        """Persistent schedule: number of pixel-queue counters (power of two <= 64)."""
        self._chk(self._L.nr_set_queue_shards(self._ctx, int(n)))
        return self

    def set_layer_chunk(self, points=0):
        """Layered schedule: points per dense-layer launch (0 = auto)."""
        self._chk(self._L.nr_set_layer_chunk(self._ctx, int(points)))
        return self

    def set_temporal_order(self, on=True):
        self._chk(self._L.nr_set_temporal_order(self._ctx, int(on)))
        return self

    def set_debug(self, flags):
        self._chk(self._L.nr_set_debug(self._ctx, int(flags)))
        return self

    def set_endgame(self, tau):
        """nr_set_endgame: bf16/fp16 rays whose 16-bit MLP output falls below tau finish their
        march in fp32x3 (default NR_ENDGAME_DEFAULT = 1e-3; 0 = the pure 16-bit march)."""
        self._chk(self._L.nr_set_endgame(self._ctx, float(tau)))
        return self

    def debug_stamps(self):
        """Per-wave stamps of the last k_trace: {start, queue drained, end (100 MHz ticks),
        iterations after drain << 32 | iterations, shader-clock cycles in refill, shading,
        MLP, scene, step, within refill: reservation, bulk generation, dealing (bf16/fp16),
        after the drain: cycles in refill + shading + step, MLP, scene, and iterations with at
        most 4 rays}."""
        n = ctypes.c_size_t()
        self._chk(self._L.nr_debug_stamps(self._ctx, None, 0, ctypes.byref(n)))
        buf = np.zeros((n.value, 16), np.uint64)
        self._chk(self._L.nr_debug_stamps(self._ctx, buf.ctypes.data, buf.size, ctypes.byref(n)))
        return buf

    def set_poll_interval(self, every):
        self._chk(self._L.nr_set_poll_interval(self._ctx, int(every)))

    def synchronize(self):
        self._chk(self._L.nr_synchronize(self._ctx))

    # -- hot path
    def render(self, W, H, max_steps=6000, with_stats=True):
        out = np.zeros((H, W), np.uint32)
        st = NRStats()
        self._chk(self._L.nr_render(self._ctx, out.ctypes.data, W, H, max_steps, NR_HOST,
                                    ctypes.byref(st) if with_stats else None))
        return (out, st.as_dict()) if with_stats else out

    def render_device(self, out_ptr, W, H, max_steps=6000, with_stats=False):
        """Render into a device buffer (e.g. a torch tensor's data_ptr())."""
        st = NRStats()
        self._chk(self._L.nr_render(self._ctx, ctypes.c_void_p(out_ptr), W, H, max_steps, NR_DEVICE,
                                    ctypes.byref(st) if with_stats else None))
        return st.as_dict() if with_stats else None

    @staticmethod
    def _frames(cams, outs):
        fr = (NRFrame * len(cams))()
        for i, (cam, o) in enumerate(zip(cams, outs)):
            iv, nm = cam[0], cam[1]
            fr[i].inv_view[:] = [float(v) for v in np.asarray(iv, np.float32).reshape(-1)]
            fr[i].normal[:] = [float(v) for v in np.asarray(nm, np.float32).reshape(-1)]
            fr[i].frame = int(cam[2]) if len(cam) > 2 else 0
            fr[i].out = o
        return fr

    def render_batch(self, W, H, cams, max_steps=6000, band=8, nshards=1, shard=0, with_stats=True):
        """nr_render_batch to host images: cams = [(inv_view, normal[, frame]), ...].
        Returns the list of (rows, W) images (and the summed stats)."""
        rows = shard_rows(H, band, nshards, shard)
        outs = [np.zeros((rows, W), np.uint32) for _ in cams]
        fr = self._frames(cams, [o.ctypes.data for o in outs])
        st = NRStats()
        self._chk(self._L.nr_render_batch(self._ctx, fr, len(cams), W, H, band, nshards, shard, max_steps, NR_HOST,
                                          ctypes.byref(st) if with_stats else None))
        return (outs, st.as_dict()) if with_stats else outs

    def render_batch_device(self, out_ptrs, W, H, cams, max_steps=6000, band=8, nshards=1, shard=0,
                            with_stats=False):
        """nr_render_batch into device buffers (one per camera)."""
        fr = self._frames(cams, list(out_ptrs))
        st = NRStats()
        self._chk(self._L.nr_render_batch(self._ctx, fr, len(cams), W, H, band, nshards, shard, max_steps, NR_DEVICE,
                                          ctypes.byref(st) if with_stats else None))
        return st.as_dict() if with_stats else None

    def render_shard(self, W, H, band, nshards, shard, max_steps=6000, with_stats=True):
        rows = shard_rows(H, band, nshards, shard)
        out = np.zeros((rows, W), np.uint32)
        st = NRStats()
        self._chk(self._L.nr_render_shard(self._ctx, out.ctypes.data, W, H, band, nshards, shard, max_steps,
                                          NR_HOST, ctypes.byref(st) if with_stats else None))
        return (out, st.as_dict()) if with_stats else out

    def render_shard_device(self, out_ptr, W, H, band, nshards, shard, max_steps=6000, with_stats=False):
        st = NRStats()
        self._chk(self._L.nr_render_shard(self._ctx, ctypes.c_void_p(out_ptr), W, H, band, nshards, shard,
                                          max_steps, NR_DEVICE, ctypes.byref(st) if with_stats else None))
        return st.as_dict() if with_stats else None

    def assemble_device(self, src_ptr, stride, dst_ptr, W, H, band, nshards):
        self._chk(self._L.nr_assemble_shards(self._ctx, ctypes.c_void_p(src_ptr), stride, ctypes.c_void_p(dst_ptr),
                                             W, H, band, nshards, NR_DEVICE))

    def mlp_forward(self, X):
        X = np.ascontiguousarray(X, np.float32)
        info = self.mlp_info()
        n = X.shape[0]
        Y = np.zeros((n, info["dims"][-1]), np.float32)
        self._chk(self._L.nr_mlp_forward(self._ctx, X.ctypes.data, Y.ctypes.data, n, NR_HOST))
        return Y

    def mlp_forward_device(self, x_ptr, y_ptr, n):
        self._chk(self._L.nr_mlp_forward(self._ctx, ctypes.c_void_p(x_ptr), ctypes.c_void_p(y_ptr), n, NR_DEVICE))

    def layer_forward(self, layer, A):
        A = np.ascontiguousarray(A, np.float32)
        info = self.mlp_info()
        Z = np.zeros((A.shape[0], info["dims"][layer + 1]), np.float32)
        self._chk(self._L.nr_layer_forward(self._ctx, layer, A.ctypes.data, Z.ctypes.data, A.shape[0], NR_HOST))
        return Z


__all__ = ["Renderer", "camera", "pack_x3", "read_keras_h5", "load_png", "save_png", "save_ppm", "shard_rows",
           "assemble_shards", "NR_COLOR_FACING", "NR_COLOR_MATCAP"]


class Group:
    """nr_group: renderers on distinct GPUs of one process joined by one RCCL communicator.
    render_batch splits every frame into row-band shards (renderer r renders shard r), checks
    every shard's status, gathers the shards to the first renderer's GPU in one RCCL call and
    re-interleaves them there (include/neural_render.h nr_group_render_batch)."""

    def __init__(self, renderers, copy=False, asynchronous=False):
        """copy: NR_GROUP_COPY (hipMemcpyPeerAsync transfers; renderers may share a GPU);
        asynchronous: NR_GROUP_ASYNC (a call returns with its gather enqueued: synchronize())."""
        self._L = lib()
        self.renderers = list(renderers)
        arr = (ctypes.c_void_p * len(self.renderers))(*[r._ctx.value for r in self.renderers])
        self._g = ctypes.c_void_p()
        flags = (NR_GROUP_COPY if copy else 0) | (NR_GROUP_ASYNC if asynchronous else 0)
        check(self._L.nr_group_create_ex(arr, len(self.renderers), flags, ctypes.byref(self._g)))

    def synchronize(self):
        check(self._L.nr_group_synchronize(self._g))
        return self

    def close(self):
        if self._g:
            self._L.nr_group_destroy(self._g)
            self._g = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def size(self):
        return self._L.nr_group_size(self._g)

    def render_batch(self, W, H, cams, max_steps=6000, band=1, with_stats=True):
        """Full frames (H, W) on the host for cams = [(inv_view, normal[, frame]), ...]."""
        outs = [np.zeros((H, W), np.uint32) for _ in cams]
        fr = Renderer._frames(cams, [o.ctypes.data for o in outs])
        st = NRStats()
        check(self._L.nr_group_render_batch(self._g, fr, len(cams), W, H, band, max_steps, NR_HOST,
                                            ctypes.byref(st) if with_stats else None))
        return (outs, st.as_dict()) if with_stats else outs

    def render_batch_device(self, out_ptrs, W, H, cams, max_steps=6000, band=1, with_stats=False):
        """Full frames into device buffers on the first renderer's GPU."""
        fr = Renderer._frames(cams, list(out_ptrs))
        st = NRStats()
        check(self._L.nr_group_render_batch(self._g, fr, len(cams), W, H, band, max_steps, NR_DEVICE,
                                            ctypes.byref(st) if with_stats else None))
        return st.as_dict() if with_stats else None
