/*
 * neural_render.h -- C ABI of libnr.so, the MI355X (gfx950) neural-SDF renderer.
 *
 * Drop-in boundary for the reference's hot path (daviesthomas/cudaNeuralRender @ v1):
 * the sphere-trace loop of src/volumeRender_kernel.cu and the batched dense-layer
 * forward of src/layers/denseLayer.cu + src/neuralNetwork.cpp.  Every entry point
 * takes plain pointers and sizes; state lives in an opaque per-device context
 * (the reference keeps it in non-reentrant globals, volumeRender_kernel.cu:31-35,
 * :578-585).  Functions return NR_OK (0) or a negative NR_E* code; the message is
 * available from nr_last_error().  Nothing in the library calls exit()/abort()
 * (the reference exits inside checkCudaErrors, helper_cuda.h:576-591).
 *
 * Threading: one context per GPU; calls on one context are not thread-safe, calls
 * on different contexts are.  Each context owns one HIP stream.
 */
#ifndef NEURAL_RENDER_H
#define NEURAL_RENDER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NR_ABI_VERSION 3   /* 2: nr_stats.endgame_evals, nr_set_endgame (round 5); 3: nr_stats.endgame_switches (round 6) */

/* status codes */
#define NR_OK 0
#define NR_E_INVALID (-1)    /* bad argument */
#define NR_E_HIP (-2)        /* HIP runtime error */
#define NR_E_IO (-3)         /* file missing / unreadable */
#define NR_E_FORMAT (-4)     /* unsupported HDF5 / PNG content */
#define NR_E_STATE (-5)      /* call out of order (e.g. render before load) */
#define NR_E_NOMEM (-6)

/* MLP arithmetic for the 32x32 hidden layers */
#define NR_PRECISION_FP32 0  /* bit-exact with the CPU oracle (f32 MFMA = fmaf chain) */
#define NR_PRECISION_BF16 1  /* bf16 MFMA, f32 accumulate; normals (the 4 tetrahedron samples) in fp32x3,
                                 nr_set_debug bit 15: fp32; rays near a surface finish in fp32x3
                                 (nr_set_endgame, on by default) */
#define NR_PRECISION_FP16 2  /* fp16 MFMA, f32 accumulate; normals and endgame as bf16 */
#define NR_PRECISION_FP32X3 3 /* fp32-class on the fp16 matrix core: three-term split a.w ~ ah.wh + al.wh + ah.wl,
                                  f32 accumulate (~2-3x the f32 chain's error against an exact
                                  evaluation); normals evaluated in fp32 (bit-exact); points with
                                  inputs outside the pack's bounds run the fp32 MLP */

/* scene composition, sceneSDF (volumeRender_kernel.cu:217-230) */
#define NR_SCENE_V1 0        /* v1: manySphere(p, nSDF, true) -- 9-sphere smooth union (:222) */
#define NR_SCENE_TANH 1      /* tanh(nSDF), the pure neural surface (:229) */
#define NR_SCENE_SUBTRACT 2  /* manySphere(p, nSDF, false) -- 9 spheres smooth-subtracted (:139-142, :190-191) */
#define NR_SCENE_CYLINDERS 3 /* manyCylinderCut(p, nSDF) -- 300 cylinders smooth-subtracted (:157-174) */
#define NR_SCENE_DISPLACE 4  /* displacementPattern(p, nSDF) = sdfOpDisplace(p, tanh(nSDF)) (:104-110, :152-154) */
#define NR_SCENE_ROUND 5     /* sdfOpRound(tanh(nSDF), 0.04) (:112-115, :221) */

/* colouring, c_coloringType (volumeRender_kernel.cu:33) */
#define NR_COLOR_FACING 0    /* facingColor (:380-384) */
#define NR_COLOR_MATCAP 1    /* matCapColor (:387-413) */

/* march schedule (nr_set_schedule) */
#define NR_SCHED_PERSISTENT 0 /* one persistent k_trace launch per frame (default) */
#define NR_SCHED_WAVEFRONT 1  /* one k_march launch per iteration over a compacted ray queue */
#define NR_SCHED_LAYERED 2    /* the reference's structure: per iteration one dense-layer launch per
                                 layer over the live-ray queue, then the step; replayed as a hipGraph.
                                 Any dense [3|4, ..., 1] network, fp32.  Networks the fused kernels
                                 do not take ([3|4, 32, ..., 32, 1]) always render this way. */

/* buffer location flags */
#define NR_HOST 0
#define NR_DEVICE 1

typedef struct nr_ctx nr_ctx;

typedef struct nr_stats {
    uint64_t ray_steps;      /* MLP evaluations of marching rays (one per live ray per iteration) */
    uint64_t shade_evals;    /* MLP evaluations for tetrahedral normals (4 per coloured ray) */
    uint64_t rays_hit;       /* rays that entered the bounding sphere */
    uint64_t rays_shaded;    /* pixels coloured */
    int32_t iterations;      /* march iterations that had live rays (reference host-loop count) */
    int32_t launches;        /* kernel launches issued */
    float ms_total;          /* device time of the render, HIP events */
    uint64_t endgame_evals;  /* bf16/fp16 with the endgame (nr_set_endgame): the march evaluations
                                in fp32x3, included in ray_steps */
    uint64_t endgame_switches; /* the rays handed to the endgame: each one's switch point is evaluated
                                in 16 bits and again in fp32x3, and both evaluations are counted in
                                ray_steps (ray_steps - endgame_switches counts every march point once) */
} nr_stats;

/* ---- context ------------------------------------------------------------ */
int nr_create(int device, nr_ctx **out);
int nr_destroy(nr_ctx *ctx);
/* Last error of this context (ctx may be NULL: last error of the calling thread). */
const char *nr_last_error(const nr_ctx *ctx);
int nr_abi_version(void);
/* Stream the context's work is issued on: own != 0 selects the context's private
 * (non-blocking) stream; otherwise hip_stream is used verbatim, NULL meaning HIP's
 * default (null) stream -- e.g. torch.cuda.current_stream().cuda_stream. */
int nr_set_stream(nr_ctx *ctx, void *hip_stream, int own);
int nr_synchronize(nr_ctx *ctx);

/* ---- network (NeuralNetwork::load / DenseLayer ctor) ---------------------- */
/* Replaces NeuralNetwork::load(fp) (neuralNetwork.cpp:85-151): root groups in HDF5
 * name order, each holding one subgroup with "bias:0" (1-D) and "kernel:0" (2-D,
 * Keras (in, out)); last layer linear, others ReLU. */
int nr_load_h5(nr_ctx *ctx, const char *path);
/* Replaces DenseLayer(name, weights, biases, act) x nlayers (denseLayer.cu:180-227).
 * dims[nlayers+1]; kernels[l] is the Keras (in=dims[l], out=dims[l+1]) row-major
 * matrix, biases[l] has dims[l+1] floats.  ReLU on all layers but the last. */
int nr_load_mlp(nr_ctx *ctx, int nlayers, const int *dims,
                const float *const *kernels, const float *const *biases);
/* The fp32x3 pack of a [3|4, 32, ..., 32, 1] network (host only, no GPU): fp16 hi / residual
 * operands a[*a_len] in the kernels' layout and the floats f[*f_len] (scaled biases, final layer,
 * scales); *ok = 0 when the scales do not fit fp16 (the kernels then run fp32).  Copies only when
 * the capacities suffice (call with a = f = NULL for the lengths).  For the test oracle's fp32x3
 * emulation (the bf16/fp16 tracers' normals); not part of the reference's interface. */
int nr_pack_x3(int nlayers, const int *dims, const float *const *kernels, const float *const *biases,
               uint16_t *a, long a_cap, float *f, long f_cap, long *a_len, long *f_len, int *ok);
int nr_mlp_info(const nr_ctx *ctx, int *nlayers, int *dims /* >= nlayers+1 or NULL */,
                int *num_weight_params, int *num_bias_params);
int nr_set_precision(nr_ctx *ctx, int precision);

/* ---- per-frame settings (copyViewMatrices / copyStaticSettings) ---------- */
/* Replaces copyViewMatrices (volumeRender_kernel.cu:694-700): inv_view = rows 0..2
 * of the model-view matrix (3x4 row-major, c_invViewMatrix), normal = its inverse
 * (4x4 row-major, c_normalMatrix), frame = c_frameNumber. */
int nr_set_view(nr_ctx *ctx, const float inv_view[12], const float normal[16], int frame);
/* Replaces copyStaticSettings (volumeRender_kernel.cu:702-706). */
int nr_set_static(nr_ctx *ctx, int color_type, int num_inputs);
int nr_set_scene(nr_ctx *ctx, int scene);
/* Replaces Image::loadPNG + the matcap argument of render_kernel (image.cu:36-65):
 * w*h texels packed a<<24 | b<<16 | g<<8 | r, row 0 = first PNG row. */
int nr_set_matcap(nr_ctx *ctx, const uint32_t *rgba, int w, int h);

/* ---- the hot path --------------------------------------------------------- */
/* Replaces render_kernel (volumeRender_kernel.cu:608-692): renders a W x H frame,
 * at most max_steps march iterations (reference MAX_STEPS = 6000), into out
 * (W*H packed RGBA, row y*W + x, unconverged / missed pixels 0).  out_loc is
 * NR_HOST or NR_DEVICE.  stats may be NULL.  Any dense network with 3 or 4 inputs and
 * one output renders (NeuralNetwork takes any layer list, neuralNetwork.cpp:85-151):
 * [3|4, 32, ..., 32, 1] on the fused kernels of the selected schedule, every other
 * shape on NR_SCHED_LAYERED. */
int nr_render(nr_ctx *ctx, uint32_t *out, int W, int H, int max_steps, int out_loc,
              nr_stats *stats);
/* Multi-GPU shard of a frame: rows are dealt in bands of band_rows, band b goes to
 * shard b % nshards.  out receives this shard's rows only, in increasing y
 * (nr_shard_rows() of them, each W wide).  Pixels are identical to the same rows
 * of nr_render. */
int nr_render_shard(nr_ctx *ctx, uint32_t *out, int W, int H, int band_rows,
                    int nshards, int shard, int max_steps, int out_loc, nr_stats *stats);

/* Batched frames (persistent schedule): render nframes frames -- each with its own camera
 * (the nr_set_view matrices), frame number and output image -- of the same size/shard
 * in as few launches as possible (up to 32 frames per launch).  The pixel queue runs
 * through the frames in order, so one frame's longest rays march while the next
 * frame's pixels keep the matrix cores busy: the throughput form of a sequence of
 * nr_render_shard calls, with identical pixels.  The network, precision, scene,
 * colouring and matcap are the context's.  `out` is a device or host pointer per `loc`;
 * stats are summed over the frames.  Schedules other than persistent, and the debug
 * flags 1 and 8, render frame by frame. */
typedef struct nr_frame {
    float inv_view[12];
    float normal[16];
    int frame;
    uint32_t *out;
} nr_frame;
int nr_render_batch(nr_ctx *ctx, const nr_frame *frames, int nframes, int W, int H, int band, int nshards,
                    int shard, int max_steps, int loc, nr_stats *stats);
int nr_shard_rows(int H, int band_rows, int nshards, int shard);
/* Frames per k_trace launch nr_render_batch uses for this shard: min(nframes, 32), further
 * capped so that every pixel-queue position of a launch, plus the positions its waves can
 * over-reserve, fits the 32-bit queue counters (queue_shards = nr_set_queue_shards' n).
 * Returns 0 when not even one frame fits (nr_render_batch then fails with NR_E_INVALID). */
int nr_batch_frames_per_launch(int W, int H, int band_rows, int nshards, int shard, int nframes, int queue_shards);
/* Re-interleave gathered shards (shard s's rows at src + s*stride_pixels) into a full
 * frame.  Host or device buffers (loc applies to both). */
int nr_assemble_shards(nr_ctx *ctx, const uint32_t *src, size_t stride_pixels,
                       uint32_t *dst, int W, int H, int band_rows, int nshards, int loc);

/* ---- multi-GPU, one process (main.cpp's render loop over the GPUs of a node) --------------
 * A group joins contexts on distinct GPUs (each created by nr_create on its device, with the
 * same network, precision, scene, colouring, matcap and schedule settings) with one RCCL
 * communicator (ncclCommInitAll).  nr_group_render_batch renders nframes frames across them:
 * context r renders row-band shard r of every frame (bands of `band` rows dealt round-robin,
 * the contexts in parallel, one host thread each), every shard's status is checked before any
 * transfer (a failed shard returns its error and starts no collective), ONE RCCL gather per call
 * (ncclSend / ncclRecv in one ncclGroupStart / ncclGroupEnd) brings the shards to the first
 * context's GPU, and one re-interleave launch per frame writes frames[i].out -- device pointers
 * on the first context's GPU (loc = NR_DEVICE) or host pointers (NR_HOST).  Pixels are
 * identical to nr_render on one GPU.  stats: summed over the shards (ms_total: the slowest). */
typedef struct nr_group nr_group;
int nr_group_create(nr_ctx *const *ctxs, int n, nr_group **out);
/* flags (round 5): NR_GROUP_COPY moves the shards with hipMemcpyPeerAsync instead of RCCL (the same
 * layout and re-interleave; contexts may then share a GPU -- how a one-GPU box runs multi-rank
 * groups); NR_GROUP_ASYNC returns once the call's gather and re-interleave are enqueued on the
 * group's communication streams, so the next call's render overlaps this call's transfer (shard
 * and gather buffers are double-buffered): frames[i].out of an NR_DEVICE call is complete after
 * nr_group_synchronize -- or, without the flag, when the call returns.  A call with host outputs
 * (loc != NR_DEVICE) always returns with its frames written.  Round 6: with NR_GROUP_ASYNC and
 * stats == NULL the renders are only enqueued too (the transfer streams wait for them device-side),
 * so the host submits call k + 1 while call k renders; a launch error still ends the call before
 * any transfer, a fault during the march is returned by the next call or nr_group_synchronize.
 * Asking for stats makes the call wait for its renders (the counters are read from the devices).
 * With NR_GROUP_COPY the contexts may sit on distinct GPUs as well. */
#define NR_GROUP_COPY 1
#define NR_GROUP_ASYNC 2
int nr_group_create_ex(nr_ctx *const *ctxs, int n, int flags, nr_group **out);
int nr_group_destroy(nr_group *group);
int nr_group_size(const nr_group *group);
int nr_group_render_batch(nr_group *group, const nr_frame *frames, int nframes, int W, int H, int band,
                          int max_steps, int loc, nr_stats *stats);
int nr_group_synchronize(nr_group *group);
/* The gather layout nr_group_render_batch uses: frame i's shard on every rank at i * shard_px
 * (shard_px = nr_shard_rows(H, band, n, 0) * W, the largest shard), rank r's shards at
 * r * per_rank of the gather buffer (per_rank = shard_px * nframes). */
int nr_group_layout(int W, int H, int band, int n, int nframes, size_t *shard_px, size_t *per_rank);

/* Replaces NeuralNetwork::forward(X) (neuralNetwork.cpp:54-63) on a batch:
 * X [n][dims[0]] fp32, Y [n][dims[nlayers]] fp32.  loc = NR_HOST or NR_DEVICE. */
int nr_mlp_forward(nr_ctx *ctx, const float *X, float *Y, long n, int loc);
/* One DenseLayer::forward (denseLayer.cu:229-278) on device buffers: layer l of the
 * loaded network applied to A [n][dims[l]] -> Z [n][dims[l+1]]. */
int nr_layer_forward(nr_ctx *ctx, int layer, const float *A, float *Z, long n, int loc);

/* Stateless dense layer on device (or host) buffers: Z = act(W A + b) per row of A,
 * W out-major [out][in] (DenseLayer's layout, denseLayer.cu:217-227), act = ReLU if
 * relu != 0 else linear.  Runs on ctx's stream (DenseLayer::forward objects that are
 * not part of a loaded network). */
int nr_dense_forward(nr_ctx *ctx, const float *W, const float *b, int in, int out, int relu,
                     const float *A, float *Z, long n, int loc);

/* ---- measurement ------------------------------------------------------------ */
/* Per-launch HIP events around every kernel of nr_render* on the context's stream
 * (the stream those kernels run on).  nr_prof_collect() waits for the stream, sums
 * the recorded durations since the previous collect and resets them. */
typedef struct nr_kernel_prof {
    double march_ms;         /* sum over k_march launches */
    double shade_ms;         /* sum over k_shade launches */
    double init_ms;          /* sum over k_init launches */
    uint64_t march_launches, shade_launches, init_launches;
    uint64_t renders;        /* nr_render* calls covered */
} nr_kernel_prof;
int nr_set_profiling(nr_ctx *ctx, int on);
int nr_prof_collect(nr_ctx *ctx, nr_kernel_prof *out);
/* The pixel contract per schedule (round 6): fp32 frames are identical on all three schedules, and
 * so are bf16 / fp16 frames on the persistent and wavefront schedules, endgame included (the
 * wavefront schedule runs it as a second, fp32x3 queue per iteration); the layered schedule renders
 * fp32 whatever the precision.  tests/test_gpu_endgame.py test_schedule_pixel_contract asserts this. */
int nr_set_schedule(nr_ctx *ctx, int schedule);
/* Diagnostics: flags bit 0 = per-wave s_memrealtime stamps in k_trace
 * {start, pixel queue drained, end (100 MHz), (wave iterations after the drain << 32) |
 * wave iterations, shader-clock cycles spent in refill, shading, MLP, scene, step, and within
 * refill (bf16/fp16 tracers) in the queue reservation, bulk ray generation and dealing; after
 * the queue drained: cycles in refill + shading + step, MLP, scene, iterations with at most
 * 4 rays}; the stamps instance marches bf16/fp16 without the endgame (the pure 16-bit march);
 * nr_debug_stamps copies the last
 * frame's (16 u64 per wave, *n = waves).  Bit 3 = iteration map: the persistent
 * schedule writes each hit pixel's iteration count instead of its colour.  Bit 6 =
 * MLP latency probe: nr_mlp_forward(X >= 64 points, Y >= 65 floats, n = repetitions, on
 * the device) runs one wave of ceil(wave_rays / 16) tiles n times back to back and
 * writes the shader cycles per evaluation to Y[0]; bit 7 times it without the final
 * layer; for fp32, bit 13 in the clamped-ReLU form the tracers run (scaled pack) and bit 14 with
 * the hidden layers unrolled for 7 (the network must have 7).  Bit 8 = NR_SCHED_LAYERED issues its launches one by one instead of replaying
 * the captured hipGraph (for profilers that do not follow graph launches).  Bit 9 = the plain ReLU
 * forms on the scaled packs: bf16 by v_pk_max_i16 instead of the conversion's clamp bit,
 * fp32 by add + max instead of v_add_f32 with the clamp bit (the same values: parity and
 * A/B of the two forms); fp32x3 by the fp32 MLP for every wave (its fallback, bit-exact fp32).  Bit 10 = nr_render_batch deals its pixel queue frame after
 * frame instead of interleaving the frames in 64-pixel chunks (pixels are unaffected).  Bit 11 = the
 * bf16/fp16 MLP of 7-hidden-layer networks in its builtin-compiled form instead of the
 * software-pipelined instruction streams (nr_mlp16_asm.h; the same values, for A/B and parity).
 * Bit 12 = nr_mlp_forward's bf16/fp16 MLP (k_mlp16, 7 hidden layers) with the hidden layers on
 * v_mfma_f32_16x16x32 instead of 32x32x16 (round 6; the same values; 3-5 % slower for bf16 and
 * 4-12 % for fp16, profiles/r6_mlp_s16_ab.txt, so it is an A/B form, not the default).
 * Bit 15 = the bf16/fp16 tracers' normals (the four tetrahedron
 * samples of every coloured ray) by the fp32 MLP instead of the fp32x3 split (A/B; the frames'
 * march is the same, their shading moves by the two forms' rounding). */
int nr_set_debug(nr_ctx *ctx, int flags);
/* The reduced-precision endgame (bf16 / fp16, round 5): a marching ray whose
 * 16-bit MLP output falls below tau (a surface is near) re-evaluates that point in fp32x3 and
 * takes every later step of its march in fp32x3, so the convergence test (tstep < 1e-6,
 * volumeRender_kernel.cu:474), the background test and the hit point are decided at fp32-class
 * precision while the bulk of the march stays 16-bit.  Default NR_ENDGAME_DEFAULT; 0 = the pure
 * 16-bit march.  It needs the network's fp32x3 pack (the 7-hidden-layer [3|4, 32..., 1] shape whose
 * scales fit, as for the fp32x3 normals) and is off with nr_set_debug bit 15 (fp32 normals); the
 * wavefront schedule applies it too (round 6: a fine queue per iteration, the same frames), the
 * layered schedule renders fp32.  nr_stats.endgame_evals counts the fp32x3
 * evaluations, nr_stats.endgame_switches the rays handed over.  The default (round 6, DESIGN.md
 * section 2): the threshold that meets the fixed quality targets of tests/test_gpu_lowp_contract.py
 * against the exact-MLP frame (C3 identical >= 0.77, C4 >= 0.88 with mean |delta| <= 5.0, coverage
 * IoU >= 0.99 / 0.98): 1e-3 (round 5's 3e-4 left C4's mean |delta| at 6.4). */
#define NR_ENDGAME_DEFAULT 0.001f
int nr_set_endgame(nr_ctx *ctx, float tau);
/* Temporal scheduling: each launch (a frame, or a batch's launch of up to 32 frames)
 * records its 8x8 pixel blocks' longest ray (the max over the batch's frames) and the next
 * launch of the same size/shard dispenses blocks longest-first (pixels are unaffected --
 * only the order work is handed out changes).  on = 2: each block's cost is the max over its
 * 3x3 neighbourhood (for a moving camera, whose silhouettes shift between frames). */
int nr_set_temporal_order(nr_ctx *ctx, int on);
/* Persistent-schedule grid: blocks of 4 waves per CU (0 = default).  A bf16/fp16 launch with the
 * endgame on runs one 12-wave workgroup per CU (3 blocks' worth, with the fp32x3 weights in its LDS;
 * networks of more than 9 hidden layers: at most 3 blocks of 4 waves), whatever is set here. */
int nr_set_occupancy(nr_ctx *ctx, int blocks_per_cu);
/* Rays per wave (persistent schedule, 1-64; 0 = automatic, the default): a wave marches at
 * most this many rays at once (in lanes 0..rays-1), so 16 or 32 make every iteration one or
 * two 16-ray tiles -- shorter per-iteration latency for small frames or shards, where the
 * longest ray rather than the matrix-core throughput sets the frame time.  Automatic: 64, or
 * 32 for an fp32 launch whose pixels fill at most 2x its waves' 64-ray slots (a frame on 4 or
 * 8 shards). */
int nr_set_wave_rays(nr_ctx *ctx, int rays);
/* Pixel-queue shards (persistent schedule; power of two <= 64, default 8): the queue's
 * atomic counters, each on its own 128-byte line, that the waves take pixels from. */
int nr_set_queue_shards(nr_ctx *ctx, int n);
/* NR_SCHED_LAYERED: points per dense-layer launch (the activations of one chunk are the
 * layer scratch: 2 x points x widest hidden layer x 4 B).  0 = auto (128 MiB per buffer).
 * The reference sizes Z for the whole batch, W*H*4 points (volumeRender_kernel.cu:659-661). */
int nr_set_layer_chunk(nr_ctx *ctx, long points);
/* Pixel spread (persistent schedule): the pixel queue deals each group of
 * `group_blocks` 8x8 blocks pixel-major -- one refill takes one pixel from each of up
 * to 64 blocks -- so the rays of one slow block are spread over many waves (0 =
 * block-major; -1 = automatic, the default: 16 for launches of fewer than 4 frames and
 * for fp32 batches of under 8 M pixels in all, 0 for the other nr_render_batch launches).
 * Pixels are unaffected. */
int nr_set_pixel_spread(nr_ctx *ctx, int group_blocks);
/* Cost probe (persistent schedule): before each frame, march the centre ray of every
 * 8x8 block for at most `max_steps` iterations (`rays_per_wave` rays per wave, so the
 * probe runs at short per-iteration latency), then hand the blocks out in decreasing
 * order of their probe's iteration count, so the frame's longest rays start first
 * (max_steps 0 = off; a valid temporal order takes precedence).  Pixels are unaffected. */
int nr_set_cost_probe(nr_ctx *ctx, int max_steps, int rays_per_wave);
int nr_debug_stamps(nr_ctx *ctx, unsigned long long *out, size_t cap, size_t *n);
/* Host polls the live-ray count every `every` iterations to stop early (0 = never). */
int nr_set_poll_interval(nr_ctx *ctx, int every);

/* ---- host helpers (the reference's main.cpp / image.cu side) -------------- */
/* updateViewMatrices (main.cpp:207-222): M = Rx(-rx deg) * Ry(-ry deg), then
 * translate(-(tx, ty, -zoom)); inv_view = rows 0..2 of M, normal = M^-1. */
int nr_camera(float rx_deg, float ry_deg, float zoom, float tx, float ty,
              float inv_view[12], float normal[16]);
/* The same with a choice of arithmetic.  NR_CAMERA_F64 (nr_camera's): the rotation and its
 * exact transpose-inverse in double, rounded once to float.  NR_CAMERA_EIGEN: main.cpp's float
 * Eigen expression restated step by step -- AngleAxisf * AngleAxisf as a quaternion product,
 * toRotationMatrix, Affine3f rotate/translate, Matrix4f::inverse by cofactors (Eigen 3.3's scalar
 * paths; Eigen is not available to pin it, and an SSE build inverts 4x4 floats differently). */
#define NR_CAMERA_F64 0
#define NR_CAMERA_EIGEN 1
int nr_camera_ex(float rx_deg, float ry_deg, float zoom, float tx, float ty, int mode,
                 float inv_view[12], float normal[16]);
/* Minimal HDF5 (superblock v0, symbol-table groups, contiguous datasets) Keras
 * reader.  Call with kernels/biases NULL to query sizes. */
int nr_h5_read_keras(const char *path, int max_layers, int *nlayers, int *dims,
                     float *params /* per layer: kernel (in x out) then bias, or NULL */,
                     size_t params_cap);
/* HDF5 object tree: the calls HighFive makes for NeuralNetwork::load (neuralNetwork.cpp:86-129)
 * and simpleInfer's loadModelFromH5 (simpleInfer.cpp:13-79) -- File(fp, ReadOnly),
 * listObjectNames, getObjectType, getGroup, getNumberObjects, getDataSet, getDimensions,
 * read -- over the same minimal reader; the headers in include/highfive/ wrap them in HighFive's
 * class names.  Objects are identified by their object-header addresses; group members
 * come in HDF5 name order (what HighFive's listObjectNames returns). */
typedef struct nr_h5_file nr_h5_file;
#define NR_H5_OTHER 0
#define NR_H5_GROUP 1
#define NR_H5_DATASET 2
int nr_h5_open(const char *path, nr_h5_file **out);
void nr_h5_close(nr_h5_file *f);
int nr_h5_root(const nr_h5_file *f, uint64_t *obj);
int nr_h5_object_type(nr_h5_file *f, uint64_t obj, int *type);
int nr_h5_num_members(nr_h5_file *f, uint64_t group, size_t *n);
/* member i of a group: name (NUL-terminated, cap bytes; NULL to query *name_len) and id */
int nr_h5_member(nr_h5_file *f, uint64_t group, size_t i, char *name, size_t cap, size_t *name_len,
                 uint64_t *obj);
/* dims may be NULL to query *ndims */
int nr_h5_dims(nr_h5_file *f, uint64_t dataset, uint64_t *dims, int cap, int *ndims);
/* all elements, row-major, converted to float; count must equal the element count */
int nr_h5_read_f32(nr_h5_file *f, uint64_t dataset, float *out, size_t count);
/* PNG decode to packed RGBA (image.cu:36-65 packing).  *rgba is malloc'ed; free
 * with nr_free(). */
int nr_png_load(const char *path, uint32_t **rgba, int *w, int *h);
/* Image::savePNG (image.cu:67-110): flip=1 reproduces the reference's 180 deg
 * rotation (quirk Q9). */
int nr_png_save(const char *path, const uint32_t *rgba, int w, int h, int flip);
/* sdkSavePPM4ub-style P6 (helper_image.h:310-328), buffer row 0 first. */
int nr_ppm_save(const char *path, const uint32_t *rgba, int w, int h);
void nr_free(void *p);

#ifdef __cplusplus
}
#endif
#endif /* NEURAL_RENDER_H */
