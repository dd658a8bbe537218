// nr_kernels.h -- kernel argument blocks and launchers (nr_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Workgroups per CU the persistent tracer's endgame instances (bf16/fp16 with nr_set_endgame) are
// built for: their registers (161 VGPRs) and the fine queue's LDS leave room for this many, so the
// host caps their grid at it (nr_api.hip trace_bpc; a larger grid would queue workgroups behind the
// resident ones)
#ifndef NR_TRACE_BPC_EG
#define NR_TRACE_BPC_EG 3
#endif
// Waves per workgroup of the endgame instances (round 6): 12 -- one workgroup per CU, the same 3
// waves per SIMD -- so that one LDS copy of the fp32x3 pack (~31 KB, read by the fine passes and
// the normals) fits beside the 16-bit pack and the 12 waves' queues; 4 = round 5's form (three
// 4-wave workgroups per CU, the fp32x3 weights read from global memory / L2)
#ifndef NR_EG_WAVES
#define NR_EG_WAVES 12
#endif
// LDS per CU on gfx950 (MI355X_MICROARCH.md): one workgroup's static + dynamic LDS must fit
constexpr int NR_LDS_PER_CU = 160 * 1024;

namespace nr {

// Network packs resident in device memory, staged into LDS by every block.
struct MlpArgs {
    const float *pk;        // fp32 pack (nr_internal.h PK_*; 32- or 16-wide layout)
    const uint16_t *lp;     // bf16/fp16 A operands (precision != fp32)
    const float *lpf;       // float side of the low-precision pack
    int pk_bytes, lp_bytes, lpf_bytes;
    int in0, nh;
    int lp_clamp;           // bf16 pack scaled for the clamped ReLU (nr_pack.cpp): valid for
                            // inputs within LP_INPUT_BOUND; the launch clears it otherwise
    int f32_clamp;          // fp32 pack scaled for the clamped ReLU (pack_fp32_16): used by the
                            // waves whose inputs are all within F32_INPUT_BOUND
    int lp_stream;          // 16-bit MLP as the pipelined streams of nr_mlp16_asm.h (7 hidden
                            // layers); 0 (nr_set_debug bit 11): the builtin form, same values
    const uint16_t *x3lp;   // bf16/fp16 tracers: the fp32x3 pack (global memory), for their normals
    const float *x3fl;
    int x3n;                // bf16/fp16: 1 = the normals (4 MLP evaluations per coloured ray) in fp32x3
                            // (mlp16_x3_normal), 0 = in fp32
    const uint16_t *lps;    // bf16/fp16, 7 hidden layers: the 16x16x32 layout of lp / lpf for k_mlp16
    const float *lpfs;      // (nr_pack.cpp pack_lowp_s16; null: not built, or nr_set_debug bit 12 clear)
    int lp_s16;             // k_mlp16 only (launch_mlp16): lp / lpf ARE the 16x16x32 layout, every
                            // chunk takes the NR_S16_* stream
};

// Per-render constants (the reference's __constant__ state, volumeRender_kernel.cu:31-35,
// passed by value so contexts are independent).
struct RenderArgs {
    uint32_t *out;          // this shard's rows, W per row
    int W, H, rows, band, nshards, shard;
    int max_steps, scene, frame, color_type;
    const uint32_t *matcap;
    int mw, mh;
    float inv_view[12];
    float normal[16];
    double inv_w, inv_band;  // 1/W, 1/band for udiv_r (set_recips)
    // 1/W, 1/H where W (H) is a power of two, else 0: initMarcher's (float)x / (float)W is then
    // (float)x * (1/W) exactly (a power-of-two divisor only shifts the exponent), which saves
    // ray generation two correctly rounded divisions (set_recips; pixel_uv)
    float rcp_w, rcp_h;
};
inline float pow2_rcp(int n) { return n > 0 && (n & (n - 1)) == 0 ? 1.0f / (float)n : 0.0f; }
inline void set_recips(RenderArgs &A) {
    A.inv_w = 1.0 / (double)A.W;
    A.inv_band = 1.0 / (double)A.band;
    A.rcp_w = pow2_rcp(A.W);
    A.rcp_h = pow2_rcp(A.H);
}

// Ray queues: live rays {p.xyz, tfar} + {d.xyz, pixel}; converged rays {p.xyz, -} + {d.xyz, pixel}.
struct QueueArgs {
    const uint32_t *cnt_in;
    uint32_t *cnt_out;
    const float4 *p_in, *d_in;
    float4 *p_out, *d_out;
    uint32_t *shade_cnt;
    float4 *shade_p, *shade_d;
    uint32_t *shade_it;     // per-iteration count of waves that enqueued converged rays
    long seg_cap;           // segmented queues (wavefront schedule): WF_SEGS segments of
                            // seg_cap entries, one counter each (cnt_*[s], shade_cnt[s])
    // the endgame on the wavefront schedule (round 6; bf16/fp16): the coarse pass appends the rays
    // whose 16-bit SDF falls below eg_tau, unstepped, to this iteration's fine queue (fcnt, fp, fd;
    // segmented like the live queue) and counts them in *fsw
    uint32_t *fcnt;
    float4 *fp, *fd;
    uint32_t *fsw;
    float eg_tau;
};
constexpr int WF_SEGS = 8;

// One dense layer over a chunk of points (k_dense; layered schedule and the generic
// nr_mlp_forward).  Z is chunk-local [chunk][out].
struct DenseArgs {
    const float *W, *b;        // out-major [out][in], bias [out]
    const float *A;            // SRC 0: chunk-local rows [chunk][in]
    float *Z;
    const float4 *pts;         // SRC 1: live-ray queue; SRC 2: converged-ray queue
    const uint32_t *count;     // device-side point count (x count_mul), or NULL: use n
    const RenderArgs *args;    // SRC 1/2: the frame number (4th input)
    long n, chunk0, chunk_n;
    int count_mul, in, out, relu, lds;
};

// Persistent-schedule state (nr_trace.hip).
// One frame of a batched launch (nr_render_batch): its camera, sphere-grid offset,
// animation input and output image.  Staged into LDS by k_trace<.., BATCH>.
struct FrameArgs {
    float inv_view[12];
    float normal[16];
    double zoff;        // sphere_zoff(frame)
    uint32_t *out;
    float frame_f;      // the network's 4th input when it takes one
    int frame;
};
constexpr int NR_MAX_BATCH = 32;


struct TraceArgs {
    uint32_t *pix_ctr;          // 2^nq_shift pixel-queue shard counters, one per 128-byte line (stride 32)
    int nq_shift;
    unsigned long long *stats;  // [0] ray-steps, [1] rays hit, [2] max iterations, [3] rays shaded,
                                // [4] fp32x3 march evaluations (the endgame)
    unsigned long long *stamps; // diagnostics (nr_set_debug): per wave {start, queue drained, end, ray-steps}
    // pixel queue over 8x8 pixel blocks of the shard image, dispensed in `order`
    // (NULL = raster order); bcost (may be NULL) receives each block's max ray iterations
    const uint32_t *order;
    uint32_t *bcost;
    int bw, nblocks;            // blocks per row, blocks in the shard image
    // pixel spread: the queue deals a group of 2^spread_shift blocks pixel-major (a refill
    // takes one pixel from each of 64 blocks), so a block of long rays is marched by 64
    // different waves instead of one (0/1 = block-major)
    int spread_shift;           // log2 of the spread group (0 = block-major)
    int itmap;                  // diagnostics: write each pixel's iteration count instead of its colour
    double inv_bw, inv_band;    // 1/bw, 1/band for udiv_r
    // cost probe (k_trace<.., true>): one ray per block
    int probe, take;
    uint64_t lane_cap;          // lanes a wave may fill: (1 << take) - 1, all 64 for take = 64
    const FrameArgs *frames;    // batched launch: nframes frames (k_trace<.., BATCH>)
    int nframes;
    int interleave;             // batched: 64-position queue chunks dealt to the frames in turn
                                // (all frames progress together) instead of frame-major
    double inv_nframes;         // 1 / nframes for udiv_r
    float eg_tau;               // bf16/fp16 with an fp32x3 pack: the endgame's switch threshold (0 = off;
                                // k_trace's EG instances, nr_set_endgame)
    int x3lp_bytes, x3fl_bytes; // sizes of the fp32x3 pack (16-byte multiples): the endgame
                                // instances stage it in LDS beside the 16-bit pack (NR_EG_WAVES)
};

int dense_lds_bytes(int in, int out);
hipError_t launch_dense(const DenseArgs &D, int src, int grid, hipStream_t st);
hipError_t launch_init_f(const RenderArgs &A, const FrameArgs *F, const QueueArgs &Q, long npix, long total,
                         int grid, hipStream_t st);
hipError_t launch_march16(const RenderArgs &A, const MlpArgs &M, const QueueArgs &Q, const FrameArgs *F, int prec,
                          int it, int grid, hipStream_t st, int mode = 0);
hipError_t launch_shade16(const RenderArgs &A, const MlpArgs &M, const QueueArgs &Q, const FrameArgs *F, int grid,
                          hipStream_t st);
hipError_t launch_set_args(const RenderArgs &A, RenderArgs *d, hipStream_t st);
hipError_t launch_init_l(const RenderArgs *Ad, const QueueArgs &Q, long npix, hipStream_t st);
hipError_t launch_march_l(const RenderArgs *Ad, const QueueArgs &Q, const float *sdf, int it, int grid, hipStream_t st);
hipError_t launch_shade_l(const RenderArgs *Ad, const QueueArgs &Q, const float *sdf4, int grid, hipStream_t st);
hipError_t launch_trace(const RenderArgs &A, const MlpArgs &M, const TraceArgs &T, int prec, int grid, hipStream_t st);
hipError_t launch_mlp16(const MlpArgs &M, int prec, const float *X, float *Y, long n, int grid, hipStream_t st);
hipError_t launch_mlp_latency(const MlpArgs &M, int prec, const float *X, float *Y, int reps, int nt, int part,
                              hipStream_t st);
hipError_t launch_order(const uint32_t *bcost, uint32_t *order, int nblocks, int bw, int dilate, hipStream_t st);
hipError_t launch_assemble(const uint32_t *src, size_t stride, uint32_t *dst, int W, int H, int band, int nshards,
                           hipStream_t st);

}  // namespace nr
