// nr_trace.hip -- persistent sphere tracer: one launch marches every ray of the frame.
//
// Replaces the reference's host loop (volumeRender_kernel.cu:652-689: per iteration
// 9 GEMM launches + singleMarch + a full-image thrust scan + a blocking 4-byte D2H)
// with a single persistent launch:
//   * every wave owns 64 ray slots (ray state in registers, point p in lane p);
//   * free slots are refilled from a pixel queue sharded 8 ways (one counter per
//     shard, each on its own cache line; a wave starts on shard blockIdx % 8 and moves
//     on when it is drained) -- the ray is generated in-lane (initMarcher :293-358);
//   * each wave iteration runs the MLP on the live points (nr_mlp16.h, 16-point MFMA
//     tiles, weights in LDS), then one sphere-trace step per ray (singleMarch :416-477);
//     each ray counts its own iterations, so the reference's global iteration cap
//     (MAX_STEPS / the configs' 64-256) holds per ray, bit for bit;
//   * once the queue is drained the live rays are compacted into the lowest tiles, so
//     the tail costs ceil(live/16) tiles per iteration instead of a full wave;
//   * converged rays go to a per-wave LDS stash; whenever 16 are stashed (or the queue
//     is drained) the wave evaluates their 4 tetrahedral samples as one full 4-tile MLP
//     pass (surfaceNormal :361-377, always fp32) and colours them (:380-413) -- so the
//     normal work fills the tail of the frame instead of a separate launch.
#include "nr_mlp16.h"

#include <cstddef>

namespace nr {

// workgroups per CU the register allocation of k_trace targets (4 waves each)
#ifndef NR_TRACE_BPC
#define NR_TRACE_BPC 3
#endif
// the batched fp32 instance and the reduced-precision ones: 4 workgroups per CU (<= 128 VGPRs,
// a few values spilled outside the MLP) -- fp32 launches of >= 8 M pixels run 4 (1024^2 x 20
// frames 1.795 -> 1.772 ms/frame), bf16 launches too (0.416 -> 0.408 ms/frame, C3 batch 1.660 ->
// 1.632; profiles/r2_f32_batch_bounds.txt, r2_lowp_bpc4.txt)
#ifndef NR_TRACE_BPC_WIDE
#define NR_TRACE_BPC_WIDE 4
#endif
// the bf16/fp16 instances (A/B knobs: workgroups per CU their registers are allocated for, the
// bulk-generation ring, rays per shading pass)
#ifndef NR_TRACE_BPC_LOWP
#define NR_TRACE_BPC_LOWP NR_TRACE_BPC_WIDE
#endif
constexpr int NR_RING_LOWP = 64;
constexpr int NR_SHADE_RAYS_LOWP = 16;
// the bulk-generating tracers keep each marching ray's direction and pixel in LDS (one float4
// per lane, read back by the step) instead of four VGPRs live across the MLP
constexpr int NR_RAY_D_LDS = 1;

// Issue priority of a wave outside its MLP (scene, step, refill, shading).  A wave there
// issues VALU in the shadows of the other waves' MFMAs instead of waiting behind them
// (issue arbitration is priority, then age), so it is back in its MLP sooner and the
// matrix pipe idles less: fp32 batch 2.050 -> 2.012 ms/frame (prio 1/2/3: 2.018/2.016/
// 2.012; profiles/r1_ab_experiments.txt).  0 = off.  fp32 only (bf16: +1%).
constexpr int NR_NONMLP_PRIO = 3;

// bf16/fp16: issue priority NR_MLP_PRIO_LOWP inside the march MLP (the age-ordered arbitration
// otherwise lets an older wave's scene/refill VALU cut into a younger wave's MFMA chain), 0
// elsewhere.  Alternating A/B (tools/ab_trace_rounds.sh, profiles/r4_ab_prio.txt): march 2 -> C3
// batch 1.370 / 1.389 vs 1.379 / 1.405 ms, C5 1.410 / 1.417 vs 1.437 / 1.421; a priority in the
// shading pass, either alone or with it, and 3 workgroups per CU were no better
constexpr int NR_MLP_PRIO_LOWP = 2;


// Wave-private pools of pixel-queue positions reserved one atomic ahead (bf16/fp16
// tracers only: their iterations are short, so the ~1 us reservation latency is a large
// part of the refill; the fp32 tracer's MLP hides it and the pools only lengthen the
// tail -- tools/ab_multi.sh, profiles/r1_ab_experiments.txt).
constexpr int NR_QUEUE_PREFETCH_LOWP = 1;
constexpr int NR_QUEUE_PREFETCH_FP32 = 0;
constexpr int NR_QUEUE_CHUNK = 32;
constexpr int NR_QUEUE_LOW = 8;

constexpr int NR_DENSE_GEN = 1;
// Bulk generation's queue reservations (round 3): up to two ranges per generation (what is
// left of the wave's pool + the pending reservation), chunks of NR_QUEUE_CHUNK_DENSE positions
// requested whenever the pool holds fewer than that -- launches of >= 4 frames; launches of
// fewer take chunks of NR_QUEUE_CHUNK_DENSE1, since positions a wave holds ahead lengthen a
// single frame's tail (tools/ab_lowp.sh, profiles/r3_ab_experiments.txt (17)).
constexpr int NR_QUEUE_TWO_RANGES = 1;
constexpr int NR_QUEUE_CHUNK_DENSE = 64;
constexpr int NR_QUEUE_CHUNK_DENSE1 = 32;
// (fp32: A/B only -- its ring would cost the batched instance its fourth workgroup per CU)
constexpr int NR_DENSE_GEN_FP32 = 0;

// Refill only once this many ray slots are free (or the wave is empty), so that the ray
// generation and the queue bookkeeping are paid for several rays at a time: bf16 batch
// 0.611 -> 0.571 ms/frame at 8 (4: 0.589, 16: 0.575), fp32 1.978 -> 1.964 at 4
// (profiles/r1_ab_experiments.txt).
constexpr int NR_REFILL_MIN_LOWP = 8;
constexpr int NR_REFILL_MIN_FP32 = 4;

typedef __attribute__((address_space(1))) uint32_t *gptr_u32;

// Phase markers for tools/phase_isa.py (a -DNR_PHASE_MARKS=1 assembly listing only): an assembler
// comment at each phase boundary of k_trace's loop, so the listing can be cut into refill /
// shading / fine / compaction / MLP / scene / step and the instructions of each counted.
#ifndef NR_PHASE_MARKS
#define NR_PHASE_MARKS 0
#endif
#if NR_PHASE_MARKS
#define NR_PHASE(name) asm volatile("; NRPHASE " #name)
#else
#define NR_PHASE(name) ((void)0)
#endif

constexpr int STASH = 80;  // converged rays waiting for colour, per wave (<= 15 + 64)
// the A/B knobs' bounds: a shading pass leaves at most SHR - 1 stashed rays, and one
// iteration adds at most 64; the generated-ray ring is indexed with & (RB - 1)
static_assert(16 - 1 + 64 <= STASH && NR_SHADE_RAYS_LOWP - 1 + 64 <= STASH && NR_SHADE_RAYS_LOWP >= 1,
              "NR_SHADE_RAYS_LOWP overflows the per-wave LDS stash");
static_assert((NR_RING_LOWP & (NR_RING_LOWP - 1)) == 0 && NR_RING_LOWP >= 16 && NR_RING_LOWP <= 64,
              "NR_RING_LOWP must be a power of two in [16, 64]");


// Image row of local row lr of the shard (rows are dealt in bands of A.band).
__device__ __forceinline__ int shard_row(const RenderArgs &A, const TraceArgs &T, int lr) {
    if (A.nshards <= 1) return lr;
    const int bi = (int)udiv_r((uint32_t)lr, (uint32_t)A.band, T.inv_band);
    return (bi * A.nshards + A.shard) * A.band + (lr - bi * A.band);
}

// The ray direction of pixel x of local row lr (initMarcher :293-358).
__device__ __forceinline__ F3 ray_dir(const RenderArgs &A, const TraceArgs &T, const float *M, int x, int lr) {
    const int y = shard_row(A, T, lr);
    float u = pixel_uv(x, A.W, A.rcp_w);
    float v = pixel_uv(y, A.H, A.rcp_h);
    F3 dd = normalize3(mk3(u, v, -2.0f));
    return mk3(dot3(dd, mk3(M[0], M[1], M[2])), dot3(dd, mk3(M[4], M[5], M[6])), dot3(dd, mk3(M[8], M[9], M[10])));
}

// Ray generation for pixel x of local row lr of the shard (initMarcher :293-358).
// Returns hit.
__device__ __forceinline__ bool gen_ray(const RenderArgs &A, const TraceArgs &T, const float *M, int x, int lr,
                                        F3 &p, F3 &d, float &tfar) {
    F3 o = mk3(dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 0), dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 4),
               dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 8));
    const F3 dd = ray_dir(A, T, M, x, lr);
    float tnear;
    if (!intersect_bounding(o, dd, tnear, tfar)) return false;
    if (tnear < 0.0f) tnear = 0.0f;
    p = add3(o, mul3s(dd, tnear));
    d = dd;
    return true;
}

// The per-frame values a batched k_trace keeps in LDS (FrameArgs minus the normal matrix,
// which only the colouring reads, from global memory): 72 of 136 bytes per frame.
struct FrameLds {
    float inv_view[12];
    double zoff;
    uint32_t *out;
    float frame_f;
    int pad;
};
static_assert(sizeof(FrameLds) == 72 && offsetof(FrameLds, zoff) == 48 && offsetof(FrameLds, frame_f) == 64,
              "FrameLds layout (staged word by word in k_trace)");
static_assert(offsetof(FrameArgs, zoff) == 112 && offsetof(FrameArgs, out) == 120 && offsetof(FrameArgs, frame_f) == 128,
              "FrameArgs layout (staged word by word in k_trace)");

// The atomic add of lane 0 on pixel-queue shard sh (its counter on a 128-byte line), issued by every
// lane -- lanes 1-63 at an offset past the counters, dropped by the buffer's range check -- so that no
// lane-divergent branch surrounds it: around `if (lane == 0) v = atomicAdd(..)` hipcc waited for
// the return at the branch's join, which made the reservation requested one refill ahead
// (NR_QUEUE_PREFETCH) a full round trip to memory at every request.  Returns lane 0's old value
// (read it with readfirstlane where it is needed).
__device__ __forceinline__ uint32_t queue_add(const __amdgpu_buffer_rsrc_t rq, int lane, int sh, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32((int)v, rq, lane == 0 ? sh * 128 : 0x7fffff00, 0, 0);
}

// s_setprio takes an immediate
__device__ __forceinline__ void set_priority(int prio) {
    switch (prio) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// k_trace's arguments re-read from the kernarg segment (scalar loads) where a phase uses them,
// instead of being held in SGPRs -- or spilled to VGPR lanes, one v_readlane per use -- across the
// whole loop.  The pointer is made opaque per use, so the loads cannot be
// hoisted out of the loop.  The struct mirrors the kernarg layout of k_trace(A, M, T): each
// argument at its natural alignment, in order (the code object metadata, llvm-readelf --notes:
// by_value arguments at offsets 0, 200 and 304; tests/test_lib_cpu.py
// test_trace_kernarg_layout_matches_trace_kargs checks every instance of the built library, and every
// GPU parity test reads through it).  (Taking the parameters' addresses instead makes the compiler
// copy them to scratch: 368 bytes per lane.)
// (SGPRs spilled to VGPR lanes: the bf16 batched tracer with fp32x3 normals 124 -> 59, its endgame
// instance 151 -> 51, the fp32 batched tracer 85 -> 8.)
#ifndef NR_ARG_RELOAD
#define NR_ARG_RELOAD 1
#endif
struct TraceKargs {
    RenderArgs A;
    MlpArgs M;
    TraceArgs T;
};
__device__ __forceinline__ const TraceKargs *fresh_kargs() {
    auto p = (const __attribute__((address_space(4))) TraceKargs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return (const TraceKargs *)p;
}

// The shading pass's fp32x3 normals as two one-tile passes (1, round 4: fewer live registers at the
// shading site) or one two-tile pass (0; A/B); _EG: in the endgame instances, whose 150+ VGPRs hold
// the two-tile pass without spilling: 1-2 % faster batched (round 6, profiles/r6_x3n_eg_ab.txt)
#ifndef NR_X3N_ONE
#define NR_X3N_ONE 1
#endif
#ifndef NR_X3N_ONE_EG
#define NR_X3N_ONE_EG 0
#endif

// PROBE: the cost-probe pre-pass (TraceArgs::probe) -- one ray per 8x8 block, at most
// T.take rays per wave, no pixels written; each block's bcost gets its probe ray's
// iteration count (max_steps is the probe's cap).
// STAMPS: the diagnostic build (nr_set_debug bit 0) -- per-wave s_memrealtime stamps
// and per-phase shader-clock counters; a separate instance so that the counters cost
// the production kernel no registers.
// BATCH: T.nframes frames in one launch (nr_render_batch).  The pixel queue runs through
// the frames one after another, so one frame's longest rays march while the next
// frame's pixels fill the freed slots; every ray carries its frame index (rf) and the
// frame-dependent values (camera, sphere offset, animation input, output image) come
// from the FrameArgs staged in LDS.
// fp32x3: its MLP holds the hi and residual operands of two tiles besides the accumulators;
// 3 workgroups per CU (<= 168 VGPRs) keep it out of scratch
#ifndef NR_TRACE_BPC_X3
#define NR_TRACE_BPC_X3 3
#endif
// NX3: the bf16/fp16 instances whose normals are fp32x3 (MlpArgs::x3n; mlp16_x3_normal).
// EG: the bf16/fp16 instances with the fp32x3 endgame (TraceArgs::eg_tau > 0, round 5): a marching
// ray whose 16-bit MLP output falls below eg_tau leaves its lane for the wave's fine queue in LDS
// without taking the step; whenever the queue holds a full 32-point tile (or the pixel queue is
// drained) the wave takes up to 64 queued rays through a fine pass -- the fp32x3 MLP on their
// points (mlp16_x3_normal's per-point rule: the split within the x3 pack's bounds, the fp32 MLP
// outside), the scene and singleMarch's step -- and returns the survivors to the queue.  So the
// switch iteration's step, the convergence test (:474), the background test and every later step
// of the ray are decided in fp32x3, on full tiles.  Oracle: nr_oracle.c or_set_endgame.
// (3 workgroups per CU: the fine pass's registers -- 161 VGPRs; at 4 per CU, <= 128 VGPRs, the
// spills cost C3 +25 %, C5 +40-55 %; a pass per 64 queued rays instead of 32: C5 batch +5-10 %;
// profiles/r5_ab_eg.txt)
// (NR_TRACE_BPC_EG: nr_kernels.h, where the host side caps the grid with it)
// EGL (EG only): the NR_EG_WAVES-wave workgroup with the fp32x3 pack in LDS; false = 4-wave
// workgroups reading it from global memory, for networks whose two packs do not fit the CU's LDS
// beside the 12 waves' queues (more than 9 hidden layers; launch_trace_k chooses)
template <int PREC, bool PROBE, bool STAMPS = false, bool BATCH = false, bool NX3 = false, bool EG = false,
          bool EGL = true>
__global__ __launch_bounds__(EG && EGL ? 64 * NR_EG_WAVES : 256, EG ? NR_TRACE_BPC_EG
                                  : PREC == NR_PRECISION_FP32X3 ? NR_TRACE_BPC_X3
                                  : PREC != NR_PRECISION_FP32 ? NR_TRACE_BPC_LOWP
                                  : BATCH ? NR_TRACE_BPC_WIDE : NR_TRACE_BPC) void k_trace(RenderArgs A, MlpArgs M, TraceArgs T) {
    constexpr int prec = PREC;
    constexpr bool QPF = PREC == NR_PRECISION_FP32 ? NR_QUEUE_PREFETCH_FP32 : NR_QUEUE_PREFETCH_LOWP;  // queue pools
    constexpr int NONMLP_PRIO = PREC == NR_PRECISION_FP32 ? NR_NONMLP_PRIO : 0;
    constexpr int MLP_PRIO = PREC == NR_PRECISION_BF16 || PREC == NR_PRECISION_FP16 ? NR_MLP_PRIO_LOWP : 0;
    constexpr int RMIN = PREC == NR_PRECISION_FP32 ? NR_REFILL_MIN_FP32 : NR_REFILL_MIN_LOWP;  // free slots per refill
    // rays generated in bulk through an LDS buffer (NR_DENSE_GEN): the reduced-precision tracers
    constexpr bool DENSE = NR_DENSE_GEN && (PREC != NR_PRECISION_FP32 || NR_DENSE_GEN_FP32) && !PROBE;
    constexpr bool TWO = DENSE && NR_QUEUE_TWO_RANGES;
    // pool size; the next reservation is requested when the pool holds fewer than QLOW
    const uint32_t QCHUNK = TWO ? (BATCH && T.nframes >= 4 ? NR_QUEUE_CHUNK_DENSE : NR_QUEUE_CHUNK_DENSE1) : NR_QUEUE_CHUNK;
    const uint32_t QLOW = TWO ? QCHUNK : NR_QUEUE_LOW;
    __shared__ FrameLds sf[BATCH ? NR_MAX_BATCH : 1];
    if constexpr (BATCH) {
        for (int i = threadIdx.x; i < T.nframes * 18; i += blockDim.x) {  // 18 words per FrameLds
            const int f = i / 18, w = i - 18 * f;
            const uint32_t *src = reinterpret_cast<const uint32_t *>(T.frames + f);
            // inv_view [0, 12), zoff + out [28, 32) -> [12, 16), frame_f [32] -> 16
            reinterpret_cast<uint32_t *>(sf + f)[w] = w < 12 ? src[w] : (w < 16 ? src[16 + w] : (w == 16 ? src[32] : 0u));
        }
    }
    // waves per workgroup: 4, or NR_EG_WAVES for the endgame instances, which then hold the fp32x3
    // pack in LDS (X3L) for their fine passes and normals
    constexpr int NW = EG && EGL ? NR_EG_WAVES : 4;
    constexpr bool X3L = EG && EGL && NR_EG_WAVES > 4;
    const uint16_t *x3l = M.x3lp;
    const float *x3f = M.x3fl;
    if constexpr (X3L) stage_x3<PREC>(M, T.x3lp_bytes, T.x3fl_bytes, x3l, x3f);
    Smem16 S = stage16<PREC, true>(M);  // (its __syncthreads also covers sf and the fp32x3 copy)
    // converged rays per wave: {p.xyz, pixel} and the frame (the direction is regenerated from
    // the pixel for facingColor; matCapColor does not read it): 21 instead of 42 KB per CU,
    // so that 4 fp32 workgroups share a CU
    __shared__ float4 stash[NW][STASH];
    __shared__ uint8_t stash_f[NW][BATCH ? STASH : 1];
    // DENSE: per wave a ring of RB generated rays {p.xyz, tfar}, {d.xyz, pixel} (+ frame), as two
    // arrays of 16-byte entries so that consecutive lanes' ds_write_b128 / ds_read_b128 stay
    // conflict-free: 64 rays, 8.25 KB per workgroup (the fp32 tracer's ring, an A/B build option,
    // holds 16: its 4 workgroups per CU have 2 KB of LDS left each)
    constexpr int RB = PREC == NR_PRECISION_FP32 ? 16 : NR_RING_LOWP;
    __shared__ float4 rbuf_p[DENSE ? NW : 1][DENSE ? RB : 1], rbuf_d[DENSE ? NW : 1][DENSE ? RB : 1];
    __shared__ uint8_t rbuf_f[DENSE && BATCH ? NW : 1][DENSE && BATCH ? RB : 1];
    // each lane's marching ray {d.xyz, pixel} (DLDS): 4 KB per workgroup
    constexpr bool DLDS = DENSE && NR_RAY_D_LDS;
    __shared__ float4 ray_dp[DLDS ? NW : 1][DLDS ? 64 : 1];
    // EG: per wave the fine queue {p.xyz, tfar}, {d.xyz, pixel}, iteration | frame << 24: a pass
    // leaves fewer than 32 rays (or none), one iteration adds at most 64
    static_assert(!EG || (DLDS && NX3 && (PREC == NR_PRECISION_BF16 || PREC == NR_PRECISION_FP16)), "EG instances");
    constexpr int FQ = EG ? 32 - 1 + 64 : 1;
    __shared__ float4 fq_p[EG ? NW : 1][FQ], fq_d[EG ? NW : 1][FQ];
    __shared__ uint32_t fq_i[EG ? NW : 1][FQ];
    int nfq = 0;        // rays in the wave's fine queue (EG)
    uint32_t nfine = 0;  // fp32x3 march evaluations (EG)
    uint32_t nswitch = 0;  // rays handed to the fine queue (EG; wave-uniform)
    const int lane = lane_id();
    const int wid = threadIdx.x >> 6;
    const long nchunks = T.nblocks;
    const auto rq = __builtin_amdgcn_make_buffer_rsrc(T.pix_ctr, 0, 128 << T.nq_shift, 0x00020000);  // the shard counters
    const float fr = (float)A.frame;
    const double zoff0 = sphere_zoff(A.frame);
    // frame-dependent values of frame f (single-frame launches: the uniform ones in A)
    // the output image of frame f as a global-address-space pointer: a batched frame's
    // pointer comes from the LDS FrameArgs, and as a generic pointer its stores would be
    // flat_store (counted on both vmcnt and lgkmcnt) instead of global_store
    auto out_of = [&](int f) -> gptr_u32 { return (gptr_u32)(BATCH ? sf[f].out : A.out); };
    auto zoff_of = [&](int f) -> double { return BATCH ? sf[f].zoff : zoff0; };
    auto fr_of = [&](int f) -> float { return BATCH ? (M.in0 == 4 ? sf[f].frame_f : 0.0f) : fr; };
    auto put = [&](int f, uint32_t i, uint32_t v) { out_of(f)[i] = v; };
    const int q4 = lane & 3;
    int nstash = 0;
    const int nq = 1 << T.nq_shift;  // pixel-queue shards
    // a 12-wave endgame workgroup spreads its waves over 3 shards, as three 4-wave ones did
    int shard = (NW > 4 ? (int)(blockIdx.x * (NW / 4) + (threadIdx.x >> 8)) : (int)blockIdx.x) & (nq - 1), tries = 0;
    bool qempty = false;
    uint32_t pool_base = 0, pool_cnt = 0, pend_v = 0;  // NR_QUEUE_PREFETCH state
    bool pend = false;
    uint32_t rb_n = 0, rb_head = 0;  // DENSE: rays in the wave's buffer, ring position of the first
    F3 p = mk3(0, 0, 0), d = mk3(0, 0, 0);
    float tfar = 0.0f;
    uint32_t pix = 0;
    int rf = 0;  // the ray's frame (BATCH)
    int it = -1, maxit = 0;  // it: iterations of the slot's ray; -1: no ray (an int, not a
                             // bool, so that the compiler keeps it in a VGPR, not a lane mask)
    // per-wave statistics in 32 bits (fewer scalar registers to spill): a wave's rays hit and shaded
    // are at most its share of the launch's < 2^32 queue positions; its ray-steps can exceed that
    // (x max_steps), so they are flushed to the launch's counter past 2^30
    uint32_t nsteps = 0, nhit = 0, nconv = 0;
    uint32_t wit = 0, wit_tail = 0;  // wave iterations, those after the queue drained (stamps)
    // stamps: cycles in refill, shading, MLP, scene, step; and within refill: queue reservation,
    // bulk ray generation, dealing from the ring
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tph = 0;
    // after the queue drained: cycles in refill + shading + step, MLP, scene; iterations with <= 4 rays
    unsigned long long pt[4] = {0, 0, 0, 0};
    constexpr bool timing = STAMPS;
    const long gwave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned long long t_start = STAMPS ? __builtin_amdgcn_s_memrealtime() : 0ull, t_empty = 0ull;
    int nl_drain = -1;  // stamps: live rays at the first iteration after the drain
    while (true) {
        if constexpr (timing) tph = __builtin_amdgcn_s_memtime();
        // The loop's control state is wave-uniform (the whole wave is active here);
        // readfirstlane lets the compiler keep it in SGPRs and branch on it as such.
        nstash = __builtin_amdgcn_readfirstlane(nstash);
        qempty = __builtin_amdgcn_readfirstlane((int)qempty) != 0;
        shard = __builtin_amdgcn_readfirstlane(shard);
        tries = __builtin_amdgcn_readfirstlane(tries);
        pool_base = (uint32_t)__builtin_amdgcn_readfirstlane((int)pool_base);
        pool_cnt = (uint32_t)__builtin_amdgcn_readfirstlane((int)pool_cnt);
        pend = __builtin_amdgcn_readfirstlane((int)pend) != 0;
        rb_n = (uint32_t)__builtin_amdgcn_readfirstlane((int)rb_n);
        rb_head = (uint32_t)__builtin_amdgcn_readfirstlane((int)rb_head);
        if constexpr (EG) nfq = __builtin_amdgcn_readfirstlane(nfq);
        NR_PHASE(refill);
        // ---- refill free slots from the pixel queue
        if (!qempty || (DENSE && rb_n > 0)) {
#if NR_ARG_RELOAD
            const TraceKargs *K = fresh_kargs();
            const RenderArgs &A = K->A;
            const TraceArgs &T = K->T;
            // (and the queue constants derived from them, formed here instead of held)
            const uint32_t QCHUNK = TWO ? (BATCH && T.nframes >= 4 ? NR_QUEUE_CHUNK_DENSE : NR_QUEUE_CHUNK_DENSE1) : NR_QUEUE_CHUNK;
            const uint32_t QLOW = TWO ? QCHUNK : NR_QUEUE_LOW;
            const long nchunks = T.nblocks;
            const auto rq = __builtin_amdgcn_make_buffer_rsrc(T.pix_ctr, 0, 128 << T.nq_shift, 0x00020000);
            const int nq = 1 << T.nq_shift;
#endif
            // rays live in lanes [0, take): a wave capped at 16 or 32 rays marches 1 or
            // 2 tiles per iteration (short iterations when a frame shard is small)
            const uint64_t freem = __ballot(it < 0) & T.lane_cap;
            const uint32_t nfree = (uint32_t)__popcll(freem);
            // (a drained queue's buffered rays are dealt at once: they are the frame's last)
            if (nfree >= (uint32_t)RMIN || (nfree && nfree == (uint32_t)T.take) || (DENSE && qempty && nfree)) {
                auto shard_total = [&](int sh) -> long {
                    const long sh_chunks = sh < nchunks ? ((nchunks - 1 - sh) >> T.nq_shift) + 1 : 0;
                    return (PROBE ? sh_chunks : sh_chunks * 64) * (BATCH ? T.nframes : 1);
                };
                // Up to `want` positions of the queue -> [base, base + got).  Queue positions are
                // broadcast with readfirstlane (the whole wave is active here), not __shfl, so
                // that the compiler sees them as uniform and keeps the queue logic in scalar
                // branches instead of lane-mask control flow.
                auto reserve = [&](uint32_t want, uint32_t &base, uint32_t &got) {
                    got = 0;
                    if constexpr (QPF) {
                        // Positions come from a wave-private pool of reserved queue positions;
                        // the next reservation is requested (one atomic, not waited for) when the
                        // pool runs low and absorbed when it is empty, so its ~1 us return
                        // latency overlaps the MLP instead of stalling the refill.
                        if (pool_cnt == 0) {
                            if (pend) {
                                const uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend_v);
                                pend = false;
                                const long tot = shard_total(shard);
                                if ((long)b < tot) {
                                    pool_base = b;
                                    pool_cnt = (uint32_t)min((long)QCHUNK, tot - (long)b);
                                }
                            }
                            while (pool_cnt == 0) {  // nothing reserved: a blocking reservation
                                const long tot = shard_total(shard);
                                const uint32_t w = max(want, (uint32_t)QCHUNK);
                                const uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)queue_add(rq, lane, shard, w));
                                if ((long)b < tot) {
                                    pool_base = b;
                                    pool_cnt = (uint32_t)min((long)w, tot - (long)b);
                                    break;
                                }
                                shard = (shard + 1) & (nq - 1);
                                if (++tries >= nq) {
                                    qempty = true;
                                    if (STAMPS) t_empty = __builtin_amdgcn_s_memrealtime();
                                    break;
                                }
                            }
                        }
                        if (pool_cnt) {
                            base = pool_base;
                            got = min(want, pool_cnt);
                            pool_base += got;
                            pool_cnt -= got;
                        }
                        if (!qempty && !pend && pool_cnt < QLOW) {
                            pend_v = queue_add(rq, lane, shard, (uint32_t)QCHUNK);
                            pend = true;
                        }
                    } else {
                        while (true) {
                            const long total = shard_total(shard);
                            base = (uint32_t)__builtin_amdgcn_readfirstlane((int)queue_add(rq, lane, shard, want));
                            if ((long)base < total) {
                                got = (uint32_t)min((long)want, total - (long)base);
                                break;
                            }
                            shard = (shard + 1) & (nq - 1);
                            if (++tries >= nq) {
                                qempty = true;
                                if (STAMPS) t_empty = __builtin_amdgcn_s_memrealtime();
                                break;
                            }
                        }
                    }
                };
                // The frame f and pixel (px, py) of queue position q; false outside the image.
                auto pixel_of = [&](uint32_t q, int &f, int &px, int &py) -> bool {
                    f = 0;
                    if constexpr (BATCH) {
                        if (T.interleave) {  // 64-position chunk c goes to frame c % n
                            const uint32_t c = q >> 6, cq = udiv_r(c, (uint32_t)T.nframes, T.inv_nframes);
                            f = (int)(c - cq * (uint32_t)T.nframes);
                            q = (cq << 6) | (q & 63u);
                        } else {  // frame-major: frame f owns [f * per, (f + 1) * per)
                            const uint32_t per = (uint32_t)((((nchunks - 1 - shard) >> T.nq_shift) + 1) * 64);
                            f = (int)udiv_r(q, per, 1.0 / (double)per);
                            q -= (uint32_t)f * per;
                        }
                    }
                    uint32_t bq = q >> 6, pq = q & 63;
                    if (PROBE) {
                        bq = q;
                        pq = 4 * 8 + 4;  // the block's centre pixel
                    } else if (T.spread_shift) {
                        const int sh = T.spread_shift;
                        const uint32_t G = 1u << sh;
                        const uint32_t sh_chunks = (uint32_t)(((nchunks - 1 - shard) >> T.nq_shift) + 1);
                        const uint32_t g = q >> (6 + sh), r = q & ((64u << sh) - 1u);
                        const uint32_t nbg = min(G, sh_chunks - g * G);
                        pq = nbg == G ? r >> sh : r / nbg;  // a short group only at the end
                        bq = g * G + (r - pq * nbg);
                    }
                    const long pos = ((long)bq << T.nq_shift) + shard;
                    const int blk = T.order ? (int)T.order[pos] : (int)pos;
                    const int by = (int)udiv_r((uint32_t)blk, (uint32_t)T.bw, T.inv_bw), bx = blk - by * T.bw;
                    px = bx * 8 + (pq & 7);
                    py = by * 8 + (pq >> 3);
                    if (PROBE) {
                        px = min(px, A.W - 1);
                        py = min(py, A.rows - 1);
                    }
                    return px < A.W && py < A.rows;
                };
                if constexpr (DENSE) {
                    // Ray generation in bulk: when the buffer holds fewer rays than there are free
                    // slots, every lane of the wave generates the ray of one reserved position
                    // (up to min(take, RB) - rb_n of them) -- instead of only the few lanes a refill frees,
                    // with the rest of the wave idle through initMarcher's divisions and square
                    // roots -- and the hits are appended to the wave's LDS ray buffer (a ring
                    // of 64); background pixels are written at once.  The free slots then take
                    // rays from the buffer in order.
                    // (a wave capped at T.take lanes buffers at most that many rays, so that a small
                    // launch's rays stay spread over the waves)
                    if (rb_n < nfree && rb_n < (uint32_t)min(T.take, RB) && !qempty) {
                        uint32_t base = 0, got = 0, base2 = 0, got2 = 0;
                        unsigned long long tsub = timing ? __builtin_amdgcn_s_memtime() : 0ull;
                        const uint32_t want = (uint32_t)min(T.take, RB) - rb_n;
                        if constexpr (QPF && TWO) {
                            // Up to two ranges: what is left of the wave's pool, then the pending
                            // reservation (requested a bulk generation earlier, so it is back by now)
                            // -- a short pool remainder does not cut this generation short.
                            if (pool_cnt) {
                                base = pool_base;
                                got = min(want, pool_cnt);
                                pool_base += got;
                                pool_cnt -= got;
                            }
                            if (got < want) {
                                if (pend) {
                                    const uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend_v);
                                    pend = false;
                                    const long tot = shard_total(shard);
                                    if ((long)b < tot) {
                                        pool_base = b;
                                        pool_cnt = (uint32_t)min((long)QCHUNK, tot - (long)b);
                                    }
                                }
                                if (pool_cnt == 0 && got == 0) reserve(want, base, got);  // blocking
                                else if (pool_cnt) {
                                    base2 = pool_base;
                                    got2 = min(want - got, pool_cnt);
                                    pool_base += got2;
                                    pool_cnt -= got2;
                                }
                            }
                            if (!qempty && !pend && pool_cnt < QLOW) {
                                pend_v = queue_add(rq, lane, shard, (uint32_t)QCHUNK);
                                pend = true;
                            }
                        } else {
                            reserve(want, base, got);
                        }
                        if constexpr (timing) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[5] += t - tsub; tsub = t; }
                        bool hit = false, keep = false;
                        F3 gp = mk3(0.0f, 0.0f, 0.0f), gd = mk3(0.0f, 0.0f, 0.0f);
                        float gt = 0.0f;
                        uint32_t glp = 0;
                        int gf = 0;
                        if ((uint32_t)lane < got + got2) {
                            int px, py;
                            const uint32_t qpos = (uint32_t)lane < got ? base + (uint32_t)lane : base2 + ((uint32_t)lane - got);
                            if (pixel_of(qpos, gf, px, py)) {
                                glp = (uint32_t)((long)py * A.W + px);
                                hit = gen_ray(A, T, BATCH ? sf[gf].inv_view : A.inv_view, px, py, gp, gd, gt);
                                keep = hit && A.max_steps > 0;
                                if (!keep) put(gf, glp, 0u);  // background (:335-339) or no iterations at all
                            }
                        }
                        nhit += (uint32_t)__popcll(__ballot(hit));
                        const uint64_t km = __ballot(keep);
                        if (keep) {
                            const uint32_t slot = (rb_head + rb_n + rank_below(km)) & (uint32_t)(RB - 1);
                            rbuf_p[wid][slot] = make_float4(gp.x, gp.y, gp.z, gt);
                            rbuf_d[wid][slot] = make_float4(gd.x, gd.y, gd.z, __uint_as_float(glp));
                            if constexpr (BATCH) rbuf_f[wid][slot] = (uint8_t)gf;
                        }
                        rb_n += (uint32_t)__popcll(km);
                        if constexpr (timing) {
                            __builtin_amdgcn_s_waitcnt(0);
                            ph[6] += __builtin_amdgcn_s_memtime() - tsub;
                        }
                    }
                    const uint32_t take = min(nfree, rb_n);
                    if (take) {
                        const unsigned long long tsub = timing ? __builtin_amdgcn_s_memtime() : 0ull;
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        const uint32_t rank = rank_below(freem);
                        if (it < 0 && rank < take) {
                            const uint32_t slot = (rb_head + rank) & (uint32_t)(RB - 1);
                            const float4 ra = rbuf_p[wid][slot], rd = rbuf_d[wid][slot];
                            p = mk3(ra.x, ra.y, ra.z);
                            tfar = ra.w;
                            if constexpr (DLDS) {
                                ray_dp[wid][lane] = rd;
                            } else {
                                d = mk3(rd.x, rd.y, rd.z);
                                pix = __float_as_uint(rd.w);
                            }
                            if constexpr (BATCH) rf = (int)rbuf_f[wid][slot];
                            it = 0;
                        }
                        rb_head = (rb_head + take) & (uint32_t)(RB - 1);
                        rb_n -= take;
                        if constexpr (timing) {
                            __builtin_amdgcn_s_waitcnt(0);
                            ph[7] += __builtin_amdgcn_s_memtime() - tsub;
                        }
                    }
                } else {
                    uint32_t base = 0, got = 0;
                    reserve(nfree, base, got);
                    if (got) {
                        const uint32_t rank = rank_below(freem);
                        bool hit = false;
                        if (it < 0 && rank < got) {
                            int f, px, py;
                            if (pixel_of(base + rank, f, px, py)) {
                                const long lp = (long)py * A.W + px;
                                hit = gen_ray(A, T, BATCH ? sf[f].inv_view : A.inv_view, px, py, p, d, tfar);
                                if (hit && A.max_steps > 0) {
                                    it = 0;
                                    pix = (uint32_t)lp;
                                    rf = f;
                                } else if (!PROBE) {
                                    put(f, lp, 0u);  // background (:335-339) or no iterations at all
                                }
                            }
                        }
                        nhit += (uint32_t)__popcll(__ballot(hit));
                    }
                }
            }
        }
        // the queue drained and no ray left to deal: the tail of the launch
        const bool drained = qempty && (!DENSE || rb_n == 0);
        NR_PHASE(shading);
        // ---- colour stashed converged rays: 16 rays x 4 tetrahedron samples per pass.
        // Once the queue is drained a partial pass waits until the wave's last ray has
        // ended: a pass costs a full MLP latency on the tail's critical path whatever
        // its size, and the marching rays must not wait for it.
        if constexpr (timing) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[0] += t - tph; pt[0] += drained ? t - tph : 0; tph = t; }
        uint64_t lm = __ballot(it >= 0);
        constexpr int SHR = PREC == NR_PRECISION_FP32 ? 16 : NR_SHADE_RAYS_LOWP;  // rays per shading pass
        bool fpass = false;  // EG: a fine pass ran in this iteration
        while (true) {
#if NR_ARG_RELOAD
            const TraceKargs *K = fresh_kargs();
            const RenderArgs &A = K->A;
            const TraceArgs &T = K->T;
#endif
        while (nstash >= SHR || (drained && nstash > 0 && !lm && nfq == 0)) {
            const int nb = min(SHR, nstash);
            const int k = lane >> 2;
            const int e = nstash - nb + (k < nb ? k : 0);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const float4 sp = stash[wid][e];
            const int sfr = BATCH ? (int)stash_f[wid][e] : 0;
            // tetrahedron point q4 (c_tet, :38-43) formed here from an opaque copy of the lane
            // index, so that the compiler does not hoist it out of the loop into three VGPRs
            // held for the kernel's life: x = +1 for q = 0, 3; y = +1 for q = 2, 3; z = +1 for q = 1, 3
            int qo = q4;
            asm volatile("" : "+v"(qo));
            const F3 tp = mk3((qo == 0 || qo == 3) ? 1.0f : -1.0f, qo >= 2 ? 1.0f : -1.0f, (qo & 1) ? 1.0f : -1.0f);
            const F3 pq = add3(mk3(sp.x, sp.y, sp.z), mul3s(tp, NORMAL_EPSILON));
            const uint32_t smask = (1u << ((4 * nb + 15) >> 4)) - 1u;
            // NX3 (bf16/fp16, M.x3n): the normals in fp32x3 from the global-memory pack, whose
            // address is made opaque here so that its loop-invariant loads are not hoisted out of
            // the shading loop into registers held for the kernel's life
            int zoff_x3 = 0;
            if constexpr (NX3) asm volatile("" : "+s"(zoff_x3));
            const float sdf = NX3 ? mlp16_x3_normal<(EG ? NR_X3N_ONE_EG : NR_X3N_ONE) != 0>(M, S.s32, (X3L ? x3l : M.x3lp) + zoff_x3, (X3L ? x3f : M.x3fl) + zoff_x3, fr_of(sfr), pq.x, pq.y,
                                                    pq.z, smask)
                                  : mlp16_fp32(M, S.s32, fr_of(sfr), pq.x, pq.y, pq.z, smask);
            const F3 cq = mul3s(tp, scene_sdf(pq, sdf, A.scene, zoff_of(sfr)));
            const F3 c1 = quad_bcast3_1(cq), c2 = quad_bcast3_2(cq), c3 = quad_bcast3_3(cq);
            if (k < nb && q4 == 0 && !T.itmap) {
                const F3 nrm = normalize3(add3(add3(add3(cq, c1), c2), c3));
                const uint32_t pxl = __float_as_uint(sp.w);
                F3 rd = mk3(0.0f, 0.0f, 0.0f);
                if (A.color_type == NR_COLOR_FACING) {
                    const int lr = (int)udiv_r(pxl, (uint32_t)A.W, A.inv_w);
                    rd = ray_dir(A, T, BATCH ? sf[sfr].inv_view : A.inv_view, (int)(pxl - (uint32_t)lr * A.W), lr);
                }
                const float *nmx = BATCH ? (const float *)((const __attribute__((address_space(1))) float *)T.frames[sfr].normal)
                                         : A.normal;
                put(sfr, pxl, shade_color(A, nmx, nrm, rd));
            }
            nconv += (uint32_t)nb;
            nstash -= nb;
        }
        NR_PHASE(fine);
        // ---- EG: a fine pass whenever the fine queue holds a full 32-point tile -- one tile (32
        // rays) while it holds fewer than 64, two tiles from 64, repeated while it holds a tile --
        // and, once the pixel queue is drained, one per iteration over up to 64 (all of them when
        // no coarse ray is left).  (Passes of 33-63 rays on two tiles: C3 / C5 batch 2-9 % slower,
        // profiles/r5_ab_eg.txt.)  The stash holds fewer than SHR rays here and a pass adds at
        // most 64 converged ones.
        if constexpr (EG) {
            if (nfq >= 32 || (drained && nfq > 0 && (!lm || !fpass))) {
                fpass = true;
                const int nb = !drained && nfq < 64 ? 32 : min(64, nfq);
                const int base = nfq - nb;
                const bool act = lane < nb;
                const int e = base + (act ? lane : 0);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                const float4 qp = fq_p[wid][e], qd = fq_d[wid][e];
                const uint32_t qi = fq_i[wid][e];
                F3 fp = mk3(qp.x, qp.y, qp.z);
                float ftf = qp.w;
                const uint32_t fpix = __float_as_uint(qd.w);
                int fit = (int)(qi & 0xffffffu);
                const int ff = BATCH ? (int)(qi >> 24) : 0;
                // the fp32x3 pack's address made opaque, as in the shading pass
                int zx = 0;
                asm volatile("" : "+s"(zx));
                // (one two-tile pass: C3 batch 1.85 -> 1.72 ms against two one-tile passes)
                const float fsdf = mlp16_x3_normal<false>(M, S.s32, (X3L ? x3l : M.x3lp) + zx, (X3L ? x3f : M.x3fl) + zx, fr_of(ff), fp.x, fp.y, fp.z,
                                                          nb > 32 ? 0xfu : 0x3u);
                nfine += (uint32_t)nb;
                nsteps += (uint32_t)nb;
                bool fconv = false, keep = false;
                if (act) {
                    // singleMarch (:416-477) on the fp32x3 value, as the coarse step below
                    const float ts = scene_sdf(fp, fsdf, A.scene, zoff_of(ff));
                    ftf -= ts;
                    int used = 0;
                    if (ftf <= 0) {
                        put(ff, fpix, 0u);
                        used = fit + 1;
                    } else {
                        fp = add3(fp, mul3s(mk3(qd.x, qd.y, qd.z), ts));
                        if (ts < MARCHING_EPSILON) {
                            if (fit + 1 < A.max_steps) {
                                fconv = true;
                                used = fit + 2;
                            } else {
                                put(ff, fpix, 0u);
                                used = fit + 1;
                            }
                        } else if (++fit >= A.max_steps) {
                            put(ff, fpix, 0u);
                            used = A.max_steps;
                        }
                    }
                    if (used) {
                        maxit = max(maxit, used);
                        if (T.itmap) put(ff, fpix, (uint32_t)used);
                        if (T.bcost) {
                            const int yy = (int)(fpix / (uint32_t)A.W), xx = (int)(fpix - (uint32_t)yy * A.W);
                            atomicMax(T.bcost + (yy >> 3) * T.bw + (xx >> 3), (uint32_t)used);
                        }
                    } else {
                        keep = true;
                    }
                }
                // survivors back to the queue (positions [base, base + survivors)), converged rays
                // to the stash
                const uint64_t km = __ballot(keep), cm = __ballot(fconv);
                if (keep) {
                    const int slot = base + (int)rank_below(km);
                    fq_p[wid][slot] = make_float4(fp.x, fp.y, fp.z, ftf);
                    fq_d[wid][slot] = qd;
                    fq_i[wid][slot] = (uint32_t)fit | ((uint32_t)ff << 24);
                }
                if (fconv) {
                    const int slot = nstash + (int)rank_below(cm);
                    stash[wid][slot] = make_float4(fp.x, fp.y, fp.z, __uint_as_float(fpix));
                    if constexpr (BATCH) stash_f[wid][slot] = (uint8_t)ff;
                }
                nstash += (int)__popcll(cm);
                nfq = base + (int)__popcll(km);
                continue;
            }
        }
        break;
        }
        if constexpr (timing) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[1] += t - tph; pt[0] += drained ? t - tph : 0; tph = t; }
        if (!lm) {
            if (drained && nstash == 0 && nfq == 0) break;
            continue;
        }
        uint32_t tmask = tiles_of(lm);
        NR_PHASE(compaction);
        // ---- tail: pack the live rays into the lowest tiles
        if (drained) {
            const int nl = (int)__popcll(lm);
            const int need = (nl + 15) >> 4;
            if (__popc(tmask) > need) {
                const int src = select_bit(lm, lane < nl ? lane : 0);
                p = mk3(__shfl(p.x, src), __shfl(p.y, src), __shfl(p.z, src));
                if constexpr (DLDS) {
                    const float4 dp = ray_dp[wid][lane];
                    ray_dp[wid][lane] = make_float4(__shfl(dp.x, src), __shfl(dp.y, src), __shfl(dp.z, src), __shfl(dp.w, src));
                } else {
                    d = mk3(__shfl(d.x, src), __shfl(d.y, src), __shfl(d.z, src));
                    pix = (uint32_t)__shfl((int)pix, src);
                }
                tfar = __shfl(tfar, src);
                if constexpr (BATCH) rf = __shfl(rf, src);
                const int it_src = __shfl(it, src);
                it = lane < nl ? it_src : -1;
                lm = __ballot(it >= 0);
                tmask = (1u << need) - 1u;
            }
        }
        NR_PHASE(mlp);
        // ---- MLP on every live point, then one sphere-trace step per ray
        if (NONMLP_PRIO) __builtin_amdgcn_s_setprio(0);
        if (MLP_PRIO) set_priority(MLP_PRIO);
        const float sdf = mlp16(M, S.s32, S.slp, S.sfl, prec, fr_of(rf), p.x, p.y, p.z, tmask, M.lp_clamp != 0);
        NR_PHASE(step);
#if NR_ARG_RELOAD
        const TraceKargs *K = fresh_kargs();
        const RenderArgs &A = K->A;
        const TraceArgs &T = K->T;
#endif
        if constexpr (timing) {
            // iterations with <= 4 rays (low word) and ray-steps (high word) after the drain; the
            // live rays when the wave first saw the queue drained
            pt[3] += drained ? ((__popcll(lm) <= 4 ? 1ull : 0ull) | ((unsigned long long)__popcll(lm) << 32)) : 0ull;
            if (drained && nl_drain < 0) nl_drain = (int)__popcll(lm);
        }
        if (NONMLP_PRIO) set_priority(NONMLP_PRIO);
        if (MLP_PRIO) __builtin_amdgcn_s_setprio(0);
        if constexpr (timing) {
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            ph[2] += t - tph; pt[1] += drained ? t - tph : 0; tph = t;
        }
        nsteps += (uint32_t)__popcll(lm);
        if (nsteps >= (1u << 30)) {
            if (lane == 0) atomicAdd(T.stats + 0, (unsigned long long)nsteps);
            nsteps = 0;
        }
        if (EG && nfine >= (1u << 30)) {
            if (lane == 0) atomicAdd(T.stats + 4, (unsigned long long)nfine);
            nfine = 0;
        }
        ++wit;
        wit_tail += drained ? 1u : 0u;
        bool conv = false;
        if constexpr (EG) {
            // the endgame's switch: the ray goes to the fine queue without taking the step (the
            // fine pass re-evaluates this point in fp32x3); its lane is free for a new ray
            const bool hand = it >= 0 && sdf < T.eg_tau;
            const uint64_t hm = __ballot(hand);
            if (hm) {
                if (hand) {
                    const int slot = nfq + (int)rank_below(hm);
                    fq_p[wid][slot] = make_float4(p.x, p.y, p.z, tfar);
                    fq_d[wid][slot] = ray_dp[wid][lane];
                    fq_i[wid][slot] = (uint32_t)it | ((uint32_t)rf << 24);
                    it = -1;
                }
                nfq += (int)__popcll(hm);
                nswitch += (uint32_t)__popcll(hm);
            }
        }
        if (it >= 0) {
            NR_PHASE(scene);
            const float ts = scene_sdf(p, sdf, A.scene, zoff_of(rf));
            NR_PHASE(step);
            if constexpr (timing) {
                __builtin_amdgcn_s_waitcnt(0);
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                ph[3] += t - tph; pt[2] += drained ? t - tph : 0; tph = t;
            }
            if constexpr (DLDS) {
                const float4 dp = ray_dp[wid][lane];
                d = mk3(dp.x, dp.y, dp.z);
                pix = __float_as_uint(dp.w);
            }
            tfar -= ts;
            int used = 0;  // iterations this ray consumed, if it ends now
            if (tfar <= 0) {
                if (!PROBE) put(rf, pix, 0u);
                used = it + 1;
            } else {
                p = add3(p, mul3s(d, ts));
                if (ts < MARCHING_EPSILON) {
                    if (it + 1 < A.max_steps) {  // coloured in the next iteration (:446-457)
                        conv = !PROBE;
                        used = it + 2;
                    } else {
                        if (!PROBE) put(rf, pix, 0u);
                        used = it + 1;
                    }
                } else if (++it >= A.max_steps) {  // iteration cap: pixel stays 0 (:690)
                    if (!PROBE) put(rf, pix, 0u);
                    used = A.max_steps;
                }
            }
            if (used) {  // the ray ended
                it = -1;
                maxit = max(maxit, used);
                if (!PROBE && T.itmap) put(rf, pix, (uint32_t)used);
                if (T.bcost) {
                    const int yy = (int)(pix / (uint32_t)A.W), xx = (int)(pix - (uint32_t)yy * A.W);
                    atomicMax(T.bcost + (yy >> 3) * T.bw + (xx >> 3), (uint32_t)used);
                }
            }
        }
        const uint64_t cm = __ballot(conv);
        if (conv) {
            const int slot = nstash + (int)rank_below(cm);
            stash[wid][slot] = make_float4(p.x, p.y, p.z, __uint_as_float(pix));
            if constexpr (BATCH) stash_f[wid][slot] = (uint8_t)rf;
        }
        nstash += (int)__popcll(cm);
        if constexpr (timing) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[4] += t - tph; pt[0] += drained ? t - tph : 0; tph = t; }
        NR_PHASE(loop_end);
    }
    // ---- frame statistics: one set of atomics per wave
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) maxit = max(maxit, __shfl_xor(maxit, off));
    if (STAMPS && lane == 0) {
        unsigned long long *st = T.stamps + 16 * gwave;
        st[0] = t_start; st[1] = t_empty | ((unsigned long long)(nl_drain < 0 ? 0 : nl_drain) << 56);
        st[2] = __builtin_amdgcn_s_memrealtime();
        st[3] = ((unsigned long long)wit_tail << 32) | wit;
        for (int i = 0; i < 8; ++i) st[4 + i] = ph[i];
        for (int i = 0; i < 4; ++i) st[12 + i] = pt[i];
    }
    if (lane == 0) {
        if (nsteps) atomicAdd(T.stats + 0, (unsigned long long)nsteps);
        if (nhit) atomicAdd(T.stats + 1, (unsigned long long)nhit);
        if (nconv) atomicAdd(T.stats + 3, (unsigned long long)nconv);
        if (maxit) atomicMax(T.stats + 2, (unsigned long long)maxit);
        if (EG && nfine) atomicAdd(T.stats + 4, (unsigned long long)nfine);
        if (EG && nswitch) atomicAdd(T.stats + 5, (unsigned long long)nswitch);
    }
}

// diagnostic build (tools/mlp_stamps.py): per-wave cycle stamps of the 16-bit k_mlp16 loop in Y
#ifndef NR_MLP16_STAMPS
#define NR_MLP16_STAMPS 0
#endif
// waves per SIMD k_mlp16's registers target (<= 96 VGPRs at 5)
#ifndef NR_MLP16_WPS
#define NR_MLP16_WPS 5
#endif
#ifndef NR_MLP16_WPS_X3
#define NR_MLP16_WPS_X3 4
#endif
// bf16 / fp16: the 128-point form holds four accumulators (64 VGPRs) and their operands
#ifndef NR_MLP16_WPS_LP
#define NR_MLP16_WPS_LP 3
#endif
// Stand-alone batched MLP (NeuralNetwork::forward, neuralNetwork.cpp:54-63) on the
// matrix-core tiles: X [n][in0] -> Y [n], n < 2^26 per launch (launch_mlp16 splits).
// Grid-stride over chunks of 64 points (fp32, fp32x3) or 128 points (bf16, fp16: two per lane,
// nr_mlp16.h mlp32_lowp_128).  The inputs and outputs go through buffer resources sized to the
// arrays: a position past the end loads zeros and drops its store, so every load and store is
// unconditional -- the next chunk's inputs are requested before the current chunk's MLP and
// waited for only after it (a load behind a lane-divergent branch was waited for at once,
// stalling every wave ~1 us per chunk), and the per-lane offsets are 32-bit.
typedef uint32_t u32x3v __attribute__((ext_vector_type(3)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_of(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
// IN0: the network's inputs (3, or 4 with the frame): a template parameter, so that the load is
// not behind a branch (whose join waited for it).  4-wave workgroups deal the chunks grid-stride.
// S16 (bf16 / fp16, MlpArgs::lp_s16): every chunk on the 16x16x32 stream -- a separate instance,
// so that the 32x32x16 stream's pinned registers do not share its register allocation.
template <int PREC, int IN0, bool S16 = false>
__global__ __launch_bounds__(256, PREC == NR_PRECISION_FP32X3 ? NR_MLP16_WPS_X3
                                  : PREC == NR_PRECISION_FP32 ? NR_MLP16_WPS : NR_MLP16_WPS_LP) void k_mlp16(MlpArgs M, const float *__restrict__ X, float *__restrict__ Y, int n) {
    constexpr int WPG = 4;  // waves per workgroup
    Smem16 S = stage16<PREC, false>(M);
    const int lane = lane_id();
    constexpr int in0 = IN0;
    M.in0 = IN0;
    const auto rx = buffer_of(X, (uint32_t)n * (uint32_t)in0 * 4u), ry = buffer_of(Y, (uint32_t)n * 4u);
    // point i's inputs (zeros past the end); the 4th is the frame for 4-input networks
    auto load = [&](uint32_t i, float &x, float &y, float &z, float &f) {
        if constexpr (in0 == 4) {
            const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(rx, i * 16u, 0, 0);
            x = __uint_as_float(v.x); y = __uint_as_float(v.y); z = __uint_as_float(v.z); f = __uint_as_float(v.w);
        } else {
            const u32x3v v = __builtin_amdgcn_raw_buffer_load_b96(rx, i * 12u, 0, 0);
            x = __uint_as_float(v.x); y = __uint_as_float(v.y); z = __uint_as_float(v.z); f = 0.0f;
        }
    };
    auto store = [&](uint32_t i, float v) { __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ry, i * 4u, 0, 0); };
    // the wave's chunk index is uniform (SGPRs); launch_mlp16 launches WPG-wave workgroups (blockDim,
    // read from the dispatch packet by a vector load, would put the indices in VGPRs)
    const int wave = __builtin_amdgcn_readfirstlane((int)blockIdx.x * WPG + (int)(threadIdx.x >> 6));
    const int waves = __builtin_amdgcn_readfirstlane((int)gridDim.x * WPG);
    if constexpr (PREC == NR_PRECISION_BF16 || PREC == NR_PRECISION_FP16) {
        // 128 points per wave and chunk: point base + lane and base + 64 + lane; a last chunk of
        // at most 64 points takes the 64-point form
        // The loop takes only whole 128-point chunks, so that one path leads from the next chunk's
        // input loads to their use: with the ragged chunk inside it, the merge of its one-store path
        // made hipcc wait for this chunk's stores too (s_waitcnt vmcnt(0) on every chunk, a store's
        // round trip to memory).  The ragged last chunk follows the loop, on the wave whose turn it is.
        auto run = [&](int base, const float (&x)[2], const float (&y)[2], const float (&z)[2], const float (&f)[2]) {
            const int rem = n - base;
            // the bf16 clamped pack's input bound (NaN is not within it)
            constexpr float XB = LP_INPUT_BOUND, FB = LP_INPUT_BOUND;
            const bool ok0 = __builtin_fabsf(x[0]) <= XB && __builtin_fabsf(y[0]) <= XB && __builtin_fabsf(z[0]) <= XB &&
                             __builtin_fabsf(f[0]) <= FB;
            const bool ok1 = __builtin_fabsf(x[1]) <= XB && __builtin_fabsf(y[1]) <= XB && __builtin_fabsf(z[1]) <= XB &&
                             __builtin_fabsf(f[1]) <= FB;
            if (rem <= 64 && !S16) {  // (the 16x16x32 pack serves only the 128-point stream)
                const uint32_t tmask = rem >= 64 ? 0xfu : (1u << ((rem + 15) >> 4)) - 1u;
                store((uint32_t)(base + lane), mlp16(M, S.s32, S.slp, S.sfl, PREC, f[0], x[0], y[0], z[0], tmask,
                                                     M.lp_clamp && __ballot(!ok0) == 0));
                return;
            }
            float v[2];
            if (PREC == NR_PRECISION_BF16 && M.lp_clamp && __ballot(!(ok0 && ok1)) == 0)
                mlp128_lowp_cl<PREC, true>(S.slp, S.sfl, in0, M.nh, f, x, y, z, v, S16 || M.lp_stream != 0, S16);
            else
                mlp128_lowp_cl<PREC, false>(S.slp, S.sfl, in0, M.nh, f, x, y, z, v, S16 || M.lp_stream != 0, S16);
            store((uint32_t)(base + lane), v[0]);
            store((uint32_t)(base + 64 + lane), v[1]);
        };
        const int nfull = n & ~127;
#if NR_MLP16_STAMPS
        unsigned long long st_mlp = 0;
        uint32_t st_n = 0;
#endif
        // Chunk dealing, grid-stride: a wave's chunks are wave, wave + waves, ...  (The oldest wave
        // of each SIMD wins issue arbitration and finishes its share at ~2/3 of the loop; balancing
        // the CU's waves through an LDS chunk queue or global claims did not raise the chunk rate,
        // round 4: profiles/r4_mlp_ab.txt, r4_ab_dyn.txt, r4_mlp_stamps_hwid.txt.)
        const uint32_t nch = (uint32_t)(nfull >> 7);
        int gs = wave;
        auto first = [&]() -> int {
            const int c = gs;
            gs += waves;
            return c < (int)nch ? c : -1;
        };
        int cur = first(), nxt = first();
        float nx[2], ny[2], nz[2], nf[2];
        const int c0 = cur < 0 ? (int)nch : cur;
        load((uint32_t)(c0 * 128 + lane), nx[0], ny[0], nz[0], nf[0]);
        load((uint32_t)(c0 * 128 + 64 + lane), nx[1], ny[1], nz[1], nf[1]);
        // the first chunk's inputs, waited for here (s_waitcnt vmcnt(0)): the loop is then entered
        // with nothing in flight, and hipcc's merge of the entry path into the loop's wait counts
        // adds no wait to the back edge (where the inputs arrive by copies waited for a chunk earlier)
        __builtin_amdgcn_s_waitcnt(0x0f70);
        // One chunk: wait for its inputs (requested one chunk earlier) -> every memory operation of
        // the iteration: the next chunk's input loads, the previous chunk's stores (its outputs were
        // kept in registers) -> MLP.  With them all at the top, any wait hipcc puts there is for operations a whole chunk old
        // (it merges wait counts over the loop's paths conservatively: with stores at the end of the
        // previous iteration it waited for their round trip to memory before every chunk).
        float pv[2] = {0.0f, 0.0f};
        int pbase = n;  // the previous chunk (none: its stores fall past Y's end and are dropped)
        auto body = [&]() {
            // everything in flight was issued a chunk ago: wait for it all here (free), so that
            // hipcc's scoreboard holds nothing older than this iteration's own requests
            __builtin_amdgcn_s_waitcnt(0x0f70);
            const int base = cur * 128;
            const float x[2] = {nx[0], nx[1]}, y[2] = {ny[0], ny[1]}, z[2] = {nz[0], nz[1]}, f[2] = {nf[0], nf[1]};
            const int nb = (nxt < 0 ? (int)nch : nxt) * 128;  // past the last chunk: zeros, unused
            load((uint32_t)(nb + lane), nx[0], ny[0], nz[0], nf[0]);
            load((uint32_t)(nb + 64 + lane), nx[1], ny[1], nz[1], nf[1]);
            store((uint32_t)(pbase + lane), pv[0]);
            store((uint32_t)(pbase + 64 + lane), pv[1]);
#if NR_MLP16_STAMPS
            const unsigned long long ta = __builtin_amdgcn_s_memtime();
#endif
            constexpr float XB = LP_INPUT_BOUND, FB = LP_INPUT_BOUND;
#if NR_MLP16_EXP & 2
            const bool ok = true;
#else
            const bool ok = __builtin_fabsf(x[0]) <= XB && __builtin_fabsf(y[0]) <= XB && __builtin_fabsf(z[0]) <= XB &&
                            __builtin_fabsf(f[0]) <= FB && __builtin_fabsf(x[1]) <= XB && __builtin_fabsf(y[1]) <= XB &&
                            __builtin_fabsf(z[1]) <= XB && __builtin_fabsf(f[1]) <= FB;
#endif
            if (PREC == NR_PRECISION_BF16 && M.lp_clamp && __ballot(!ok) == 0)
                mlp128_lowp_cl<PREC, true>(S.slp, S.sfl, in0, M.nh, f, x, y, z, pv, S16 || M.lp_stream != 0, S16);
            else
                mlp128_lowp_cl<PREC, false>(S.slp, S.sfl, in0, M.nh, f, x, y, z, pv, S16 || M.lp_stream != 0, S16);
#if NR_MLP16_STAMPS
            st_mlp += __builtin_amdgcn_s_memtime() - ta;
            ++st_n;
#endif
            pbase = base;
            cur = nxt;
            nxt = first();
        };
#if NR_MLP16_STAMPS
        const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
        while (cur >= 0) body();
        store((uint32_t)(pbase + lane), pv[0]);
        store((uint32_t)(pbase + 64 + lane), pv[1]);
#if NR_MLP16_STAMPS
        // diagnostic build: per wave {cycles in the loop, of them in the MLP calls, chunks} in Y
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            Y[4 * wave] = (float)(t1 - t0);
            Y[4 * wave + 1] = (float)st_mlp;
            Y[4 * wave + 2] = (float)st_n;
            Y[4 * wave + 3] = (float)(r1 - r0);  // 100 MHz ticks
            // the loop's start and end on the chip's 100 MHz clock (low 24 bits), after the per-wave block
            Y[4 * waves + 2 * wave] = (float)(r0 & 0xffffffull);
            Y[4 * waves + 2 * wave + 1] = (float)(r1 & 0xffffffull);
            // where the wave ran: HW_ID (wave, SIMD, CU, SH, SE fields) and XCC_ID, 16 bits each
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
            Y[6 * waves + 2 * wave] = (float)(hw & 0xffffu);
            Y[6 * waves + 2 * wave + 1] = (float)(((hw >> 16) & 0xffu) | ((xcc & 0xfu) << 8));
        }
        return;
#endif
        // the ragged last chunk (1-127 points): the last wave of the grid
        if (nfull < n && wave == waves - 1) {
            float x[2], y[2], z[2], f[2];
            load((uint32_t)(nfull + lane), x[0], y[0], z[0], f[0]);
            load((uint32_t)(nfull + 64 + lane), x[1], y[1], z[1], f[1]);
            run(nfull, x, y, z, f);
        }
        return;
    }
    const int stride = waves * 64;
    int base = wave * 64;
    float nx, ny, nz, nf;
    load((uint32_t)(base + lane), nx, ny, nz, nf);
    for (; base < n; base += stride) {
        base = __builtin_amdgcn_readfirstlane(base);
        const float x = nx, y = ny, z = nz, f = nf;
        load((uint32_t)(base + stride + lane), nx, ny, nz, nf);
        const int rem = n - base;
        const uint32_t tmask = rem >= 64 ? 0xfu : (1u << ((rem + 15) >> 4)) - 1u;
        store((uint32_t)(base + lane),
              mlp16(M, S.s32, S.slp, S.sfl, PREC, f, x, y, z, tmask, M.lp_clamp && inputs_in_bound(x, y, z, f)));
    }
}

// Counting sort of the blocks by their cost, descending (one workgroup): the order in
// which the next frame dispenses blocks, so that its longest rays start first.  With
// `dilate`, a block's key is the max over its 3x3 neighbourhood (bw blocks per row) --
// for a probe that saw one ray per block, a long ray next door marks a likely edge.
__device__ __forceinline__ uint32_t order_key(const uint32_t *__restrict__ bcost, int b, int nblocks, int bw,
                                              int dilate) {
    uint32_t v = bcost[b];
    if (dilate) {
        const int by = b / bw, bx = b - by * bw, bh = (nblocks + bw - 1) / bw;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                const int x = bx + dx, y = by + dy;
                if (x >= 0 && x < bw && y >= 0 && y < bh && y * bw + x < nblocks) v = max(v, bcost[y * bw + x]);
            }
    }
    return 1023 - min(v, 1023u);
}

__global__ __launch_bounds__(1024) void k_order(const uint32_t *__restrict__ bcost, uint32_t *__restrict__ order,
                                                int nblocks, int bw, int dilate) {
    __shared__ uint32_t hist[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int b = threadIdx.x; b < nblocks; b += blockDim.x) atomicAdd(&hist[order_key(bcost, b, nblocks, bw, dilate)], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan (1024 bins, once per frame)
        uint32_t run = 0;
        for (int i = 0; i < 1024; ++i) { uint32_t v = hist[i]; hist[i] = run; run += v; }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nblocks; b += blockDim.x)
        order[atomicAdd(&hist[order_key(bcost, b, nblocks, bw, dilate)], 1u)] = (uint32_t)b;
}

hipError_t launch_order(const uint32_t *bcost, uint32_t *order, int nblocks, int bw, int dilate, hipStream_t st) {
    hipLaunchKernelGGL(k_order, dim3(1), dim3(1024), 0, st, bcost, order, nblocks, bw, dilate);
    return hipGetLastError();
}

hipError_t launch_mlp16(const MlpArgs &M0, int prec, const float *X, float *Y, long n, int grid, hipStream_t st) {
    const bool lowp = prec == NR_PRECISION_BF16 || prec == NR_PRECISION_FP16;
    // bf16 / fp16 networks with 7 hidden layers: the 16x16x32 pack and stream (MlpArgs::lps)
    MlpArgs M = M0;
    M.lp_s16 = 0;
    if (lowp && M.lps && M.lp_stream && M.nh == 7) {
        M.lp = M.lps;
        M.lpf = M.lpfs;
        M.lp_s16 = 1;
    }
    const int sm = smem16_bytes(M, prec, false);
    // segments of at most 2^26 points: the kernel's buffer offsets (n * in0 * 4 bytes) are 32-bit
    constexpr long SEG = 1l << 26;
    for (long p0 = 0; p0 < n; p0 += SEG) {
        const int m = (int)std::min(SEG, n - p0);
        const float *x = X + p0 * M.in0;
        float *y = Y + p0;
        // points per workgroup: 4 waves x 64 (fp32, fp32x3) or x 128 (bf16, fp16: two per lane)
        const long per_wg = lowp ? 512 : 256;
        const int g = (int)std::max<long>(1, std::min<long>(grid, ((long)m + per_wg - 1) / per_wg));
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(g), dim3(256), sm, st, M, x, y, m); };
        const bool four = M.in0 == 4;
        if (M.lp_s16 && prec == NR_PRECISION_BF16)
            four ? go(k_mlp16<NR_PRECISION_BF16, 4, true>) : go(k_mlp16<NR_PRECISION_BF16, 3, true>);
        else if (M.lp_s16 && prec == NR_PRECISION_FP16)
            four ? go(k_mlp16<NR_PRECISION_FP16, 4, true>) : go(k_mlp16<NR_PRECISION_FP16, 3, true>);
        else if (prec == NR_PRECISION_BF16) four ? go(k_mlp16<NR_PRECISION_BF16, 4>) : go(k_mlp16<NR_PRECISION_BF16, 3>);
        else if (prec == NR_PRECISION_FP16) four ? go(k_mlp16<NR_PRECISION_FP16, 4>) : go(k_mlp16<NR_PRECISION_FP16, 3>);
        else if (prec == NR_PRECISION_FP32X3) four ? go(k_mlp16<NR_PRECISION_FP32X3, 4>) : go(k_mlp16<NR_PRECISION_FP32X3, 3>);
        else four ? go(k_mlp16<NR_PRECISION_FP32, 4>) : go(k_mlp16<NR_PRECISION_FP32, 3>);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// one k_trace instance: bf16/fp16 with fp32x3 normals when the network has the pack (M.x3n)
template <int PREC, bool PROBE, bool STAMPS, bool BATCH>
static hipError_t launch_trace_k(const RenderArgs &A, const MlpArgs &M, const TraceArgs &T, int grid, int sm,
                                 hipStream_t st) {
    constexpr bool LOWP = PREC == NR_PRECISION_BF16 || PREC == NR_PRECISION_FP16;
    if constexpr (LOWP && !PROBE) {
        if constexpr (!STAMPS) {
            if (M.x3n && T.eg_tau > 0.0f) {
                // the grid is at most NR_TRACE_BPC_EG 4-wave workgroups per CU (nr_api.hip trace_bpc):
                // as NR_EG_WAVES-wave workgroups, one per CU, with the fp32x3 pack in their LDS --
                // when the two packs fit beside the instance's static LDS (networks of up to 9 hidden
                // layers), else as round 5's 4-wave workgroups reading the pack from global memory
                constexpr int G = NR_EG_WAVES / 4;
                const int smx = smem16_bytes(M, PREC, true, T.x3lp_bytes + T.x3fl_bytes);
                static const int static_lds = [] {
                    hipFuncAttributes fa{};
                    const void *k = reinterpret_cast<const void *>(&k_trace<PREC, PROBE, STAMPS, BATCH, true, true, true>);
                    return hipFuncGetAttributes(&fa, k) == hipSuccess ? (int)fa.sharedSizeBytes : (1 << 30);
                }();
                if (NR_EG_WAVES > 4 && static_lds + smx <= NR_LDS_PER_CU) {
                    const int g = std::max(1, (grid + G - 1) / G);
                    hipLaunchKernelGGL((k_trace<PREC, PROBE, STAMPS, BATCH, true, true, true>), dim3(g), dim3(64 * NR_EG_WAVES),
                                       smx, st, A, M, T);
                } else {
                    hipLaunchKernelGGL((k_trace<PREC, PROBE, STAMPS, BATCH, true, true, false>), dim3(grid), dim3(256), sm,
                                       st, A, M, T);
                }
                return hipGetLastError();
            }
        }
        if (M.x3n) {
            hipLaunchKernelGGL((k_trace<PREC, PROBE, STAMPS, BATCH, true>), dim3(grid), dim3(256), sm, st, A, M, T);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_trace<PREC, PROBE, STAMPS, BATCH>), dim3(grid), dim3(256), sm, st, A, M, T);
    return hipGetLastError();
}

template <bool PROBE, bool STAMPS, bool BATCH>
static hipError_t launch_trace_p(const RenderArgs &A, const MlpArgs &M, const TraceArgs &T, int prec, int grid, int sm,
                                 hipStream_t st) {
    if (prec == NR_PRECISION_BF16) return launch_trace_k<NR_PRECISION_BF16, PROBE, STAMPS, BATCH>(A, M, T, grid, sm, st);
    if (prec == NR_PRECISION_FP16) return launch_trace_k<NR_PRECISION_FP16, PROBE, STAMPS, BATCH>(A, M, T, grid, sm, st);
    if (prec == NR_PRECISION_FP32X3)
        return launch_trace_k<NR_PRECISION_FP32X3, PROBE, STAMPS, BATCH>(A, M, T, grid, sm, st);
    return launch_trace_k<NR_PRECISION_FP32, PROBE, STAMPS, BATCH>(A, M, T, grid, sm, st);
}

hipError_t launch_trace(const RenderArgs &A, const MlpArgs &M, const TraceArgs &T, int prec, int grid, hipStream_t st) {
    const int sm = smem16_bytes(M, prec, true);
    if (T.probe) return launch_trace_p<true, false, false>(A, M, T, prec, grid, sm, st);
    if (T.nframes > 0) return launch_trace_p<false, false, true>(A, M, T, prec, grid, sm, st);
    if (T.stamps) return launch_trace_p<false, true, false>(A, M, T, prec, grid, sm, st);
    return launch_trace_p<false, false, false>(A, M, T, prec, grid, sm, st);
}

}  // namespace nr
