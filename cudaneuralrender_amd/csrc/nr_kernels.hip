// nr_kernels.hip -- gfx950 (CDNA4) kernels of the neural-SDF sphere tracer.
//
// Hot path of the reference (daviesthomas/cudaNeuralRender @ v1):
//   src/volumeRender_kernel.cu:608-692 render loop, with the per-iteration
//   nn.forward (:661 -> src/layers/denseLayer.cu:126-176, 9 CUTLASS launches) and
//   singleMarch (:416-477), plus a full-image exclusive scan + 4-byte D2H sync per
//   iteration (:549-576).
// Re-designed for MI355X:
//   * k_init     ray generation (initMarcher :293-358) + wave-ballot compaction of
//                the rays that hit the bounding sphere into a dense queue.
//   * k_march    ONE launch per iteration: a wave takes 64 live rays, evaluates the
//                whole MLP on them (hidden 32x32 layers on the matrix cores, weights
//                resident in LDS, activations never leave registers), takes the
//                sphere-trace step and compacts survivors / converged rays into the
//                next queues (ballot + one atomic per wave).  No host sync, no
//                activation buffers, no full-image scans.
//   * k_shade    tetrahedral normals (surfaceNormal :361-377; 4 MLP evaluations per
//                ray, 16 rays per wave) + matcap / facing colour (:380-413).
//   * k_mlp      stand-alone batched MLP (NeuralNetwork::forward) on the same code.
//   * k_dense    generic single dense layer (DenseLayer::forward) for any shape.
//
// Numerics: compiled with -ffp-contract=off.  FP32 mode is bit-exact with the CPU
// oracle: v_mfma_f32_32x32x2_f32 is a k-ordered fmaf chain (cdna_hip_programming.md
// §3), and the weight pack permutes the hidden units so that the chain runs over
// k = 0..31 in ascending order, exactly the oracle's fmaf loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nr_device.h"

namespace nr {

// ------------------------------------------------------------- the MLP
// One wave evaluates the network on 64 points: point p of the wave is owned by
// lane p on entry and exit.  Internally the 64 points form two 32-point MFMA tiles
// (tile t = points 32t..32t+31); lane (c, h) = (lane & 31, lane >> 5) holds point c
// of each tile and the 16 hidden units of half h (register r <-> unit given by the
// pack, nr_pack.cpp).  `s` is the fp32 pack in LDS.
__device__ float mlp_fp32_wave(const float *__restrict__ s, int in0, int nh, float x, float y, float z, float fr) {
    const int lane = lane_id();
    const int h = lane >> 5, c = lane & 31;
    const float x0 = __shfl(x, c), y0 = __shfl(y, c), z0 = __shfl(z, c);
    const float x1 = __shfl(x, c + 32), y1 = __shfl(y, c + 32), z1 = __shfl(z, c + 32);
    float f0 = 0.0f, f1 = 0.0f;
    if (in0 == 4) { f0 = __shfl(fr, c); f1 = __shfl(fr, c + 32); }
    float a0[16], a1[16];
    // layer 0 on VALU: k-ordered fmaf chain from +0, then + bias, ReLU
    {
        const float4 *w0 = reinterpret_cast<const float4 *>(s + PK_L0W) + h * 16;
        const float *b0 = s + PK_L0B + h * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float4 w = w0[r];
            float acc0 = __builtin_fmaf(w.x, x0, 0.0f), acc1 = __builtin_fmaf(w.x, x1, 0.0f);
            acc0 = __builtin_fmaf(w.y, y0, acc0); acc1 = __builtin_fmaf(w.y, y1, acc1);
            acc0 = __builtin_fmaf(w.z, z0, acc0); acc1 = __builtin_fmaf(w.z, z1, acc1);
            if (in0 == 4) { acc0 = __builtin_fmaf(w.w, f0, acc0); acc1 = __builtin_fmaf(w.w, f1, acc1); }
            a0[r] = fmaxf(acc0 + b0[r], 0.0f);
            a1[r] = fmaxf(acc1 + b0[r], 0.0f);
        }
    }
    // hidden 32x32 layers: v_mfma_f32_32x32x2_f32, 16 k-steps, two tiles share the A operand
    for (int j = 0; j < nh; ++j) {
        const float *L = s + PK_HID + j * PK_HID_STRIDE;
        f32x16 c0 = {}, c1 = {};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float4 wv = reinterpret_cast<const float4 *>(L)[g * 64 + lane];
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, a0[4 * g + 0], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.x, a1[4 * g + 0], c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, a0[4 * g + 1], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.y, a1[4 * g + 1], c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, a0[4 * g + 2], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.z, a1[4 * g + 2], c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, a0[4 * g + 3], c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wv.w, a1[4 * g + 3], c1, 0, 0, 0);
        }
        const float *bb = L + 1024 + h * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = fmaxf(c0[r] + bb[r], 0.0f);
            a1[r] = fmaxf(c1[r] + bb[r], 0.0f);
        }
    }
    // final 32 -> 1 on VALU: half 0 holds units 0..15, half 1 units 16..31.  Lane
    // (c,0) runs the chain over 0..15, lane (c,1) continues it over 16..31.
    const float *wf = s + pk_final(nh) + h * 16;
    const float bf = s[pk_final(nh) + 32];
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) { p0 = __builtin_fmaf(wf[r], a0[r], p0); p1 = __builtin_fmaf(wf[r], a1[r], p1); }
    float q0 = __shfl(p0, c), q1 = __shfl(p1, c);  // partials of half 0
#pragma unroll
    for (int r = 0; r < 16; ++r) { q0 = __builtin_fmaf(wf[r], a0[r], q0); q1 = __builtin_fmaf(wf[r], a1[r], q1); }
    const float zt0 = q0 + bf, zt1 = q1 + bf;  // valid in half-1 lanes
    // point p (lane p) <- tile p>>5, held in lane (p & 31) + 32
    const float r0 = __shfl(zt0, c + 32);
    return h ? zt1 : r0;
}

// Low-precision (bf16 / fp16) hidden layers on v_mfma_f32_32x32x16_{bf16,f16};
// layer 0 and the final layer stay fp32 on VALU.  `lp` is the 16-bit A-operand
// pack, `fl` the float side pack (nr_internal.h).
template <int PREC>
__device__ float mlp_lowp_wave(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0, int nh,
                               float x, float y, float z, float fr) {
    typedef typename std::conditional<PREC == NR_PRECISION_BF16, bf16x8, f16x8>::type v8;
    typedef typename std::conditional<PREC == NR_PRECISION_BF16, __bf16, _Float16>::type e16;
    const int lane = lane_id();
    const int h = lane >> 5, c = lane & 31;
    const float x0 = __shfl(x, c), y0 = __shfl(y, c), z0 = __shfl(z, c);
    const float x1 = __shfl(x, c + 32), y1 = __shfl(y, c + 32), z1 = __shfl(z, c + 32);
    float f0 = 0.0f, f1 = 0.0f;
    if (in0 == 4) { f0 = __shfl(fr, c); f1 = __shfl(fr, c + 32); }
    float a0[16], a1[16];
    {
        const float4 *w0 = reinterpret_cast<const float4 *>(fl) + h * 16;
        const float *b0 = fl + 128 + h * 16;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float4 w = w0[r];
            float acc0 = w.x * x0 + w.y * y0 + w.z * z0, acc1 = w.x * x1 + w.y * y1 + w.z * z1;
            if (in0 == 4) { acc0 += w.w * f0; acc1 += w.w * f1; }
            a0[r] = fmaxf(acc0 + b0[r], 0.0f);
            a1[r] = fmaxf(acc1 + b0[r], 0.0f);
        }
    }
    for (int j = 0; j < nh; ++j) {
        v8 b0lo, b0hi, b1lo, b1hi;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            b0lo[e] = (e16)a0[e]; b0hi[e] = (e16)a0[8 + e];
            b1lo[e] = (e16)a1[e]; b1hi[e] = (e16)a1[8 + e];
        }
        const v8 *A = reinterpret_cast<const v8 *>(lp + (size_t)j * LP_A_ELEMS);
        v8 w_lo = A[lane], w_hi = A[64 + lane];
        const float *bb = fl + 160 + 32 * j + h * 16;
        f32x16 c0, c1;
#pragma unroll
        for (int r = 0; r < 16; ++r) { c0[r] = 0.0f; c1[r] = 0.0f; }
        if constexpr (PREC == NR_PRECISION_BF16) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w_lo, b0lo, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w_lo, b1lo, c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w_hi, b0hi, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w_hi, b1hi, c1, 0, 0, 0);
        } else {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(w_lo, b0lo, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(w_lo, b1lo, c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(w_hi, b0hi, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(w_hi, b1hi, c1, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = fmaxf(c0[r] + bb[r], 0.0f);
            a1[r] = fmaxf(c1[r] + bb[r], 0.0f);
        }
    }
    const float *wf = fl + 160 + 32 * nh + h * 16;
    const float bf = fl[160 + 32 * nh + 32];
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) { p0 = __builtin_fmaf(wf[r], a0[r], p0); p1 = __builtin_fmaf(wf[r], a1[r], p1); }
    // sum the two halves: lane (c,1) adds its partner's partial
    const float o0 = __shfl(p0, c), o1 = __shfl(p1, c);
    const float zt0 = o0 + p0 + bf, zt1 = o1 + p1 + bf;
    const float r0 = __shfl(zt0, c + 32);
    return h ? zt1 : r0;
}

__device__ __forceinline__ float mlp_wave(const MlpArgs &M, const float *s32, const uint16_t *slp, const float *sfl,
                                          int prec, float x, float y, float z, float fr) {
    if (prec == NR_PRECISION_BF16) return mlp_lowp_wave<NR_PRECISION_BF16>(slp, sfl, M.in0, M.nh, x, y, z, fr);
    if (prec == NR_PRECISION_FP16) return mlp_lowp_wave<NR_PRECISION_FP16>(slp, sfl, M.in0, M.nh, x, y, z, fr);
    return mlp_fp32_wave(s32, M.in0, M.nh, x, y, z, fr);
}

// LDS staging of the packs (block-wide, 16-byte copies)
__device__ __forceinline__ void stage(void *dst, const void *src, int bytes) {
    const int4 *s = reinterpret_cast<const int4 *>(src);
    int4 *d = reinterpret_cast<int4 *>(dst);
    for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

extern __shared__ __attribute__((aligned(16))) unsigned char nr_smem[];

struct Smem {
    float *s32;
    uint16_t *slp;
    float *sfl;
};

__device__ __forceinline__ Smem stage_mlp(const MlpArgs &M, int prec) {
    Smem S;
    S.s32 = reinterpret_cast<float *>(nr_smem);
    int b32 = M.pk_bytes;
    S.slp = reinterpret_cast<uint16_t *>(nr_smem + b32);
    S.sfl = reinterpret_cast<float *>(nr_smem + b32 + M.lp_bytes);
    stage(S.s32, M.pk, b32);
    if (prec != NR_PRECISION_FP32) {
        stage(S.slp, M.lp, M.lp_bytes);
        stage(S.sfl, M.lpf, M.lpf_bytes);
    }
    __syncthreads();
    return S;
}

// -------------------------------------------------------------- kernels

// NeuralNetwork::forward on a batch (neuralNetwork.cpp:54-63): X [n][in0] -> Y [n].
__global__ __launch_bounds__(256) void k_mlp(MlpArgs M, int prec, const float *__restrict__ X, float *__restrict__ Y,
                                             long n) {
    Smem S = stage_mlp(M, prec);
    const int lane = lane_id();
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    for (long base = wave * 64; base < n; base += nwaves * 64) {
        long i = base + lane;
        bool live = i < n;
        float x = 0, y = 0, z = 0, f = 0;
        if (live) {
            const float *p = X + i * M.in0;
            x = p[0]; y = p[1]; z = p[2];
            if (M.in0 == 4) f = p[3];
        }
        float v = mlp_wave(M, S.s32, S.slp, S.sfl, prec, x, y, z, f);
        if (live) Y[i] = v;
    }
}

// Generic dense layer, one thread per (point, output): DenseLayer::forward for any
// shape (denseLayer.cu:229-278).  W out-major [out][in].
__global__ void k_dense(const float *__restrict__ W, const float *__restrict__ b, const float *__restrict__ A,
                        float *__restrict__ Z, long n, int in, int out, int relu) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * out) return;
    long p = t / out;
    int o = (int)(t - p * out);
    const float *w = W + (long)o * in;
    const float *a = A + p * in;
    float acc = 0.0f;
    for (int k = 0; k < in; ++k) acc = __builtin_fmaf(w[k], a[k], acc);
    float v = acc + b[o];
    if (relu) v = fmaxf(v, 0.0f);
    Z[t] = v;
}

// initMarcher (:293-358) for the rows of one shard + compaction of hits.
__global__ __launch_bounds__(256) void k_init(RenderArgs A, QueueArgs Q) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long npix = (long)A.W * A.rows;
    bool hit = false;
    float4 st_p = make_float4(0, 0, 0, 0), st_d = make_float4(0, 0, 0, 0);
    if (t < npix) {
        int lr = (int)(t / A.W), x = (int)(t - (long)lr * A.W);
        int y = ((lr / A.band) * A.nshards + A.shard) * A.band + (lr % A.band);
        A.out[t] = 0u;  // caller's cudaMemset (main.cpp:408): misses and unconverged stay 0
        const float *M = A.inv_view;
        F3 o = mk3(dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 0), dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 4),
                   dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 8));
        float u = ((float)x / (float)A.W) * 2.0f - 1.0f;
        float v = ((float)y / (float)A.H) * 2.0f - 1.0f;
        F3 d = normalize3(mk3(u, v, -2.0f));
        d = mk3(dot3(d, mk3(M[0], M[1], M[2])), dot3(d, mk3(M[4], M[5], M[6])), dot3(d, mk3(M[8], M[9], M[10])));
        // intersectSphere (:199-215), bounding sphere c = 0, r = 1.2
        F3 Qv = mk3(o.x - 0.0f, o.y - 0.0f, o.z - 0.0f);
        float a = dot3(d, d);
        float b = (float)(2.0 * (double)dot3(Qv, d));
        float cc = dot3(Qv, Qv) - 1.2f * 1.2f;
        float disc = b * b - 4 * a * cc;
        if (disc > 0) {
            float sq = sqrtf(disc);
            float tnear = (float)((double)(-b - sq) / (2.0 * (double)a));
            float tfar = (float)((double)(-b + sq) / (2.0 * (double)a));
            if (tnear < 0.0f) tnear = 0.0f;
            F3 p = add3(o, mul3s(d, tnear));
            st_p = make_float4(p.x, p.y, p.z, tfar);
            st_d = make_float4(d.x, d.y, d.z, __uint_as_float((uint32_t)t));
            hit = true;
        }
    }
    uint32_t slot = wave_append(hit, Q.cnt_out);
    if (hit) { Q.p_out[slot] = st_p; Q.d_out[slot] = st_d; }
}

// One march iteration over the live queue: MLP + singleMarch (:416-477) + compaction.
__global__ __launch_bounds__(256) void k_march(RenderArgs A, MlpArgs M, QueueArgs Q, int prec, int it) {
    Smem S = stage_mlp(M, prec);
    const uint32_t n = *Q.cnt_in;
    const int lane = lane_id();
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    const bool can_shade = (it + 1) < A.max_steps;
    const float fr = (float)A.frame;
    for (long base = wave * 64; base < (long)n; base += nwaves * 64) {
        long i = base + lane;
        bool live = i < (long)n;
        float4 sp = make_float4(0, 0, 0, 0), sd = make_float4(0, 0, 0, 0);
        if (live) { sp = Q.p_in[i]; sd = Q.d_in[i]; }
        float sdf = mlp_wave(M, S.s32, S.slp, S.sfl, prec, sp.x, sp.y, sp.z, fr);
        bool alive = false, conv = false;
        F3 p = mk3(sp.x, sp.y, sp.z);
        float tfar = sp.w;
        if (live) {
            float tstep = scene_sdf(p, sdf, A.scene, sphere_zoff(A.frame));
            tfar -= tstep;
            if (tfar <= 0) {
                // background: output already 0
            } else {
                p = add3(p, mul3s(mk3(sd.x, sd.y, sd.z), tstep));
                if (tstep < MARCHING_EPSILON) conv = can_shade;  // mask = COLOR_MASK_VAL
                else alive = true;
            }
        }
        uint32_t so = wave_append(alive, Q.cnt_out);
        if (alive) { Q.p_out[so] = make_float4(p.x, p.y, p.z, tfar); Q.d_out[so] = sd; }
        uint32_t ss = wave_append(conv, Q.shade_cnt);
        if (conv) { Q.shade_p[ss] = make_float4(p.x, p.y, p.z, 0.0f); Q.shade_d[ss] = sd; }
        const uint64_t cm = __ballot(conv);
        if (cm != 0ull && lane == __ffsll((unsigned long long)cm) - 1) atomicAdd(Q.shade_it + it, 1u);
    }
}

// surfaceNormal + colour for every converged ray (16 rays x 4 tetrahedron points per wave).
__global__ __launch_bounds__(256) void k_shade(RenderArgs A, MlpArgs M, QueueArgs Q) {
    Smem S = stage_mlp(M, NR_PRECISION_FP32);
    const uint32_t n = *Q.shade_cnt;
    const int lane = lane_id();
    const int q = lane & 3;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    const float fr = (float)A.frame;
    for (long base = wave * 16; base < (long)n; base += nwaves * 16) {
        long r = base + (lane >> 2);
        bool live = r < (long)n;
        float4 sp = make_float4(0, 0, 0, 0), sd = make_float4(0, 0, 0, 0);
        if (live) { sp = Q.shade_p[r]; sd = Q.shade_d[r]; }
        F3 tp = mk3(c_tet[3 * q], c_tet[3 * q + 1], c_tet[3 * q + 2]);
        F3 pq = add3(mk3(sp.x, sp.y, sp.z), mul3s(tp, NORMAL_EPSILON));
        float sdf = mlp_fp32_wave(S.s32, M.in0, M.nh, pq.x, pq.y, pq.z, fr);
        F3 cq = mul3s(tp, scene_sdf(pq, sdf, A.scene, sphere_zoff(A.frame)));
        const int l0 = lane & ~3;
        float c1x = __shfl(cq.x, l0 + 1), c1y = __shfl(cq.y, l0 + 1), c1z = __shfl(cq.z, l0 + 1);
        float c2x = __shfl(cq.x, l0 + 2), c2y = __shfl(cq.y, l0 + 2), c2z = __shfl(cq.z, l0 + 2);
        float c3x = __shfl(cq.x, l0 + 3), c3y = __shfl(cq.y, l0 + 3), c3z = __shfl(cq.z, l0 + 3);
        if (live && q == 0) {
            F3 acc = add3(add3(add3(cq, mk3(c1x, c1y, c1z)), mk3(c2x, c2y, c2z)), mk3(c3x, c3y, c3z));
            F3 nrm = normalize3(acc);
            uint32_t pix = __float_as_uint(sd.w);
            A.out[pix] = shade_color(A, A.normal, nrm, mk3(sd.x, sd.y, sd.z));
        }
    }
}

// shards -> full frame (bands of `band` rows dealt round-robin)
__global__ void k_assemble(const uint32_t *__restrict__ src, size_t stride, uint32_t *__restrict__ dst, int W, int H,
                           int band, int nshards) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)W * H) return;
    int y = (int)(t / W), x = (int)(t - (long)y * W);
    int bidx = y / band, s = bidx % nshards;
    int lr = (bidx / nshards) * band + (y % band);
    dst[t] = src[(size_t)s * stride + (size_t)lr * W + x];
}

// ---------------------------------------------------------- launchers
int smem_bytes(const MlpArgs &M, int prec) {
    return M.pk_bytes + (prec != NR_PRECISION_FP32 ? M.lp_bytes + M.lpf_bytes : 0);
}

hipError_t launch_mlp(const MlpArgs &M, int prec, const float *X, float *Y, long n, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_mlp, dim3(grid), dim3(256), smem_bytes(M, prec), st, M, prec, X, Y, n);
    return hipGetLastError();
}
hipError_t launch_dense(const float *W, const float *b, const float *A, float *Z, long n, int in, int out, int relu,
                        hipStream_t st) {
    long tot = n * out;
    if (tot <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dense, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, W, b, A, Z, n, in, out, relu);
    return hipGetLastError();
}
hipError_t launch_init(const RenderArgs &A, const QueueArgs &Q, hipStream_t st) {
    long npix = (long)A.W * A.rows;
    if (npix <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_init, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, A, Q);
    return hipGetLastError();
}
hipError_t launch_march(const RenderArgs &A, const MlpArgs &M, const QueueArgs &Q, int prec, int it, int grid,
                        hipStream_t st) {
    hipLaunchKernelGGL(k_march, dim3(grid), dim3(256), smem_bytes(M, prec), st, A, M, Q, prec, it);
    return hipGetLastError();
}
hipError_t launch_shade(const RenderArgs &A, const MlpArgs &M, const QueueArgs &Q, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_shade, dim3(grid), dim3(256), smem_bytes(M, NR_PRECISION_FP32), st, A, M, Q);
    return hipGetLastError();
}
hipError_t launch_assemble(const uint32_t *src, size_t stride, uint32_t *dst, int W, int H, int band, int nshards,
                           hipStream_t st) {
    long tot = (long)W * H;
    if (tot <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_assemble, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, src, stride, dst, W, H, band,
                       nshards);
    return hipGetLastError();
}

}  // namespace nr
