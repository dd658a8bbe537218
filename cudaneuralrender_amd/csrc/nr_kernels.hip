// nr_kernels.hip -- gfx950 (CDNA4) queue kernels of the neural-SDF sphere tracer.
//
// Hot path of the reference (daviesthomas/cudaNeuralRender @ v1):
//   src/volumeRender_kernel.cu:608-692 render loop, with the per-iteration
//   nn.forward (:661 -> src/layers/denseLayer.cu:126-176, 9 CUTLASS launches) and
//   singleMarch (:416-477), plus a full-image exclusive scan + 4-byte D2H sync per
//   iteration (:549-576).
// This file holds the two schedules that keep the rays in a queue in HBM (the
// persistent one-launch tracer is nr_trace.hip):
//   * wavefront (k_init_f / k_march16 / k_shade16): ONE launch per iteration over a
//     segmented, block-aggregated ray queue of one frame or of up to 32; the whole MLP
//     runs per wave on the matrix cores (nr_mlp16.h), no activation buffers, no scans,
//     no host sync;
//   * layered (k_init_l / k_dense* / k_march_l / k_shade_l): the reference's structure
//     for networks of any shape -- one dense-layer launch per layer per iteration,
//     replayed as a hipGraph.
// Plus the generic dense layers (DenseLayer::forward for any shape) and k_assemble.
//
// Numerics: compiled with -ffp-contract=off.  FP32 mode is bit-exact with the CPU
// oracle: v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain (cdna_hip_programming.md
// §3), so the packs and the dense kernels order k ascending, exactly the oracle's loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nr_mlp16.h"

namespace nr {

// -------------------------------------------------------------- kernels

// Generic dense layer, one thread per (point, output): DenseLayer::forward for any
// shape (denseLayer.cu:229-278).  W out-major [out][in], staged in LDS with rows padded
// to in + 1 floats (lanes of a wave read consecutive rows) when it fits.  The point
// count is D.n, or read from the device (D.count x D.count_mul) when the points are a
// ray queue whose length the host does not know; the launch covers points
// [chunk0, chunk0 + chunk_n) of it.  SRC: 0 = rows of D.A (chunk-local), 1 = the live
// rays' positions (+ the frame number as a 4th input), 2 = the four tetrahedron points
// of each converged ray (surfaceNormal, :361-377).  Arithmetic: ascending-k fmaf chain,
// then + bias, then ReLU (the fused kernels' and the oracle's order).
template <int SRC>
__global__ __launch_bounds__(256) void k_dense(DenseArgs D) {
    extern __shared__ float sw[];
    const long n = D.count ? (long)(*D.count) * D.count_mul : D.n;
    const long nc = min(n - D.chunk0, D.chunk_n);
    if (nc <= 0) return;  // uniform over the block
    const int in = D.in, out = D.out;
    const float *W = D.W;
    int ws = in;
    if (D.lds) {
        ws = in + 1;
        for (int i = threadIdx.x; i < in * out; i += blockDim.x) sw[(i / in) * ws + i % in] = D.W[i];
        __syncthreads();
        W = sw;
    }
    float fr = 0.0f;
    if constexpr (SRC != 0) fr = (float)D.args->frame;
    const long tot = nc * out;
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (long)gridDim.x * blockDim.x) {
        const long p = t / out;
        const int o = (int)(t - p * out);
        const float *w = W + o * ws;
        float acc = 0.0f;
        if constexpr (SRC == 0) {
            const float *a = D.A + p * in;
            for (int k = 0; k < in; ++k) acc = __builtin_fmaf(w[k], a[k], acc);
        } else {
            float x, y, z;
            if constexpr (SRC == 1) {
                const float4 sp = D.pts[D.chunk0 + p];
                x = sp.x; y = sp.y; z = sp.z;
            } else {
                const long i = D.chunk0 + p;
                const float4 sp = D.pts[i >> 2];
                const int q = (int)(i & 3);
                const F3 pq = add3(mk3(sp.x, sp.y, sp.z),
                                   mul3s(mk3(c_tet[3 * q], c_tet[3 * q + 1], c_tet[3 * q + 2]), NORMAL_EPSILON));
                x = pq.x; y = pq.y; z = pq.z;
            }
            const float a4[4] = {x, y, z, fr};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < in) acc = __builtin_fmaf(w[k], a4[k], acc);
        }
        float v = acc + D.b[o];
        if (D.relu) v = fmaxf(v, 0.0f);
        D.Z[t] = v;
    }
}

// The first layer (in <= 4) on the matrix cores, for out >= 16.  v_mfma_f32_16x16x4_f32 is an
// ascending-k fmaf chain over its four k (lane group g feeds k0 + g) accumulated onto C,
// so one instruction per 4-k step, k0 = 0, 4, ..., gives every output exactly k_dense's
// chain; k >= in is padded with zero weights AND zero activations (the fma then adds
// +0 to a chain that is never -0).  A wave computes 32 outputs x 64 points (2 x 4
// tiles) from the ray queues' positions (SRC 1 / 2, see k_dense).
typedef float dense_f32x4 __attribute__((ext_vector_type(4)));
template <int SRC>
__global__ __launch_bounds__(256) void k_dense_mfma(DenseArgs D) {
    const long n = D.count ? (long)(*D.count) * D.count_mul : D.n;
    const long nc = min(n - D.chunk0, D.chunk_n);
    if (nc <= 0) return;
    const int in = D.in, out = D.out;
    const int lane = lane_id(), j = lane & 15, g = lane >> 4;
    const int oblocks = (out + 31) >> 5;
    const long units = ((nc + 63) >> 6) * oblocks;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    float fr = 0.0f;
    if constexpr (SRC != 0) fr = (float)D.args->frame;
    for (long u = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; u < units; u += nwaves) {
        const long pb = u / oblocks;
        const int o0 = (int)(u - pb * oblocks) * 32;
        const long p0 = pb * 64;
        dense_f32x4 c[2][4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int t = 0; t < 4; ++t) c[mt][t] = dense_f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const float *wrow[2];
        bool wok[2], pok[4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            wok[mt] = o0 + 16 * mt + j < out;
            wrow[mt] = D.W + (long)(wok[mt] ? o0 + 16 * mt + j : 0) * in;
        }
        {
            // layer 0: in <= 4, one k-step; lane (j, g) feeds input g of point j
            float w[2], a[4];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) w[mt] = (g < in && wok[mt]) ? wrow[mt][g] : 0.0f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const long p = p0 + 16 * t + j;
                pok[t] = p < nc;
                float x = 0.0f, y = 0.0f, z = 0.0f;
                if (pok[t]) {
                    if constexpr (SRC == 1) {
                        const float4 sp = D.pts[D.chunk0 + p];
                        x = sp.x; y = sp.y; z = sp.z;
                    } else {
                        const long i = D.chunk0 + p;
                        const float4 sp = D.pts[i >> 2];
                        const int q = (int)(i & 3);
                        const F3 pq = add3(mk3(sp.x, sp.y, sp.z),
                                           mul3s(mk3(c_tet[3 * q], c_tet[3 * q + 1], c_tet[3 * q + 2]), NORMAL_EPSILON));
                        x = pq.x; y = pq.y; z = pq.z;
                    }
                }
                const float v = g == 0 ? x : (g == 1 ? y : (g == 2 ? z : fr));
                a[t] = (g < in && pok[t]) ? v : 0.0f;
            }
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    c[mt][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mt], a[t], c[mt][t], 0, 0, 0);
        }
        // lane (j, g), register r: output o0 + 16 mt + 4 g + r of point p0 + 16 t + j
        const bool zvec = (out & 3) == 0 && ((uintptr_t)D.Z & 15) == 0;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const int o = o0 + 16 * mt + 4 * g;
            float bias[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bias[r] = o + r < out ? D.b[o + r] : 0.0f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (!pok[t]) continue;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = c[mt][t][r] + bias[r];
                    if (D.relu) v[r] = fmaxf(v[r], 0.0f);
                }
                float *zp = D.Z + (p0 + 16 * t + j) * (long)out + o;
                if (zvec && o + 3 < out) {
                    *reinterpret_cast<float4 *>(zp) = make_float4(v[0], v[1], v[2], v[3]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (o + r < out) zp[r] = v[r];
                }
            }
        }
    }
}

// Hidden layers (rows of D.A, out >= 16) on the matrix cores, LDS-tiled: a block
// computes 64 outputs x 128 points; per 32-k chunk it stages the activation tile
// [128][32] and the weight tile [64][32] (rows padded to 36 floats: the fragment reads
// of 16 rows x 4 consecutive k hit 64 distinct banks) with coalesced float4 loads, then
// each wave (32 outputs x 64 points) runs 8 k-steps of 2 x 4 v_mfma_f32_16x16x4_f32 in
// ascending k.  Zero padding past `in` / `out` / the chunk end as in k_dense_mfma.
constexpr int DT_P = 128, DT_O = 64, DT_K = 32, DT_S = 36;
__device__ __forceinline__ void dense_stage(float *__restrict__ dst, const float *__restrict__ src, long rows_ok,
                                            long row0, int ld, int kc, int nrows) {
    // nrows x DT_K floats from src[(row0 + r) * ld + kc + c] into dst[r * DT_S + c]
    const bool vec = (ld & 3) == 0 && ((uintptr_t)src & 15) == 0;
    for (int i = threadIdx.x; i < nrows * (DT_K / 4); i += blockDim.x) {
        const int r = i >> 3, c = (i & 7) * 4;
        const long row = row0 + r;
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (row < rows_ok) {
            const float *q = src + row * (long)ld + kc + c;
            if (vec && kc + c + 3 < ld) {
                v = *reinterpret_cast<const float4 *>(q);
            } else {
                v.x = kc + c < ld ? q[0] : 0.0f;
                v.y = kc + c + 1 < ld ? q[1] : 0.0f;
                v.z = kc + c + 2 < ld ? q[2] : 0.0f;
                v.w = kc + c + 3 < ld ? q[3] : 0.0f;
            }
        }
        *reinterpret_cast<float4 *>(dst + r * DT_S + c) = v;
    }
}
__global__ __launch_bounds__(256) void k_dense_tiled(DenseArgs D) {
    __shared__ __attribute__((aligned(16))) float sA[DT_P * DT_S];
    __shared__ __attribute__((aligned(16))) float sW[DT_O * DT_S];
    const long n = D.count ? (long)(*D.count) * D.count_mul : D.n;
    const long nc = min(n - D.chunk0, D.chunk_n);
    if (nc <= 0) return;
    const int in = D.in, out = D.out;
    const int lane = lane_id(), j = lane & 15, g = lane >> 4;
    const int wv = threadIdx.x >> 6, wo = (wv & 1) * 32, wp = (wv >> 1) * 64;
    const int oblocks = (out + DT_O - 1) / DT_O;
    const long tiles = ((nc + DT_P - 1) / DT_P) * oblocks;
    for (long tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const long pb = tile / oblocks;
        const int o0 = (int)(tile - pb * oblocks) * DT_O;
        const long p0 = pb * DT_P;
        dense_f32x4 c[2][4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int t = 0; t < 4; ++t) c[mt][t] = dense_f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        for (int kc = 0; kc < in; kc += DT_K) {
            __syncthreads();  // previous chunk's fragment reads are done
            dense_stage(sA, D.A + p0 * (long)in, nc - p0, 0, in, kc, DT_P);
            dense_stage(sW, D.W + (long)o0 * in, out - o0, 0, in, kc, DT_O);
            __syncthreads();
#pragma unroll
            for (int ks = 0; ks < DT_K / 4; ++ks) {
                float w[2], a[4];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) w[mt] = sW[(wo + 16 * mt + j) * DT_S + 4 * ks + g];
#pragma unroll
                for (int t = 0; t < 4; ++t) a[t] = sA[(wp + 16 * t + j) * DT_S + 4 * ks + g];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        c[mt][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[mt], a[t], c[mt][t], 0, 0, 0);
            }
        }
        const bool zvec = (out & 3) == 0 && ((uintptr_t)D.Z & 15) == 0;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const int o = o0 + wo + 16 * mt + 4 * g;
            float bias[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bias[r] = o + r < out ? D.b[o + r] : 0.0f;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const long p = p0 + wp + 16 * t + j;
                if (p >= nc) continue;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = c[mt][t][r] + bias[r];
                    if (D.relu) v[r] = fmaxf(v[r], 0.0f);
                }
                float *zp = D.Z + p * (long)out + o;
                if (zvec && o + 3 < out) {
                    *reinterpret_cast<float4 *>(zp) = make_float4(v[0], v[1], v[2], v[3]);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (o + r < out) zp[r] = v[r];
                }
            }
        }
    }
}

// The one-output layer (the SDF) over rows of D.A: one lane per point runs the whole
// ascending-k fmaf chain, reading its row from an LDS tile [256][32] (row stride 33:
// the 64 lanes' scalar reads hit distinct banks) staged with coalesced loads.
__global__ __launch_bounds__(256) void k_dense_col(DenseArgs D) {
    __shared__ float sA[256 * 33];
    const long n = D.count ? (long)(*D.count) * D.count_mul : D.n;
    const long nc = min(n - D.chunk0, D.chunk_n);
    if (nc <= 0) return;
    const int in = D.in;
    const float b = D.b[0];
    for (long p0 = (long)blockIdx.x * 256; p0 < nc; p0 += (long)gridDim.x * 256) {
        const long p = p0 + threadIdx.x;
        float acc = 0.0f;
        for (int kc = 0; kc < in; kc += 32) {
            __syncthreads();
            for (int i = threadIdx.x; i < 256 * 32; i += 256) {
                const int r = i >> 5, k = i & 31;
                const long row = p0 + r;
                sA[r * 33 + k] = (row < nc && kc + k < in) ? D.A[row * (long)in + kc + k] : 0.0f;
            }
            __syncthreads();
            const int kn = min(32, in - kc);
            for (int k = 0; k < kn; ++k) acc = __builtin_fmaf(D.W[kc + k], sA[threadIdx.x * 33 + k], acc);
        }
        float v = acc + b;
        if (D.relu) v = fmaxf(v, 0.0f);
        if (p < nc) D.Z[p] = v;
    }
}

// initMarcher (:293-358) for pixel t of the shard, camera M (3x4): the ray's queue
// entry {p, tfar}, {d, -} if it hits the bounding sphere.
__device__ __forceinline__ bool gen_hit(const RenderArgs &A, const float *M, long t, float4 &st_p, float4 &st_d) {
    const int lr = (int)udiv_r((uint32_t)t, (uint32_t)A.W, A.inv_w), x = (int)t - lr * A.W;
    const int bi = (int)udiv_r((uint32_t)lr, (uint32_t)A.band, A.inv_band);
    const int y = (bi * A.nshards + A.shard) * A.band + (lr - bi * A.band);
    F3 o = mk3(dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 0), dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 4),
               dot4(0.0f, 0.0f, 0.0f, 1.0f, M + 8));
    float u = pixel_uv(x, A.W, A.rcp_w);
    float v = pixel_uv(y, A.H, A.rcp_h);
    F3 d = normalize3(mk3(u, v, -2.0f));
    d = mk3(dot3(d, mk3(M[0], M[1], M[2])), dot3(d, mk3(M[4], M[5], M[6])), dot3(d, mk3(M[8], M[9], M[10])));
    // intersectSphere (:199-215), bounding sphere c = 0, r = 1.2
    float tnear, tfar;
    if (!intersect_bounding(o, d, tnear, tfar)) return false;
    if (tnear < 0.0f) tnear = 0.0f;
    F3 p = add3(o, mul3s(d, tnear));
    st_p = make_float4(p.x, p.y, p.z, tfar);
    st_d = make_float4(d.x, d.y, d.z, 0.0f);
    return true;
}

// one pixel per thread (block-uniform), hits appended to the queue tagged with the pixel
__device__ __forceinline__ void init_rays(const RenderArgs &A, const QueueArgs &Q) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long npix = (long)A.W * A.rows;
    bool hit = false;
    float4 st_p = make_float4(0, 0, 0, 0), st_d = make_float4(0, 0, 0, 0);
    if (t < npix) {
        A.out[t] = 0u;  // caller's cudaMemset (main.cpp:408): misses and unconverged stay 0
        hit = gen_hit(A, A.inv_view, t, st_p, st_d);
        st_d.w = __uint_as_float((uint32_t)t);
    }
    const Slots sl = block_append2(hit, Q.cnt_out, false, nullptr);
    if (hit) { Q.p_out[sl.a] = st_p; Q.d_out[sl.a] = st_d; }
}
__global__ __launch_bounds__(256) void k_init_l(const RenderArgs *__restrict__ Ad, QueueArgs Q) { init_rays(*Ad, Q); }

// singleMarch (:416-477) for one block of queue entries given their SDFs, + compaction
// (block-uniform: every thread of the block calls it).
__device__ __forceinline__ void march_rays(const RenderArgs &A, const QueueArgs &Q, int it, bool live, float4 sp,
                                           float4 sd, float sdf, double zoff) {
    const bool can_shade = (it + 1) < A.max_steps;
    bool alive = false, conv = false;
    F3 p = mk3(sp.x, sp.y, sp.z);
    float tfar = sp.w;
    if (live) {
        float tstep = scene_sdf(p, sdf, A.scene, zoff);
        tfar -= tstep;
        if (tfar <= 0) {
            // background: output already 0
        } else {
            p = add3(p, mul3s(mk3(sd.x, sd.y, sd.z), tstep));
            if (tstep < MARCHING_EPSILON) conv = can_shade;  // mask = COLOR_MASK_VAL
            else alive = true;
        }
    }
    const Slots sl = block_append2(alive, Q.cnt_out, conv, Q.shade_cnt);
    if (alive) { Q.p_out[sl.a] = make_float4(p.x, p.y, p.z, tfar); Q.d_out[sl.a] = sd; }
    if (conv) { Q.shade_p[sl.b] = make_float4(p.x, p.y, p.z, 0.0f); Q.shade_d[sl.b] = sd; }
    if (threadIdx.x == 0 && sl.nb != 0) Q.shade_it[it] = 1u;  // a flag: plain stores, no atomic
}

// surfaceNormal (:361-377) + colour: lane (ray, q) holds tetrahedron point q's SDF.
__device__ __forceinline__ void shade_rays(const RenderArgs &A, const float *nm, uint32_t *out, double zoff, bool live,
                                           float4 sp, float4 sd, uint32_t pix, float sdf) {
    const int lane = lane_id(), q = lane & 3;
    F3 tp = mk3(c_tet[3 * q], c_tet[3 * q + 1], c_tet[3 * q + 2]);
    F3 pq = add3(mk3(sp.x, sp.y, sp.z), mul3s(tp, NORMAL_EPSILON));
    F3 cq = mul3s(tp, scene_sdf(pq, sdf, A.scene, zoff));
    const F3 c1 = quad_bcast3_1(cq), c2 = quad_bcast3_2(cq), c3 = quad_bcast3_3(cq);
    if (live && q == 0) {
        F3 acc = add3(add3(add3(cq, c1), c2), c3);
        F3 nrm = normalize3(acc);
        out[pix] = shade_color(A, nm, nrm, mk3(sd.x, sd.y, sd.z));
    }
}

// One march iteration over the live queue: MLP + singleMarch (:416-477) + compaction.
// Layered schedule: the same step with the SDFs the dense-layer chain left in sdf[].
__global__ __launch_bounds__(256) void k_march_l(const RenderArgs *__restrict__ Ad, QueueArgs Q,
                                                 const float *__restrict__ sdf, int it) {
    const uint32_t n = *Q.cnt_in;
    for (long base = (long)blockIdx.x * blockDim.x; base < (long)n; base += (long)gridDim.x * blockDim.x) {
        long i = base + threadIdx.x;
        bool live = i < (long)n;
        float4 sp = make_float4(0, 0, 0, 0), sd = make_float4(0, 0, 0, 0);
        float v = 0.0f;
        if (live) { sp = Q.p_in[i]; sd = Q.d_in[i]; v = sdf[i]; }
        march_rays(*Ad, Q, it, live, sp, sd, v, sphere_zoff(Ad->frame));
    }
}

// surfaceNormal + colour for every converged ray (16 rays x 4 tetrahedron points per wave).
// Layered schedule: colour the converged rays from the tetrahedron SDFs in sdf4[4 r + q].
__global__ __launch_bounds__(256) void k_shade_l(const RenderArgs *__restrict__ Ad, QueueArgs Q,
                                                 const float *__restrict__ sdf4) {
    const uint32_t n = *Q.shade_cnt;
    const int lane = lane_id();
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    for (long base = wave * 16; base < (long)n; base += nwaves * 16) {
        long r = base + (lane >> 2);
        bool live = r < (long)n;
        float4 sp = make_float4(0, 0, 0, 0), sd = make_float4(0, 0, 0, 0);
        float v = 0.0f;
        if (live) { sp = Q.shade_p[r]; sd = Q.shade_d[r]; v = sdf4[4 * r + (lane & 3)]; }
        shade_rays(*Ad, Ad->normal, Ad->out, sphere_zoff(Ad->frame), live, sp, sd, __float_as_uint(sd.w), v);
    }
}

// ------------------------------------ wavefront schedule on the 16-point-tile MLP
// One queue holds the rays of one frame or of up to 32 (nr_render_batch): entry
// {x, y, z, tfar}, {dx, dy, dz, tag}, tag = pixel | frame << WF_FSHIFT; a ray's camera,
// sphere offset, 4th network input and output image come from F[frame].  The queue is
// split into WF_SEGS segments of seg_cap entries with a counter each: pixel t starts in
// segment t / seg_cap and its ray stays there (survivors and converged rays of a
// segment never outnumber its pixels), so the appends of a block go to one of 8
// counters on their own cache lines instead of all to one (same-address atomics
// serialise at ~10 ns; 32 frames = 131k appending blocks per iteration).
constexpr int WF_FSHIFT = 27;
constexpr uint32_t WF_PMASK = (1u << WF_FSHIFT) - 1u;
constexpr int WF_CSTRIDE = 32;  // counters of one iteration: WF_SEGS x 128-byte lines

// the view of segment s of a segmented queue
__device__ __forceinline__ QueueArgs seg_view(const QueueArgs &Q, int s) {
    QueueArgs V = Q;
    V.cnt_out = Q.cnt_out + s * WF_CSTRIDE;
    V.p_out = Q.p_out + s * Q.seg_cap;
    V.d_out = Q.d_out + s * Q.seg_cap;
    V.shade_cnt = Q.shade_cnt + s * WF_CSTRIDE;
    V.shade_p = Q.shade_p + s * Q.seg_cap;
    V.shade_d = Q.shade_d + s * Q.seg_cap;
    V.fcnt = Q.fcnt + s * WF_CSTRIDE;
    V.fp = Q.fp + s * Q.seg_cap;
    V.fd = Q.fd + s * Q.seg_cap;
    return V;
}

// work unit u (of `per`-entry chunks over the segments' counts) -> segment, entry offset
__device__ __forceinline__ bool seg_unit(const uint32_t *cnt, long u, int per, int &s, long &off, long &n_s) {
    for (s = 0; s < WF_SEGS; ++s) {
        n_s = cnt[s * WF_CSTRIDE];
        const long units = (n_s + per - 1) / per;
        if (u < units) { off = u * per; return true; }
        u -= units;
    }
    return false;
}
__device__ __forceinline__ long seg_units(const uint32_t *cnt, int per) {
    long U = 0;
    for (int s = 0; s < WF_SEGS; ++s) U += ((long)cnt[s * WF_CSTRIDE] + per - 1) / per;
    return U;
}

__global__ __launch_bounds__(256) void k_init_f(RenderArgs A, const FrameArgs *__restrict__ F, QueueArgs Q, long npix,
                                                long total, double inv_npix) {
    // grid-stride over 256-pixel chunks: a 32-frame batch has 131 k of them, and
    // dispatching one workgroup per chunk cost ~1 ms
    for (long c0 = (long)blockIdx.x * blockDim.x; c0 < total; c0 += (long)gridDim.x * blockDim.x) {
        const long t = c0 + threadIdx.x;
        bool hit = false;
        float4 st_p = make_float4(0, 0, 0, 0), st_d = make_float4(0, 0, 0, 0);
        if (t < total) {
            const int f = (int)udiv_r((uint32_t)t, (uint32_t)npix, inv_npix);
            const long px = t - (long)f * npix;
            F[f].out[px] = 0u;
            hit = gen_hit(A, F[f].inv_view, px, st_p, st_d);
            st_d.w = __uint_as_float((uint32_t)px | ((uint32_t)f << WF_FSHIFT));
        }
        // seg_cap is a multiple of the block size: the chunk's pixels share a segment
        const QueueArgs V = seg_view(Q, (int)(c0 / Q.seg_cap));
        const Slots sl = block_append2(hit, V.cnt_out, false, nullptr);
        if (hit) { V.p_out[sl.a] = st_p; V.d_out[sl.a] = st_d; }
    }
}

// One iteration over the queue: 64 rays per wave through mlp16 (4 x 16-point tiles, the
// k_trace / k_mlp16 MLP), then the step and the block-aggregated compaction into the
// ray's segment.  Blocks take 256-ray work units over the segments, grid-stride.
// The endgame (round 6, bf16/fp16; nr_set_endgame, the persistent tracer's EG rule restated on
// queues): MODE 1 = the coarse pass -- a ray whose 16-bit MLP output is below Q.eg_tau goes,
// unstepped, to this iteration's fine queue; MODE 2 = the fine pass over that queue -- the fp32x3
// MLP on every point (mlp16_x3_normal: the split within the x3 pack's bounds, the fp32 MLP
// outside), then the same step, survivors to the next iteration's fine queue.  So every ray takes
// one step per iteration, the switch iteration's and all later ones in fp32x3, as in k_trace and
// the oracle (or_set_endgame).
template <int PREC, int MODE = 0>
__global__ __launch_bounds__(256) void k_march16(RenderArgs A, MlpArgs M, QueueArgs Q, const FrameArgs *__restrict__ F,
                                                 int it) {
    Smem16 S = stage16<PREC, false>(M);
    const int wv = threadIdx.x >> 6;
    const long U = seg_units(Q.cnt_in, 256);
    for (long u = blockIdx.x; u < U; u += gridDim.x) {
        int s;
        long off, n_s;
        seg_unit(Q.cnt_in, u, 256, s, off, n_s);
        const long i = off + threadIdx.x;
        const bool live = i < n_s;
        float4 sp = make_float4(0, 0, 0, 0), sd = make_float4(0, 0, 0, 0);
        if (live) { sp = Q.p_in[s * Q.seg_cap + i]; sd = Q.d_in[s * Q.seg_cap + i]; }
        const int f = live ? (int)(__float_as_uint(sd.w) >> WF_FSHIFT) : 0;
        const long rem = n_s - (off + 64 * wv);
        const uint32_t tmask = rem >= 64 ? 0xfu : (rem <= 0 ? 0u : (1u << ((rem + 15) >> 4)) - 1u);
        float sdf = 0.0f;
        if constexpr (MODE == 2) {
            if (tmask) sdf = mlp16_x3_normal<false>(M, S.s32, M.x3lp, M.x3fl, F[f].frame_f, sp.x, sp.y, sp.z, tmask);
        } else {
            if (tmask) sdf = mlp16(M, S.s32, S.slp, S.sfl, PREC, F[f].frame_f, sp.x, sp.y, sp.z, tmask, M.lp_clamp != 0);
        }
        const QueueArgs V = seg_view(Q, s);
        if constexpr (MODE == 1) {
            const bool sw = live && sdf < Q.eg_tau;
            march_rays(A, V, it, live && !sw, sp, sd, sdf, F[f].zoff);
            const Slots sl = block_append2(sw, V.fcnt, false, nullptr);
            if (sw) { V.fp[sl.a] = sp; V.fd[sl.a] = sd; }
            if (threadIdx.x == 0 && sl.na) atomicAdd(Q.fsw, sl.na);
        } else {
            march_rays(A, V, it, live, sp, sd, sdf, F[f].zoff);
        }
    }
}

// surfaceNormal + colour for the converged rays of the queue's frames: 16 rays x 4
// tetrahedron points per wave, one fp32 4-tile mlp16 pass.
__global__ __launch_bounds__(256) void k_shade16(RenderArgs A, MlpArgs M, QueueArgs Q, const FrameArgs *__restrict__ F) {
    Smem16 S = stage16<NR_PRECISION_FP32, true>(M);
    const int lane = lane_id(), q = lane & 3;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
    const long U = seg_units(Q.shade_cnt, 16);
    for (long u = wave; u < U; u += nwaves) {
        int s;
        long off, n_s;
        seg_unit(Q.shade_cnt, u, 16, s, off, n_s);
        const long r = off + (lane >> 2);
        const bool live = r < n_s;
        float4 sp = make_float4(0, 0, 0, 0), sd = make_float4(0, 0, 0, 0);
        if (live) { sp = Q.shade_p[s * Q.seg_cap + r]; sd = Q.shade_d[s * Q.seg_cap + r]; }
        const uint32_t tag = __float_as_uint(sd.w);
        const int f = live ? (int)(tag >> WF_FSHIFT) : 0;
        const F3 tp = mk3(c_tet[3 * q], c_tet[3 * q + 1], c_tet[3 * q + 2]);
        const F3 pq = add3(mk3(sp.x, sp.y, sp.z), mul3s(tp, NORMAL_EPSILON));
        const long rem = n_s - off;  // rays; 4 per 16-point tile
        const uint32_t tmask = rem >= 16 ? 0xfu : (1u << ((rem + 3) >> 2)) - 1u;
        // bf16/fp16: the normals in fp32x3 (M.x3n), as the persistent tracer's
        const float sdf = M.x3n
                              ? mlp16_x3_normal(M, S.s32, M.x3lp, M.x3fl, F[f].frame_f, pq.x, pq.y, pq.z, tmask)
                              : mlp16_fp32(M, S.s32, F[f].frame_f, pq.x, pq.y, pq.z, tmask);
        shade_rays(A, F[f].normal, F[f].out, F[f].zoff, live, sp, sd, tag & WF_PMASK, sdf);
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

int dense_lds_bytes(int in, int out) {
    const long b = (long)out * (in + 1) * 4;
    return b <= 64 * 1024 ? (int)b : 0;
}
hipError_t launch_dense(const DenseArgs &D0, int src, int grid, hipStream_t st) {
    DenseArgs D = D0;
    if (src == 0 && D.out >= 16) {  // LDS-tiled matrix-core layer, grid-stride over 64 x 128 tiles
        hipLaunchKernelGGL(k_dense_tiled, dim3(grid), dim3(256), 0, st, D);
        return hipGetLastError();
    }
    if (src == 0 && D.out == 1) {
        hipLaunchKernelGGL(k_dense_col, dim3(grid), dim3(256), 0, st, D);
        return hipGetLastError();
    }
    if (D.out >= 16) {  // first layer on the matrix cores: 32-output x 64-point wave units
        if (src == 1) hipLaunchKernelGGL(k_dense_mfma<1>, dim3(grid), dim3(256), 0, st, D);
        else hipLaunchKernelGGL(k_dense_mfma<2>, dim3(grid), dim3(256), 0, st, D);
        return hipGetLastError();
    }
    const int lds = dense_lds_bytes(D.in, D.out);
    D.lds = lds > 0;
    if (src == 0) hipLaunchKernelGGL(k_dense<0>, dim3(grid), dim3(256), lds, st, D);
    else if (src == 1) hipLaunchKernelGGL(k_dense<1>, dim3(grid), dim3(256), lds, st, D);
    else hipLaunchKernelGGL(k_dense<2>, dim3(grid), dim3(256), lds, st, D);
    return hipGetLastError();
}
__global__ void k_set_args(RenderArgs A, RenderArgs *d) {
    if (threadIdx.x == 0) *d = A;
}
hipError_t launch_set_args(const RenderArgs &A, RenderArgs *d, hipStream_t st) {
    hipLaunchKernelGGL(k_set_args, dim3(1), dim3(64), 0, st, A, d);
    return hipGetLastError();
}
hipError_t launch_init_l(const RenderArgs *Ad, const QueueArgs &Q, long npix, hipStream_t st) {
    if (npix <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_init_l, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, Ad, Q);
    return hipGetLastError();
}
hipError_t launch_march_l(const RenderArgs *Ad, const QueueArgs &Q, const float *sdf, int it, int grid,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_march_l, dim3(grid), dim3(256), 0, st, Ad, Q, sdf, it);
    return hipGetLastError();
}
hipError_t launch_shade_l(const RenderArgs *Ad, const QueueArgs &Q, const float *sdf4, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_shade_l, dim3(grid), dim3(256), 0, st, Ad, Q, sdf4);
    return hipGetLastError();
}
hipError_t launch_init_f(const RenderArgs &A, const FrameArgs *F, const QueueArgs &Q, long npix, long total,
                         int grid, hipStream_t st) {
    if (total <= 0) return hipSuccess;
    grid = (int)std::max<long>(1, std::min<long>((total + 255) / 256, grid));
    hipLaunchKernelGGL(k_init_f, dim3(grid), dim3(256), 0, st, A, F, Q, npix, total, 1.0 / (double)npix);
    return hipGetLastError();
}
hipError_t launch_march16(const RenderArgs &A, const MlpArgs &M, const QueueArgs &Q, const FrameArgs *F, int prec,
                          int it, int grid, hipStream_t st, int mode) {
    const int sm = smem16_bytes(M, prec, false);
    if (mode == 1 && prec == NR_PRECISION_BF16)
        hipLaunchKernelGGL((k_march16<NR_PRECISION_BF16, 1>), dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else if (mode == 1 && prec == NR_PRECISION_FP16)
        hipLaunchKernelGGL((k_march16<NR_PRECISION_FP16, 1>), dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else if (mode == 2 && prec == NR_PRECISION_BF16)
        hipLaunchKernelGGL((k_march16<NR_PRECISION_BF16, 2>), dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else if (mode == 2 && prec == NR_PRECISION_FP16)
        hipLaunchKernelGGL((k_march16<NR_PRECISION_FP16, 2>), dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else if (prec == NR_PRECISION_BF16)
        hipLaunchKernelGGL(k_march16<NR_PRECISION_BF16>, dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else if (prec == NR_PRECISION_FP16)
        hipLaunchKernelGGL(k_march16<NR_PRECISION_FP16>, dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else if (prec == NR_PRECISION_FP32X3)
        hipLaunchKernelGGL(k_march16<NR_PRECISION_FP32X3>, dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    else
        hipLaunchKernelGGL(k_march16<NR_PRECISION_FP32>, dim3(grid), dim3(256), sm, st, A, M, Q, F, it);
    return hipGetLastError();
}
hipError_t launch_shade16(const RenderArgs &A, const MlpArgs &M, const QueueArgs &Q, const FrameArgs *F, int grid,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_shade16, dim3(grid), dim3(256), smem16_bytes(M, NR_PRECISION_FP32, true), st, A, M, Q, F);
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
