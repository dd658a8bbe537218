// nr_mlp16.h -- the MLP on 16-point MFMA tiles (v_mfma_f32_16x16x4_f32 for fp32,
// v_mfma_f32_16x16x32_{bf16,f16} for reduced precision).
//
// A wave holds 64 points, point p in lane p.  They form 4 tiles of 16 points
// (tile t = points 16t..16t+15); inside a tile lane (j, g) = (lane & 15, lane >> 4)
// holds point j and 8 of the 32 hidden units (group g).  Only tiles whose bit is set
// in `tmask` are computed (wave-uniform), so a wave with few live rays pays for
// ceil(live/16) tiles, not 4 -- the granularity that keeps the tail of the march short.
//
// FP32 numerics: the f32 MFMA is a k-ordered fmaf chain (cdna_hip_programming.md §3);
// the pack (nr_pack.cpp, pack_fp32_16) permutes hidden units so that each dot product
// runs over k = 0..31 in ascending order from +0, then adds the bias -- bit-for-bit the
// reference dense layer as restated by the oracle (denseLayer.cu:126-176).
#pragma once
#include "nr_device.h"

namespace nr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// z_t lives in lane (j, 3) = 48 + j of tile t; point p = 16t + j gets it back in lane p.
__device__ __forceinline__ float tile_outputs(const float zt[4]) {
    const int lane = lane_id(), j = lane & 15, t = lane >> 4;
    float r0 = __shfl(zt[0], 48 + j), r1 = __shfl(zt[1], 48 + j);
    float r2 = __shfl(zt[2], 48 + j), r3 = __shfl(zt[3], 48 + j);
    return t == 0 ? r0 : (t == 1 ? r1 : (t == 2 ? r2 : r3));
}

// FP32 MLP on NT active tiles (tiles 0..NT-1; the caller keeps live points there).
// PART != 0 only in the latency diagnostic (nr_diag.hip): stop after the hidden layers.
template <int NT, int PART = 0>
__device__ __forceinline__ float mlp16_fp32_nt(const float *__restrict__ s, int in0, int nh, float fr, float x,
                                               float y, float z) {
    // fr: this lane's 4th input (the frame number when rendering; used iff in0 == 4)
    const int lane = lane_id(), g = lane >> 4, j = lane & 15;
    float a[NT][8];
    f32x4 c[NT][2];
    // layer 0 on the matrix core too: K = in0 padded to 4 (weight 0 for the pad, whose
    // fma adds +0 to a chain that can never be -0), one v_mfma_f32_16x16x4_f32 per
    // row tile.  Lane (j, g) feeds input g of point j.
    {
        const float w0 = s[PK_L0W + lane], w1 = s[PK_L0W + 64 + lane];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float px = __shfl(x, 16 * t + j), py = __shfl(y, 16 * t + j), pz = __shfl(z, 16 * t + j);
            const float pw = in0 == 4 ? __shfl(fr, 16 * t + j) : 0.0f;
            const float b = g == 0 ? px : (g == 1 ? py : (g == 2 ? pz : pw));
            c[t][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0, b, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
            c[t][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1, b, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        }
        const float4 *bb = reinterpret_cast<const float4 *>(s + PK_L0B + g * 8);
        const float4 blo = bb[0], bhi = bb[1];
        const float bias[8] = {blo.x, blo.y, blo.z, blo.w, bhi.x, bhi.y, bhi.z, bhi.w};
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) a[t][4 * mt + r] = fmaxf(c[t][mt][r] + bias[4 * mt + r], 0.0f);
    }
    // hidden 32x32 layers: 8 k-steps x 2 row tiles of v_mfma_f32_16x16x4_f32 per point tile
    for (int jl = 0; jl < nh; ++jl) {
        const float *L = s + PK_HID + jl * PK_HID_STRIDE;
        float4 wq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) wq[q] = reinterpret_cast<const float4 *>(L)[q * 64 + lane];
#pragma unroll
        for (int st = 0; st < 8; ++st) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const int m = 2 * st + mt;
                const float4 wv = wq[m >> 2];
                const float w = (m & 3) == 0 ? wv.x : ((m & 3) == 1 ? wv.y : ((m & 3) == 2 ? wv.z : wv.w));
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    c[t][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        w, a[t][st], st == 0 ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : c[t][mt], 0, 0, 0);
            }
        }
        const float4 *bb = reinterpret_cast<const float4 *>(L + 1024 + g * 8);
        const float4 blo = bb[0], bhi = bb[1];
        const float bias[8] = {blo.x, blo.y, blo.z, blo.w, bhi.x, bhi.y, bhi.z, bhi.w};
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) a[t][4 * mt + r] = fmaxf(c[t][mt][r] + bias[4 * mt + r], 0.0f);
    }
    if constexpr (PART != 0) return a[0][0] + a[NT - 1][7];
    // final 32 -> 1 on VALU: group g holds units 8g..8g+7; the fmaf chain runs through
    // groups 0 -> 1 -> 2 -> 3 with one cross-lane hand-off per group.
    const float *wf = s + pk_final(nh) + g * 8;
    const float bf = s[pk_final(nh) + 32];
    float w8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w8[k] = wf[k];
    float zt[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = __builtin_fmaf(w8[k], a[t][k], acc);
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            float nacc = __shfl(acc, (lane + 48) & 63);  // from lane - 16 (group g - 1)
#pragma unroll
            for (int k = 0; k < 8; ++k) nacc = __builtin_fmaf(w8[k], a[t][k], nacc);
            acc = (g == q) ? nacc : acc;
        }
        zt[t] = acc + bf;
    }
    return tile_outputs(zt);
}

__device__ __forceinline__ float mlp16_fp32(const float *__restrict__ s, int in0, int nh, float fr, float x, float y,
                                            float z, uint32_t tmask) {
    const int nt = 32 - __clz((int)tmask);  // highest active tile + 1
    if (nt >= 4) return mlp16_fp32_nt<4>(s, in0, nh, fr, x, y, z);
    if (nt == 3) return mlp16_fp32_nt<3>(s, in0, nh, fr, x, y, z);
    if (nt == 2) return mlp16_fp32_nt<2>(s, in0, nh, fr, x, y, z);
    return mlp16_fp32_nt<1>(s, in0, nh, fr, x, y, z);
}

// bf16 / fp16 hidden layers: one v_mfma_f32_16x16x32 per row tile per layer (K = 32
// in a single instruction, bias preloaded as the accumulator); layer 0 on the f32
// matrix core as in the fp32 path; final layer in fp32 on VALU.  Register k = 4mt + r
// of group g holds unit 16mt + 4g + r (the MFMA C layout, unpermuted).
// bias + ReLU of one tile's two accumulators straight into the packed 16-bit B operand
// of the next layer: v_cvt_pk_{bf16,f16}_f32 rounds pairs (RNE), v_pk_max_i16 against 0
// is the ReLU on the 16-bit patterns (negative values and -0 have the sign bit set) --
// 8 VALU per tile instead of 8 fmaxf + 4 conversions.
template <int PREC>
__device__ __forceinline__ void relu_pack(const f32x4 &c0, const f32x4 &c1, uint32_t ap[4]) {
    typedef typename std::conditional<PREC == NR_PRECISION_BF16, __bf16, _Float16>::type e16;
    typedef e16 e16x2 __attribute__((ext_vector_type(2)));
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 v[4] = {{c0[0], c0[1]}, {c0[2], c0[3]}, {c1[0], c1[1]}, {c1[2], c1[3]}};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const s16x2 h = __builtin_bit_cast(s16x2, __builtin_convertvector(v[q], e16x2));
        ap[q] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(h, (s16x2){0, 0}));
    }
}

template <int PREC>
__device__ __forceinline__ f32x4 mfma_lowp(const void *w, const uint32_t ap[4], const f32x4 &cinit) {
    typedef typename std::conditional<PREC == NR_PRECISION_BF16, bf16x8, f16x8>::type v8;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const v8 b = __builtin_bit_cast(v8, (u32x4){ap[0], ap[1], ap[2], ap[3]});
    if constexpr (PREC == NR_PRECISION_BF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const v8 *>(w), b, cinit, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const v8 *>(w), b, cinit, 0, 0, 0);
}

template <int PREC, int NT>
__device__ __forceinline__ float mlp16_lowp_nt(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                               int nh, float fr, float x, float y, float z) {
    typedef typename std::conditional<PREC == NR_PRECISION_BF16, bf16x8, f16x8>::type v8;
    const int lane = lane_id(), g = lane >> 4, j = lane & 15;
    uint32_t ap[NT][4];  // activations of the hidden layers, packed 16-bit B operands
    float a[NT][8];      // fp32 activations feeding the final layer
    f32x4 c0[NT], c1[NT];
    {
        const float w0 = fl[lane], w1 = fl[64 + lane];
        const float4 *bb = reinterpret_cast<const float4 *>(fl + 128 + g * 8);
        const float4 blo = bb[0], bhi = bb[1];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const float px = __shfl(x, 16 * t + j), py = __shfl(y, 16 * t + j), pz = __shfl(z, 16 * t + j);
            const float pw = in0 == 4 ? __shfl(fr, 16 * t + j) : 0.0f;
            const float b = g == 0 ? px : (g == 1 ? py : (g == 2 ? pz : pw));
            c0[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0, b, f32x4{blo.x, blo.y, blo.z, blo.w}, 0, 0, 0);
            c1[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1, b, f32x4{bhi.x, bhi.y, bhi.z, bhi.w}, 0, 0, 0);
        }
    }
    // hidden layers; the last one's output stays fp32 for the final layer
    // (tile t's pack is issued right before its MFMAs, so it overlaps tile t-1's)
    for (int jl = 0; jl < nh; ++jl) {
        const v8 *A = reinterpret_cast<const v8 *>(lp + (size_t)jl * LP_A_ELEMS);
        const v8 w0 = A[lane], w1 = A[64 + lane];
        const float4 *bb = reinterpret_cast<const float4 *>(fl + 160 + 32 * jl + g * 8);
        const float4 blo = bb[0], bhi = bb[1];
        const f32x4 c0i = {blo.x, blo.y, blo.z, blo.w}, c1i = {bhi.x, bhi.y, bhi.z, bhi.w};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            relu_pack<PREC>(c0[t], c1[t], ap[t]);
            c0[t] = mfma_lowp<PREC>(&w0, ap[t], c0i);
            c1[t] = mfma_lowp<PREC>(&w1, ap[t], c1i);
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            a[t][r] = fmaxf(c0[t][r], 0.0f);
            a[t][4 + r] = fmaxf(c1[t][r], 0.0f);
        }
    const float *wf = fl + 160 + 32 * nh + g * 8;
    const float bf = fl[160 + 32 * nh + 32];
    float zt[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = __builtin_fmaf(wf[k], a[t][k], acc);
        acc += __shfl_xor(acc, 16);
        acc += __shfl_xor(acc, 32);
        zt[t] = acc + bf;
    }
    return tile_outputs(zt);
}

template <int PREC>
__device__ __forceinline__ float mlp16_lowp(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                            int nh, float fr, float x, float y, float z, uint32_t tmask) {
    const int nt = 32 - __clz((int)tmask);
    if (nt >= 4) return mlp16_lowp_nt<PREC, 4>(lp, fl, in0, nh, fr, x, y, z);
    if (nt == 3) return mlp16_lowp_nt<PREC, 3>(lp, fl, in0, nh, fr, x, y, z);
    if (nt == 2) return mlp16_lowp_nt<PREC, 2>(lp, fl, in0, nh, fr, x, y, z);
    return mlp16_lowp_nt<PREC, 1>(lp, fl, in0, nh, fr, x, y, z);
}

__device__ __forceinline__ float mlp16(const MlpArgs &M, const float *s32, const uint16_t *slp, const float *sfl,
                                       int prec, float fr, float x, float y, float z, uint32_t tmask) {
    if (prec == NR_PRECISION_BF16) return mlp16_lowp<NR_PRECISION_BF16>(slp, sfl, M.in0, M.nh, fr, x, y, z, tmask);
    if (prec == NR_PRECISION_FP16) return mlp16_lowp<NR_PRECISION_FP16>(slp, sfl, M.in0, M.nh, fr, x, y, z, tmask);
    return mlp16_fp32(s32, M.in0, M.nh, fr, x, y, z, tmask);
}

__device__ __forceinline__ uint32_t tiles_of(uint64_t m) {
    return ((m & 0xffffull) ? 1u : 0u) | (((m >> 16) & 0xffffull) ? 2u : 0u) | (((m >> 32) & 0xffffull) ? 4u : 0u) |
           ((m >> 48) ? 8u : 0u);
}

// LDS staging of the 16-wide packs (dynamic shared memory, block-wide 16-byte copies)
extern __shared__ __attribute__((aligned(16))) unsigned char nr_smem16[];

struct Smem16 {
    float *s32;       // fp32 16-wide pack
    uint16_t *slp;    // bf16/fp16 A operands
    float *sfl;       // float side of the low-precision pack
};

__device__ __forceinline__ Smem16 stage16(const MlpArgs &M, int prec) {
    Smem16 S;
    S.s32 = reinterpret_cast<float *>(nr_smem16);
    S.slp = reinterpret_cast<uint16_t *>(nr_smem16 + M.pk_bytes);
    S.sfl = reinterpret_cast<float *>(nr_smem16 + M.pk_bytes + M.lp_bytes);
    const int4 *src = reinterpret_cast<const int4 *>(M.pk);
    int4 *dst = reinterpret_cast<int4 *>(S.s32);
    for (int i = threadIdx.x; i < M.pk_bytes / 16; i += blockDim.x) dst[i] = src[i];
    if (prec != NR_PRECISION_FP32) {
        src = reinterpret_cast<const int4 *>(M.lp);
        dst = reinterpret_cast<int4 *>(S.slp);
        for (int i = threadIdx.x; i < M.lp_bytes / 16; i += blockDim.x) dst[i] = src[i];
        src = reinterpret_cast<const int4 *>(M.lpf);
        dst = reinterpret_cast<int4 *>(S.sfl);
        for (int i = threadIdx.x; i < M.lpf_bytes / 16; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();
    return S;
}

}  // namespace nr
