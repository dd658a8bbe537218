// nr_mlp16.h -- the MLP on the matrix cores: 16-point tiles of v_mfma_f32_16x16x4_f32 for
// fp32 (below), 32-point tiles of v_mfma_f32_32x32x16_{bf16,f16} for reduced precision
// (mlp32_lowp_nt further down).
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
#include "nr_mlp16_asm.h"

// A/B experiment builds only (make EXTRA=-DNR_MLP16_EXP=n; wrong values): 1 no final layer,
// 2 no input range check, 4 no input-layer split in k_mlp16's stream path
#ifndef NR_MLP16_EXP
#define NR_MLP16_EXP 0
#endif

namespace nr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Cross-lane moves by v_permlane{16,32}_swap (VALU, no LDS round trip, no per-lane address
// register for the compiler to hoist out of the tracer's loop), on lane groups g = lane >> 4:
//   permlane16_swap(a, b) = {[a0 b0 a2 b2], [a1 b1 a3 b3]},  permlane32_swap(a, b) = {[a0 a1 b0 b1], [a2 a3 b2 b3]}
// (element k of a list = the 16 lanes of group k).
__device__ __forceinline__ uint32_t pl16(uint32_t a, uint32_t b, int half) {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    return half ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t pl32(uint32_t a, uint32_t b, int half) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    return half ? r[1] : r[0];
}

// NT <= 2 tiles (the 3-4 tile form transposes instead): z_t lives in lane (j, 3) = 48 + j of tile t; point p = 16t + j gets it back
// in lane p: [z0 g1, z1 g1, z0 g3, z1 g3], then the upper half's groups to the lower half.
template <int NT>
__device__ __forceinline__ float tile_outputs(const float zt[4]) {
    const uint32_t r = pl16(__float_as_uint(zt[0]), __float_as_uint(zt[NT > 1 ? 1 : 0]), 1);
    return __uint_as_float(pl32(r, r, 1));
}

// The value group q - 1 holds, delivered to group q (q = 1, 2, 3; other groups: unspecified).
__device__ __forceinline__ float from_prev_group(float v, int q) {
    const uint32_t u = __float_as_uint(v);
    if (q == 1) return __uint_as_float(pl16(u, u, 0));     // [v0 v0 v2 v2]
    if (q == 2) {
        const uint32_t t = pl16(u, u, 1);                  // [v1 v1 v3 v3]
        return __uint_as_float(pl32(t, t, 0));             // [v1 v1 v1 v1]
    }
    const uint32_t t = pl32(u, u, 1);                      // [v2 v3 v2 v3]
    return __uint_as_float(pl16(t, t, 0));                 // [v2 v2 v2 v2]
}

// LDS byte address of a pointer into shared memory
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// The 7 hidden layers of the clamped fp32 MLP on NT <= 2 tiles as the generated stream
// (nr_mlp16_asm.h NR_F32_HID7_NT*, tools/gen_mlp_asm.py build_f32): the loop below's instructions and
// operands, software-pipelined -- the next layer's weights requested during this one, the ReLU of
// row tile 1 deferred past the next layer's k-steps 0-3 -- for the latency of a wave with few rays
// (the single frame's tail).  a: in = layer 0's ReLU'd outputs, out = the last
// hidden layer's; the values of the loop, bit for bit.  Measured (profiles/r6_f32_stream.txt): a lone
// wave's MLP 5,396 -> 4,756 cycles on one tile, 9,628 -> 8,876 on two; but in the fp32 tracers
// (NR_F32_STREAM=1: one-tile waves take it) the single frame moved by -0.4 % and the batched
// headline lost 2-3 % (the pinned registers raise the kernel's allocation, 113 -> 120 VGPRs), so
// the tracers keep the loop and the stream is the latency diagnostic's form (nr_diag.hip part 6).
#ifndef NR_F32_STREAM
#define NR_F32_STREAM 0
#endif
template <int NT>
__device__ __forceinline__ void f32_hidden7_stream(const float *s, float (&a)[NT][8]) {
    typedef float f32x8 __attribute__((ext_vector_type(8)));
    const int lane = lane_id();
    const uint32_t va = lds_addr(s + PK_HID) + 16u * (uint32_t)lane;
    const uint32_t vb = lds_addr(s + PK_HID + 1024) + 32u * (uint32_t)(lane >> 4);
    f32x8 k[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
        k[t] = f32x8{a[t][0], a[t][1], a[t][2], a[t][3], a[t][4], a[t][5], a[t][6], a[t][7]};
    f32x16 c0, c1, w0, w1, b0;
    if constexpr (NT == 1) {
        asm volatile(NR_F32_HID7_NT1
                     : "+{v[16:23]}"(k[0]), "=&{v[0:15]}"(c0), "=&{v[24:39]}"(w0), "=&{v[40:55]}"(w1),
                       "=&{v[56:71]}"(b0)
                     : [va] "v"(va), [vb] "v"(vb)
                     : "memory");
    } else {
        asm volatile(NR_F32_HID7_NT2
                     : "+{v[32:39]}"(k[0]), "+{v[40:47]}"(k[NT - 1]), "=&{v[0:15]}"(c0), "=&{v[16:31]}"(c1),
                       "=&{v[48:63]}"(w0), "=&{v[64:79]}"(w1), "=&{v[80:95]}"(b0)
                     : [va] "v"(va), [vb] "v"(vb)
                     : "memory");
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 8; ++i) a[t][i] = k[t][i];
}

// FP32 MLP on NT active tiles (tiles 0..NT-1; the caller keeps live points there).
// PART != 0 only in the latency diagnostic (nr_diag.hip): stop after the hidden layers.
// CL: bias add and ReLU as one v_add_f32 / v_fma_f32 with the clamp bit (clamp to [0, 1]),
// valid on the scaled pack (nr_pack.cpp pack_fp32_16) for inputs within F32_INPUT_BOUND,
// where every activation is at most 1/2: bit-equal to fmaxf(v, 0) (NaN and -0 aside, which
// the chains of the next layer map to the same values).  Every VALU instruction costs f32
// matrix time on gfx950 (profiles/r1_mfma_peak.txt), and this halves the activation VALU.
// NH == 7 (the caller checks nh == 7): the stream below for NT <= 2 with the clamped ReLU
template <int NT, int PART = 0, bool CL = false, int NH = 0>
__device__ __forceinline__ float mlp16_fp32_nt(const float *__restrict__ s, int in0, int nh_rt, float fr, float x,
                                               float y, float z) {
    const int nh = NH > 0 ? NH : nh_rt;
    auto relu = [](float v) { return CL ? __builtin_amdgcn_fmed3f(v, 0.0f, 1.0f) : fmaxf(v, 0.0f); };
    // fr: this lane's 4th input (the frame number when rendering; used iff in0 == 4)
    const int lane = lane_id(), g = lane >> 4;
    float a[NT][8];
    f32x4 c[NT][2];
    // layer 0 on the matrix core too: K = in0 padded to 4 (weight 0 for the pad, whose
    // fma adds +0 to a chain that can never be -0), one v_mfma_f32_16x16x4_f32 per
    // row tile.  Lane (j, g) of tile t's B operand feeds input g of point 16t + j: the
    // 4x4 transpose of (input, tile) lane-group blocks of {x, y, z, frame} -- four
    // v_permlane{32,16}_swap instead of 16 ds_bpermute and 12 selects.
    {
        const float w0 = s[PK_L0W + lane], w1 = s[PK_L0W + 64 + lane];
        uint32_t t0 = __float_as_uint(x), t1 = __float_as_uint(y), t2 = __float_as_uint(z);
        uint32_t t3 = __float_as_uint(in0 == 4 ? fr : 0.0f);
        auto r = __builtin_amdgcn_permlane32_swap(t0, t2, false, false);  // groups 2,3 <-> 0,1
        t0 = r[0]; t2 = r[1];
        r = __builtin_amdgcn_permlane32_swap(t1, t3, false, false);
        t1 = r[0]; t3 = r[1];
        r = __builtin_amdgcn_permlane16_swap(t0, t1, false, false);       // groups 1,3 <-> 0,2
        t0 = r[0]; t1 = r[1];
        r = __builtin_amdgcn_permlane16_swap(t2, t3, false, false);
        t2 = r[0]; t3 = r[1];
        const float bt[4] = {__uint_as_float(t0), __uint_as_float(t1), __uint_as_float(t2), __uint_as_float(t3)};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            c[t][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w0, bt[t], f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
            c[t][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w1, bt[t], f32x4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
        }
        const float4 *bb = reinterpret_cast<const float4 *>(s + PK_L0B + g * 8);
        const float4 blo = bb[0], bhi = bb[1];
        const float bias[8] = {blo.x, blo.y, blo.z, blo.w, bhi.x, bhi.y, bhi.z, bhi.w};
        // the layer-0 weights are unscaled; fma(c, 2^-e0, b 2^-e0) = (c + b) 2^-e0 in one
        // rounding (2^-e0 = 1 on an unscaled pack: c + b)
        const float s0 = s[pk_final(nh) + 33];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) a[t][4 * mt + r] = relu(__builtin_fmaf(c[t][mt][r], s0, bias[4 * mt + r]));
    }
    // hidden 32x32 layers: 8 k-steps x 2 row tiles of v_mfma_f32_16x16x4_f32 per point tile
    constexpr bool STREAM = NT <= 2 && CL && NH == 7 && PART == 0;
    if constexpr (STREAM) f32_hidden7_stream<NT>(s, a);
    for (int jl = 0; jl < (STREAM ? 0 : nh); ++jl) {
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
                for (int r = 0; r < 4; ++r) a[t][4 * mt + r] = relu(c[t][mt][r] + bias[4 * mt + r]);
    }
    if constexpr (PART != 0) return a[0][0] + a[NT - 1][7];
    if constexpr (NT >= 3) {
        // final 32 -> 1 for 3-4 tiles: a 4x4 transpose of (tile, lane group) blocks with
        // v_permlane32_swap + v_permlane16_swap puts all 32 units of point j of tile t in
        // lane (j, t) -- the point's own lane -- so one 32-long fmaf chain (units ascending,
        // the oracle's order) serves all four tiles at once: 32 swaps + 33 VALU against
        // 4 x 38 for per-tile chains handed across groups (every VALU instruction costs
        // f32 matrix time on gfx950, tools/mfma_peak.hip)
        float b[4][8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t t0 = __float_as_uint(a[0][k]), t1 = __float_as_uint(a[1][k]);
            uint32_t t2 = __float_as_uint(a[2][k]), t3 = NT > 3 ? __float_as_uint(a[NT > 3 ? 3 : 0][k]) : 0u;
            auto r = __builtin_amdgcn_permlane32_swap(t0, t2, false, false);  // groups 2,3 <-> 0,1
            t0 = r[0]; t2 = r[1];
            r = __builtin_amdgcn_permlane32_swap(t1, t3, false, false);
            t1 = r[0]; t3 = r[1];
            r = __builtin_amdgcn_permlane16_swap(t0, t1, false, false);       // groups 1,3 <-> 0,2
            t0 = r[0]; t1 = r[1];
            r = __builtin_amdgcn_permlane16_swap(t2, t3, false, false);
            t2 = r[0]; t3 = r[1];
            b[0][k] = __uint_as_float(t0); b[1][k] = __uint_as_float(t1);
            b[2][k] = __uint_as_float(t2); b[3][k] = __uint_as_float(t3);
        }
        const float4 *wf4 = reinterpret_cast<const float4 *>(s + pk_final(nh));
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float4 w = wf4[q];  // units 4q..4q+3 = group q >> 1, registers 4(q & 1)..+3
            const int gg = q >> 1, k0 = 4 * (q & 1);
            acc = __builtin_fmaf(w.x, b[gg][k0 + 0], acc);
            acc = __builtin_fmaf(w.y, b[gg][k0 + 1], acc);
            acc = __builtin_fmaf(w.z, b[gg][k0 + 2], acc);
            acc = __builtin_fmaf(w.w, b[gg][k0 + 3], acc);
        }
        return acc + s[pk_final(nh) + 32];
    }
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
            float nacc = from_prev_group(acc, q);  // group g - 1's partial chain
#pragma unroll
            for (int k = 0; k < 8; ++k) nacc = __builtin_fmaf(w8[k], a[t][k], nacc);
            acc = (g == q) ? nacc : acc;
        }
        zt[t] = acc + bf;
    }
    return tile_outputs<NT>(zt);
}

// wave-uniform: every lane's inputs are within F32_INPUT_BOUND (NaN is not)
__device__ __forceinline__ bool inputs_in_bound_f32(float x, float y, float z, float f) {
    const bool ok = __builtin_fabsf(x) <= F32_INPUT_BOUND && __builtin_fabsf(y) <= F32_INPUT_BOUND &&
                    __builtin_fabsf(z) <= F32_INPUT_BOUND && __builtin_fabsf(f) <= F32_INPUT_BOUND;
    return __ballot(!ok) == 0;
}

// cl (wave-uniform): the pack is scaled (MlpArgs::f32_clamp) and the inputs are within the
// bound -- the clamped form on the active tiles; otherwise (never on the bundled networks'
// rays) the add + max form on all four tiles, which keeps one extra copy of the MLP code
// in the kernels instead of four.  ST: one tile of a 7-hidden-layer network on the stream
// (f32_hidden7_stream; the fp32 tracers' march -- its pinned registers cost the other callers'
// register allocations more than its latency gains them)
template <bool ST = false>
__device__ __forceinline__ float mlp16_fp32(const float *__restrict__ s, int in0, int nh, float fr, float x, float y,
                                            float z, uint32_t tmask, bool cl) {
    const int nt = 32 - __clz((int)tmask);  // highest active tile + 1
    if (cl) {
        if (nt >= 4) return mlp16_fp32_nt<4, 0, true>(s, in0, nh, fr, x, y, z);
        if (nt == 3) return mlp16_fp32_nt<3, 0, true>(s, in0, nh, fr, x, y, z);
        // one or two tiles (a wave with few rays: the tail): the stream for 7 hidden layers
        if (nt == 2) return mlp16_fp32_nt<2, 0, true>(s, in0, nh, fr, x, y, z);
        if (ST && NR_F32_STREAM && nh == 7) return mlp16_fp32_nt<1, 0, true, 7>(s, in0, nh, fr, x, y, z);
        if (nt == 2) return mlp16_fp32_nt<2, 0, true>(s, in0, nh, fr, x, y, z);
        return mlp16_fp32_nt<1, 0, true>(s, in0, nh, fr, x, y, z);
    }
    return mlp16_fp32_nt<4>(s, in0, nh, fr, x, y, z);
}
template <bool ST = false>
__device__ __forceinline__ float mlp16_fp32(const MlpArgs &M, const float *s, float fr, float x, float y, float z,
                                            uint32_t tmask) {
    return mlp16_fp32<ST>(s, M.in0, M.nh, fr, x, y, z, tmask, M.f32_clamp && inputs_in_bound_f32(x, y, z, fr));
}

// bf16 / fp16: the whole MLP on 32-point tiles, v_mfma_f32_32x32x16_{bf16,f16} (nr_internal.h
// LP32_*).  The wave's 64 points form two tiles (points 0-31, 32-63); in a tile, lane l
// feeds point l & 31 and the k-slots 8h..8h+7 of its half h = l >> 5.
//   * layer 0 on the matrix core too: one K = 16 MFMA per tile over the hi/lo split of
//     weights and inputs (w x ~ wh xh + wh xl + wl xh: ~2^-16 relative, f32 accumulate),
//     bias as the accumulator init;
//   * hidden layers: two K = 16 MFMAs per tile (K = 32), bias as the accumulator init; the
//     f32 result is its own next B operand with no lane movement (registers 8s..8s+7 are
//     k-step s, the pack orders the weights to match): per tile and layer 8 v_cvt_pk with
//     the ReLU folded into their clamp bit (bf16, relu_clamp_bf16_x*; otherwise 8 more
//     v_pk_max_i16) against 2 MFMAs of 32 cycles -- the 16x16x32 form needed as many VALU
//     per point for half the MFMA time per instruction and held the issue port twice as
//     long per point;
//   * final 32 -> 1 layer: 8 v_dot2c per tile over the same packed activations, the two
//     lane halves' partial sums joined by one v_permlane32_swap.
// The lane-half views of the inputs come from v_permlane32_swap as well (no ds_bpermute).
template <int PREC> struct Lowp;
template <> struct Lowp<NR_PRECISION_BF16> { typedef __bf16 e; typedef bf16x8 v8; };
template <> struct Lowp<NR_PRECISION_FP16> { typedef _Float16 e; typedef f16x8 v8; };
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// v0 = v of lane (l & 31), v1 = v of lane 32 + (l & 31)
__device__ __forceinline__ void half_views(float v, float &v0, float &v1) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v0 = __uint_as_float(r[0]);
    v1 = __uint_as_float(r[1]);
}

template <int PREC>
__device__ __forceinline__ f32x16 mfma32(const typename Lowp<PREC>::v8 &a, const typename Lowp<PREC>::v8 &b,
                                         const f32x16 &c) {
    if constexpr (PREC == NR_PRECISION_BF16) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// a.lo * b.lo + a.hi * b.hi + c on packed 16-bit pairs (v_dot2c_f32_{bf16,f16})
template <int PREC>
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    if constexpr (PREC == NR_PRECISION_BF16)
        return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a), __builtin_bit_cast(bf16x2, b), c, false);
    else
        return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b), c, false);
}

// registers 8s..8s+7 of an accumulator -> ReLU'd 16-bit B operand of k-step s:
// v_cvt_pk rounds pairs (RNE), v_pk_max_i16 against 0 is the ReLU on the 16-bit patterns
// (negative values and -0 have the sign bit set).  (bf16 on the clamped pack folds the ReLU into
// the conversion: relu_clamp_bf16_x* below.  For fp16 hipcc would fold min(max(cvt(x), 0), 1)
// into v_cvt_pk_f16_f32 ... clamp, but the scaled pack that needs costs fp16 its precision:
// nr_pack.cpp pack_lowp_32.)
template <int PREC>
__device__ __forceinline__ typename Lowp<PREC>::v8 relu_pack8(const f32x16 &c, int s) {
    typedef typename Lowp<PREC>::e e16;
    typedef e16 e16x2 __attribute__((ext_vector_type(2)));
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    u32x4 w;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x2 v = {c[8 * s + 2 * q], c[8 * s + 2 * q + 1]};
        const s16x2 h = __builtin_bit_cast(s16x2, __builtin_convertvector(v, e16x2));
        w[q] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(h, (s16x2){0, 0}));
    }
    return __builtin_bit_cast(typename Lowp<PREC>::v8, w);
}

__device__ __forceinline__ f32x16 load_bias16(const float *b) {
    const float4 *q = reinterpret_cast<const float4 *>(b);
    const float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
    return f32x16{a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w, a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
}

// bf16 ReLU folded into the conversion: v_cvt_pk_bf16_f32 with the VOP3 clamp bit clamps to
// [0, 1] (-0 and NaN -> +0; tools/cvt_clamp_probe.hip), which is the ReLU wherever the value is
// below 1.  The clamped pack (nr_pack.cpp, M.lp_clamp) scales every layer by a power of two so
// that, for inputs within LP_INPUT_BOUND, no activation exceeds 1/4: the scaling is exact in
// bf16 / f32 (same exponent range), so clamp(cvt(x)) here equals max(cvt(x), 0) of relu_pack8
// on the same pack, bit for bit -- 8 instead of 16 VALU per tile and layer.
// No builtin sets that bit on the bf16 conversion (hipcc folds it only into v_cvt_pk_f16_f32),
// so this is inline asm, which the compiler's hazard recognizer does not see.  It is made safe
// by construction:
//   * the block takes a VALU "touch" of every accumulator it converts as an input, and the
//     compiler puts the MFMA -> VALU wait states before each touch; when the block starts,
//     every MFMA this wave issued for these tiles has completed and none of the wave's MFMAs
//     is in flight (the next ones consume the block's outputs), so no MFMA RAW/WAW/WAR
//     hazard can involve a register the block reads or writes;
//   * it ends with s_nop 1: the two wait states a VALU write needs before an MFMA reads it.
// Outputs are early-clobber so that they never share a register with an input.
#define NR_CVC(o, a, b) "v_cvt_pk_bf16_f32 %" #o ", %" #a ", %" #b " clamp\n"
__device__ __forceinline__ void relu_clamp_bf16_x2(const f32x16 &c, const f32x16 &d, u32x4 (&k)[2][2]) {
    const uint32_t t0 = __float_as_uint(c[0]) & 1u, t1 = __float_as_uint(d[0]) & 1u;  // the touches
    asm(NR_CVC(0, 16, 17) NR_CVC(1, 18, 19) NR_CVC(2, 20, 21) NR_CVC(3, 22, 23)
        NR_CVC(4, 24, 25) NR_CVC(5, 26, 27) NR_CVC(6, 28, 29) NR_CVC(7, 30, 31)
        NR_CVC(8, 32, 33) NR_CVC(9, 34, 35) NR_CVC(10, 36, 37) NR_CVC(11, 38, 39)
        NR_CVC(12, 40, 41) NR_CVC(13, 42, 43) NR_CVC(14, 44, 45) NR_CVC(15, 46, 47)
        "s_nop 1"
        : "=&v"(k[0][0][0]), "=&v"(k[0][0][1]), "=&v"(k[0][0][2]), "=&v"(k[0][0][3]),
          "=&v"(k[0][1][0]), "=&v"(k[0][1][1]), "=&v"(k[0][1][2]), "=&v"(k[0][1][3]),
          "=&v"(k[1][0][0]), "=&v"(k[1][0][1]), "=&v"(k[1][0][2]), "=&v"(k[1][0][3]),
          "=&v"(k[1][1][0]), "=&v"(k[1][1][1]), "=&v"(k[1][1][2]), "=&v"(k[1][1][3])
        : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7]),
          "v"(c[8]), "v"(c[9]), "v"(c[10]), "v"(c[11]), "v"(c[12]), "v"(c[13]), "v"(c[14]), "v"(c[15]),
          "v"(d[0]), "v"(d[1]), "v"(d[2]), "v"(d[3]), "v"(d[4]), "v"(d[5]), "v"(d[6]), "v"(d[7]),
          "v"(d[8]), "v"(d[9]), "v"(d[10]), "v"(d[11]), "v"(d[12]), "v"(d[13]), "v"(d[14]), "v"(d[15]),
          "v"(t0), "v"(t1));
}
// four tiles (the 128-point MLP): one block, so that no MFMA of the next layer can be scheduled
// between the conversions of two tile pairs while the pair not yet converted is read
__device__ __forceinline__ void relu_clamp_bf16_x4(const f32x16 &c0, const f32x16 &c1, const f32x16 &c2, const f32x16 &c3,
                                                   u32x4 (&k)[4][2]) {
    const uint32_t t0 = __float_as_uint(c0[0]) & 1u, t1 = __float_as_uint(c1[0]) & 1u;  // the touches
    const uint32_t t2 = __float_as_uint(c2[0]) & 1u, t3 = __float_as_uint(c3[0]) & 1u;
    asm(NR_CVC(0, 32, 33) NR_CVC(1, 34, 35) NR_CVC(2, 36, 37) NR_CVC(3, 38, 39)
         NR_CVC(4, 40, 41) NR_CVC(5, 42, 43) NR_CVC(6, 44, 45) NR_CVC(7, 46, 47)
         NR_CVC(8, 48, 49) NR_CVC(9, 50, 51) NR_CVC(10, 52, 53) NR_CVC(11, 54, 55)
         NR_CVC(12, 56, 57) NR_CVC(13, 58, 59) NR_CVC(14, 60, 61) NR_CVC(15, 62, 63)
         NR_CVC(16, 64, 65) NR_CVC(17, 66, 67) NR_CVC(18, 68, 69) NR_CVC(19, 70, 71)
         NR_CVC(20, 72, 73) NR_CVC(21, 74, 75) NR_CVC(22, 76, 77) NR_CVC(23, 78, 79)
         NR_CVC(24, 80, 81) NR_CVC(25, 82, 83) NR_CVC(26, 84, 85) NR_CVC(27, 86, 87)
         NR_CVC(28, 88, 89) NR_CVC(29, 90, 91) NR_CVC(30, 92, 93) NR_CVC(31, 94, 95)
        "s_nop 1"
        : "=&v"(k[0][0][0]), "=&v"(k[0][0][1]), "=&v"(k[0][0][2]), "=&v"(k[0][0][3]),
          "=&v"(k[0][1][0]), "=&v"(k[0][1][1]), "=&v"(k[0][1][2]), "=&v"(k[0][1][3]),
          "=&v"(k[1][0][0]), "=&v"(k[1][0][1]), "=&v"(k[1][0][2]), "=&v"(k[1][0][3]),
          "=&v"(k[1][1][0]), "=&v"(k[1][1][1]), "=&v"(k[1][1][2]), "=&v"(k[1][1][3]),
          "=&v"(k[2][0][0]), "=&v"(k[2][0][1]), "=&v"(k[2][0][2]), "=&v"(k[2][0][3]),
          "=&v"(k[2][1][0]), "=&v"(k[2][1][1]), "=&v"(k[2][1][2]), "=&v"(k[2][1][3]),
          "=&v"(k[3][0][0]), "=&v"(k[3][0][1]), "=&v"(k[3][0][2]), "=&v"(k[3][0][3]),
          "=&v"(k[3][1][0]), "=&v"(k[3][1][1]), "=&v"(k[3][1][2]), "=&v"(k[3][1][3])
        : "v"(c0[0]), "v"(c0[1]), "v"(c0[2]), "v"(c0[3]), "v"(c0[4]), "v"(c0[5]), "v"(c0[6]), "v"(c0[7]),
          "v"(c0[8]), "v"(c0[9]), "v"(c0[10]), "v"(c0[11]), "v"(c0[12]), "v"(c0[13]), "v"(c0[14]), "v"(c0[15]),
          "v"(c1[0]), "v"(c1[1]), "v"(c1[2]), "v"(c1[3]), "v"(c1[4]), "v"(c1[5]), "v"(c1[6]), "v"(c1[7]),
          "v"(c1[8]), "v"(c1[9]), "v"(c1[10]), "v"(c1[11]), "v"(c1[12]), "v"(c1[13]), "v"(c1[14]), "v"(c1[15]),
          "v"(c2[0]), "v"(c2[1]), "v"(c2[2]), "v"(c2[3]), "v"(c2[4]), "v"(c2[5]), "v"(c2[6]), "v"(c2[7]),
          "v"(c2[8]), "v"(c2[9]), "v"(c2[10]), "v"(c2[11]), "v"(c2[12]), "v"(c2[13]), "v"(c2[14]), "v"(c2[15]),
          "v"(c3[0]), "v"(c3[1]), "v"(c3[2]), "v"(c3[3]), "v"(c3[4]), "v"(c3[5]), "v"(c3[6]), "v"(c3[7]),
          "v"(c3[8]), "v"(c3[9]), "v"(c3[10]), "v"(c3[11]), "v"(c3[12]), "v"(c3[13]), "v"(c3[14]), "v"(c3[15]),
          "v"(t0), "v"(t1), "v"(t2), "v"(t3));
}
__device__ __forceinline__ void relu_clamp_bf16_x1(const f32x16 &c, u32x4 (&k)[2]) {
    const uint32_t t0 = __float_as_uint(c[0]) & 1u;
    asm(NR_CVC(0, 8, 9) NR_CVC(1, 10, 11) NR_CVC(2, 12, 13) NR_CVC(3, 14, 15)
        NR_CVC(4, 16, 17) NR_CVC(5, 18, 19) NR_CVC(6, 20, 21) NR_CVC(7, 22, 23)
        "s_nop 1"
        : "=&v"(k[0][0]), "=&v"(k[0][1]), "=&v"(k[0][2]), "=&v"(k[0][3]),
          "=&v"(k[1][0]), "=&v"(k[1][1]), "=&v"(k[1][2]), "=&v"(k[1][3])
        : "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7]),
          "v"(c[8]), "v"(c[9]), "v"(c[10]), "v"(c[11]), "v"(c[12]), "v"(c[13]), "v"(c[14]), "v"(c[15]),
          "v"(t0));
}
#undef NR_CVC

// ReLU'd 16-bit B operands of both k-steps of every tile: k[t][s]
template <int PREC, int NT, bool CL>
__device__ __forceinline__ void relu_pack_tiles(const f32x16 (&acc)[NT], typename Lowp<PREC>::v8 (&k)[NT][2]) {
    typedef typename Lowp<PREC>::v8 v8;
    if constexpr (CL && PREC == NR_PRECISION_BF16) {
        u32x4 u[NT][2];
        if constexpr (NT == 4) relu_clamp_bf16_x4(acc[0], acc[1], acc[2], acc[3], u);
        else if constexpr (NT == 2) relu_clamp_bf16_x2(acc[0], acc[1], u);
        else relu_clamp_bf16_x1(acc[0], u[0]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) k[t][s] = __builtin_bit_cast(v8, u[t][s]);
    } else {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) k[t][s] = relu_pack8<PREC>(acc[t], s);
    }
}

// One hidden layer's operands: the two K = 16 A operands and the bias (accumulator init).
// (Reading the next layer's operands one layer ahead, to hide their LDS latency under the
// conversions, measured no faster and made the single-frame bf16 tracer spill:
// profiles/r2_mlp_lowp_dot2_prefetch.txt.)
template <int PREC> struct Hidden32W {
    typename Lowp<PREC>::v8 a0, a1;
    f32x16 b;
};
template <int PREC>
__device__ __forceinline__ Hidden32W<PREC> hidden32_load(const uint16_t *__restrict__ lp, const float *__restrict__ fl,
                                                         int jl) {
    typedef typename Lowp<PREC>::v8 v8;
    const int lane = lane_id(), h = lane >> 5;
    const v8 *A = reinterpret_cast<const v8 *>(lp + LP32_HID + jl * LP32_HSTRIDE);
    return Hidden32W<PREC>{A[lane], A[64 + lane], load_bias16(fl + 32 + 32 * jl + 16 * h)};
}

// one hidden layer on NT tiles: acc <- W relu(acc) + b
template <int PREC, int NT, bool CL>
__device__ __forceinline__ void hidden32(const Hidden32W<PREC> &w, f32x16 (&acc)[NT]) {
    typedef typename Lowp<PREC>::v8 v8;
    v8 k[NT][2];
    relu_pack_tiles<PREC, NT, CL>(acc, k);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = mfma32<PREC>(w.a1, k[t][1], mfma32<PREC>(w.a0, k[t][0], w.b));
}

template <int PREC, int NT, int NH, bool CL>
__device__ __forceinline__ void hidden_layers(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int nh,
                                              f32x16 (&acc)[NT]) {
    if constexpr (NH > 0) {
#pragma unroll
        for (int jl = 0; jl < NH; ++jl) hidden32<PREC, NT, CL>(hidden32_load<PREC>(lp, fl, jl), acc);
    } else {
        for (int jl = 0; jl < nh; ++jl) hidden32<PREC, NT, CL>(hidden32_load<PREC>(lp, fl, jl), acc);
    }
}

// two floats -> packed 16-bit pair (a in bits 0-15), RNE: one v_cvt_pk
template <int PREC>
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
    typedef typename Lowp<PREC>::e e16;
    typedef e16 e16x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, e16x2));
}
// the value of a packed pair's low / high element
template <int PREC>
__device__ __forceinline__ float lo16f(uint32_t p) {
    if constexpr (PREC == NR_PRECISION_BF16) return __uint_as_float(p << 16);
    else return (float)__builtin_bit_cast(_Float16, (uint16_t)(p & 0xffffu));
}
template <int PREC>
__device__ __forceinline__ float hi16f(uint32_t p) {
    if constexpr (PREC == NR_PRECISION_BF16) return __uint_as_float(p & 0xffff0000u);
    else return (float)__builtin_bit_cast(_Float16, (uint16_t)(p >> 16));
}

// The pipelined stream (nr_mlp16_asm.h, tools/gen_mlp_asm.py) of the 7-hidden-layer networks runs
// k_mlp16's 128-point form (MlpArgs::lp_stream; nr_set_debug bit 11 selects the builtin form).


// CL: ReLU by the conversion's clamp (bf16 with the clamped pack, inputs within
// LP_INPUT_BOUND -- the caller checks); otherwise cvt + v_pk_max_i16 (any pack, any input).
// (The tracer's 64 points as a two-tile pipelined stream: one wave alone 2,308 -> 1,964 cycles,
// but the stream's 96 pinned registers spilled the tracer's state, C3 +9 %; round 4,
// profiles/r4_ab_stream.txt.)
template <int PREC, int NT, int NH, bool CL>
__device__ __forceinline__ float mlp32_lowp_nt(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                               int nh_rt, float fr, float x, float y, float z) {
    typedef typename Lowp<PREC>::v8 v8;
    const int nh = NH > 0 ? NH : nh_rt;
    const int lane = lane_id(), h = lane >> 5;
    f32x16 acc[NT];
    {
        // B operand of tile t, lanes 0-31 (k 0-7) of point l: {xh, yh | zh, xl | yl, zl | fh, fl};
        // lanes 32-63 (k 8-15) of point l - 32: {xh, yh | zh, fh | 0 | 0}.  Each lane splits
        // its own point once (the residuals x - xh are exact in f32) and v_permlane32_swap(a, b)
        // = {[a lanes 0-31 | b lanes 0-31], [a lanes 32-63 | b lanes 32-63]} deals the packed
        // words to both tiles: word 1 swaps {zh, xl} against {zh, fh}, words 2-3 against 0.
        // (Round 2 split both tiles' points in every lane and assembled them with bit
        // selects: the same operands, ~20 more VALU per 64 points.)
        const uint32_t p0 = cvt2<PREC>(x, y);                                   // xh, yh
        const float dx = x - lo16f<PREC>(p0), dy = y - hi16f<PREC>(p0);
        const uint32_t q = cvt2<PREC>(z, dx);                                    // zh, xl
        const uint32_t r = cvt2<PREC>(dy, z - lo16f<PREC>(q));                   // yl, zl
        uint32_t f = 0;                                                          // fh, fl
        if (in0 == 4) {
            const uint32_t f0 = cvt2<PREC>(fr, 0.0f);
            f = cvt2<PREC>(fr, fr - lo16f<PREC>(f0));
        }
        const uint32_t qf = (q & 0xffffu) | (f << 16);                           // zh, fh
        const auto w0 = __builtin_amdgcn_permlane32_swap(p0, p0, false, false);
        const auto w1 = __builtin_amdgcn_permlane32_swap(q, qf, false, false);
        const auto w2 = __builtin_amdgcn_permlane32_swap(r, 0u, false, false);
        const auto w3 = __builtin_amdgcn_permlane32_swap(f, 0u, false, false);
        const v8 A = reinterpret_cast<const v8 *>(lp)[lane];
        const f32x16 b0 = load_bias16(fl + 16 * h);
#pragma unroll
        for (int t = 0; t < NT; ++t)
            acc[t] = mfma32<PREC>(A, __builtin_bit_cast(v8, (u32x4){w0[t], w1[t], w2[t], w3[t]}), b0);
    }
    hidden_layers<PREC, NT, NH, CL>(lp, fl, nh, acc);
    // final 32 -> 1 layer on the VALU: lane l holds 16 of point (l & 31)'s units as the 8
    // packed pairs of its B operands, and the pack's row-0 A operand of (k-step s, half h)
    // holds their weights in the same order, so 8 v_dot2c_f32_{bf16,f16} per tile give the
    // half's partial sum (k-step 0 then 1, pairs ascending); one v_permlane32_swap brings
    // the other half's partial (and tile 1 to lanes 32-63), then half 0 + half 1 + bias.
    // (Four 32x32x16 MFMAs, 1 useful row of 32, per 64 points before: profiles/
    // r2_mlp_lowp_dot2_prefetch.txt.)
    const u32x4 *F4 = reinterpret_cast<const u32x4 *>(lp + lp32_final(nh));
    const u32x4 wf[2] = {F4[h], F4[2 + h]};
    const float bf = fl[32 + 32 * nh];
    v8 k[NT][2];
    relu_pack_tiles<PREC, NT, CL>(acc, k);
    float zt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        float a = 0.0f;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const u32x4 kv = __builtin_bit_cast(u32x4, k[t][st]);
#pragma unroll
            for (int q = 0; q < 4; ++q) a = dot2<PREC>(kv[q], wf[st][q], a);
        }
        zt[t] = a;
    }
    float z0, z1;
    if constexpr (NT == 1) {
        half_views(zt[0], z0, z1);
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(zt[0]), __float_as_uint(zt[1]), false, false);
        z0 = __uint_as_float(r[0]);
        z1 = __uint_as_float(r[1]);
    }
    return (z0 + z1) + bf;
}

// The 128-point form of mlp32_lowp_nt for the stand-alone MLP (k_mlp16): two points per lane
// (set s = 0, 1: point p of set s in lane p), four 32-point tiles (2s, 2s + 1).  Same
// arithmetic per point, bit for bit; what changes is that every layer's operands -- two
// ds_read_b128 of A operands and four of bias per wave -- serve four tiles instead of two.
// At two tiles those reads kept the CU's LDS array ~80 % busy beside the MFMAs (49 ds_read_b128
// per 64 points against 30 MFMAs: 196 LDS-array cycles per 960 MFMA cycles on each of the 4
// SIMDs, MI355X_MICROARCH.md section LDS), and a layer's four independent MFMA chains give the
// wave's own conversions more to overlap with.

// Input layer + 7 hidden layers + the final layer's operand conversion of four 32-point tiles as
// one software-pipelined instruction stream: tile t + 1's conversions issue beside tile t's MFMAs
// (the builtin form issues each layer's 8 MFMAs, then its 32 conversions).  In: k[t][0] = tile t's
// input-layer B operand; out: k[t][s] = the ReLU'd 16-bit B operands of the final layer -- the
// values relu_pack_tiles gives after hidden_layers, bit for bit (same instructions, same
// operands).  Registers are pinned to the stream's (v0-v143, see the generated header).
template <int PREC, bool CL>
__device__ __forceinline__ void mlp7_x4_stream(const uint16_t *__restrict__ lp, const float *__restrict__ fl,
                                               u32x4 (&k)[4][2]) {
    typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
    const int lane = lane_id();
    const uint32_t va = lds_addr(lp) + 16u * (uint32_t)lane, vb = lds_addr(fl) + 64u * (uint32_t)(lane >> 5);
    f32x16 c0, c1, c2, c3, bb0, bb1;
    u32x8 ab0, ab1;
#define NR_STREAM_OPERANDS                                                                                          \
    : "+{v[64:67]}"(k[0][0]), "=&{v[68:71]}"(k[0][1]), "+{v[72:75]}"(k[1][0]), "=&{v[76:79]}"(k[1][1]),            \
      "+{v[80:83]}"(k[2][0]), "=&{v[84:87]}"(k[2][1]), "+{v[88:91]}"(k[3][0]), "=&{v[92:95]}"(k[3][1]),            \
      "=&{v[0:15]}"(c0), "=&{v[16:31]}"(c1), "=&{v[32:47]}"(c2), "=&{v[48:63]}"(c3), "=&{v[96:103]}"(ab0),         \
      "=&{v[104:111]}"(ab1), "=&{v[112:127]}"(bb0), "=&{v[128:143]}"(bb1)                                          \
    : [va] "v"(va), [vb] "v"(vb)                                                                                   \
    : "memory"
    if constexpr (PREC == NR_PRECISION_BF16 && CL) asm volatile(NR_HID7_BF16_CLAMP NR_STREAM_OPERANDS);
    else if constexpr (PREC == NR_PRECISION_BF16) asm volatile(NR_HID7_BF16_MAX NR_STREAM_OPERANDS);
    else asm volatile(NR_HID7_F16_MAX NR_STREAM_OPERANDS);
#undef NR_STREAM_OPERANDS
}

// The same with the hidden layers on v_mfma_f32_16x16x32 (round 6; k_mlp16 with MlpArgs::lp_s16,
// the pack of nr_pack.cpp pack_lowp_s16; tools/gen_mlp_asm.py build_s16): the input layer's
// 32x32x16 outputs are dealt to eight 16-point tiles by v_permlane16_swap and the last hidden
// layer's back to the four 32-point tiles' final-layer operands -- the same interface and the
// same values, bit for bit (a 16x16x32 MFMA sums its K = 32 as two chained K = 16 steps of the
// 8-product blocks, profiles/r5_mfma_peak_random.txt (4), and the pack keeps each block's units).
// Registers v0-v127 (16 fewer than the 32x32x16 stream: a 16-point tile's bias is 4 registers).
template <int PREC, bool CL>
__device__ __forceinline__ void mlp7_x4_stream_s16(const uint16_t *__restrict__ lp, const float *__restrict__ fl,
                                                   u32x4 (&k)[4][2]) {
    typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
    const int lane = lane_id();
    const uint32_t va = lds_addr(lp) + 16u * (uint32_t)lane, vb0 = lds_addr(fl) + 64u * (uint32_t)(lane >> 5),
                   vb = lds_addr(fl) + 32u * (uint32_t)(lane >> 4);
    f32x16 c0, c1, c2, c3;
    u32x8 ab0, ab1, bb0, bb1;
#define NR_S16_OPERANDS                                                                                             \
    : "+{v[64:67]}"(k[0][0]), "=&{v[68:71]}"(k[0][1]), "+{v[72:75]}"(k[1][0]), "=&{v[76:79]}"(k[1][1]),            \
      "+{v[80:83]}"(k[2][0]), "=&{v[84:87]}"(k[2][1]), "+{v[88:91]}"(k[3][0]), "=&{v[92:95]}"(k[3][1]),            \
      "=&{v[0:15]}"(c0), "=&{v[16:31]}"(c1), "=&{v[32:47]}"(c2), "=&{v[48:63]}"(c3), "=&{v[96:103]}"(ab0),         \
      "=&{v[104:111]}"(ab1), "=&{v[112:119]}"(bb0), "=&{v[120:127]}"(bb1)                                          \
    : [va] "v"(va), [vb0] "v"(vb0), [vb] "v"(vb)                                                                   \
    : "memory"
    if constexpr (PREC == NR_PRECISION_BF16 && CL) asm volatile(NR_S16_BF16_CLAMP NR_S16_OPERANDS);
    else if constexpr (PREC == NR_PRECISION_BF16) asm volatile(NR_S16_BF16_MAX NR_S16_OPERANDS);
    else asm volatile(NR_S16_F16_MAX NR_S16_OPERANDS);
#undef NR_S16_OPERANDS
}

template <int PREC, int NH, bool CL>
__device__ __forceinline__ void mlp32_lowp_128(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                               int nh_rt, const float (&fr)[2], const float (&x)[2],
                                               const float (&y)[2], const float (&z)[2], float (&out)[2],
                                               bool stream = false, bool s16 = false) {
    typedef typename Lowp<PREC>::v8 v8;
    const int nh = NH > 0 ? NH : nh_rt;
    const int lane = lane_id(), h = lane >> 5;
    if constexpr (NH == 7) {
        if (stream) {
            u32x4 kk[4][2];
#if NR_MLP16_EXP & 4
            // experiment: the input layer's split replaced by two conversions (wrong values)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const uint32_t p0 = cvt2<PREC>(x[s], y[s]), q = cvt2<PREC>(z[s], x[s]);
                kk[2 * s][0] = (u32x4){p0, q, p0, q};
                kk[2 * s + 1][0] = (u32x4){q, p0, q, p0};
            }
            if (0)
#endif
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                // the input layer's B operands exactly as below
                const uint32_t p0 = cvt2<PREC>(x[s], y[s]);
                const float dx = x[s] - lo16f<PREC>(p0), dy = y[s] - hi16f<PREC>(p0);
                const uint32_t q = cvt2<PREC>(z[s], dx);
                const uint32_t r = cvt2<PREC>(dy, z[s] - lo16f<PREC>(q));
                uint32_t f = 0;
                if (in0 == 4) {
                    const uint32_t f0 = cvt2<PREC>(fr[s], 0.0f);
                    f = cvt2<PREC>(fr[s], fr[s] - lo16f<PREC>(f0));
                }
                const uint32_t qf = (q & 0xffffu) | (f << 16);
                const auto w0 = __builtin_amdgcn_permlane32_swap(p0, p0, false, false);
                const auto w1 = __builtin_amdgcn_permlane32_swap(q, qf, false, false);
                const auto w2 = __builtin_amdgcn_permlane32_swap(r, 0u, false, false);
                const auto w3 = __builtin_amdgcn_permlane32_swap(f, 0u, false, false);
#pragma unroll
                for (int t = 0; t < 2; ++t) kk[2 * s + t][0] = (u32x4){w0[t], w1[t], w2[t], w3[t]};
            }
            if (s16) mlp7_x4_stream_s16<PREC, CL>(lp, fl, kk);
            else mlp7_x4_stream<PREC, CL>(lp, fl, kk);
#if NR_MLP16_EXP & 1
            // experiment: no final layer (wrong values)
            out[0] = __uint_as_float(kk[0][0][0] ^ kk[1][1][3]);
            out[1] = __uint_as_float(kk[2][0][0] ^ kk[3][1][3]);
            return;
#endif
            const u32x4 *F4 = reinterpret_cast<const u32x4 *>(lp + lp32_final(7));
            const u32x4 wf[2] = {F4[h], F4[2 + h]};
            const float bf = fl[32 + 32 * 7];
            float zt[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                float a = 0.0f;
#pragma unroll
                for (int st = 0; st < 2; ++st)
#pragma unroll
                    for (int q = 0; q < 4; ++q) a = dot2<PREC>(kk[t][st][q], wf[st][q], a);
                zt[t] = a;
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(zt[2 * s]), __float_as_uint(zt[2 * s + 1]),
                                                                false, false);
                out[s] = (__uint_as_float(r[0]) + __uint_as_float(r[1])) + bf;
            }
            return;
        }
    }
    f32x16 acc[4];
    {
        const v8 A = reinterpret_cast<const v8 *>(lp)[lane];
        const f32x16 b0 = load_bias16(fl + 16 * h);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // layer 0 of set s exactly as mlp32_lowp_nt's (see there)
            const uint32_t p0 = cvt2<PREC>(x[s], y[s]);
            const float dx = x[s] - lo16f<PREC>(p0), dy = y[s] - hi16f<PREC>(p0);
            const uint32_t q = cvt2<PREC>(z[s], dx);
            const uint32_t r = cvt2<PREC>(dy, z[s] - lo16f<PREC>(q));
            uint32_t f = 0;
            if (in0 == 4) {
                const uint32_t f0 = cvt2<PREC>(fr[s], 0.0f);
                f = cvt2<PREC>(fr[s], fr[s] - lo16f<PREC>(f0));
            }
            const uint32_t qf = (q & 0xffffu) | (f << 16);
            const auto w0 = __builtin_amdgcn_permlane32_swap(p0, p0, false, false);
            const auto w1 = __builtin_amdgcn_permlane32_swap(q, qf, false, false);
            const auto w2 = __builtin_amdgcn_permlane32_swap(r, 0u, false, false);
            const auto w3 = __builtin_amdgcn_permlane32_swap(f, 0u, false, false);
#pragma unroll
            for (int t = 0; t < 2; ++t)
                acc[2 * s + t] = mfma32<PREC>(A, __builtin_bit_cast(v8, (u32x4){w0[t], w1[t], w2[t], w3[t]}), b0);
        }
    }
    hidden_layers<PREC, 4, NH, CL>(lp, fl, nh, acc);
    const u32x4 *F4 = reinterpret_cast<const u32x4 *>(lp + lp32_final(nh));
    const u32x4 wf[2] = {F4[h], F4[2 + h]};
    const float bf = fl[32 + 32 * nh];
    v8 k[4][2];
    relu_pack_tiles<PREC, 4, CL>(acc, k);
    float zt[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        float a = 0.0f;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const u32x4 kv = __builtin_bit_cast(u32x4, k[t][st]);
#pragma unroll
            for (int q = 0; q < 4; ++q) a = dot2<PREC>(kv[q], wf[st][q], a);
        }
        zt[t] = a;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(zt[2 * s]), __float_as_uint(zt[2 * s + 1]), false,
                                                        false);
        out[s] = (__uint_as_float(r[0]) + __uint_as_float(r[1])) + bf;
    }
}

template <int PREC, bool CL>
__device__ __forceinline__ void mlp128_lowp_cl(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                               int nh, const float (&fr)[2], const float (&x)[2], const float (&y)[2],
                                               const float (&z)[2], float (&out)[2], bool stream, bool s16 = false) {
    if (nh == 7) mlp32_lowp_128<PREC, 7, CL>(lp, fl, in0, nh, fr, x, y, z, out, stream, s16);
    else mlp32_lowp_128<PREC, 0, CL>(lp, fl, in0, nh, fr, x, y, z, out);
}

template <int PREC, bool CL>
__device__ __forceinline__ float mlp16_lowp_cl(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                               int nh, float fr, float x, float y, float z, uint32_t tmask) {
    // the bundled networks' depth (7 hidden layers) fully unrolled: no loop-carried
    // accumulator copies between layers
    if (nh == 7) {
        if (tmask & 0xcu) return mlp32_lowp_nt<PREC, 2, 7, CL>(lp, fl, in0, nh, fr, x, y, z);
        return mlp32_lowp_nt<PREC, 1, 7, CL>(lp, fl, in0, nh, fr, x, y, z);
    }
    if (tmask & 0xcu) return mlp32_lowp_nt<PREC, 2, 0, CL>(lp, fl, in0, nh, fr, x, y, z);
    return mlp32_lowp_nt<PREC, 1, 0, CL>(lp, fl, in0, nh, fr, x, y, z);
}

// tmask: the caller's 16-point tiles (bits 0-3); the 32-point tiles cover pairs of them.
// cl (wave-uniform): the clamped-ReLU form is valid -- the pack is clamped (M.lp_clamp) and
// every input of the call is within LP_INPUT_BOUND
template <int PREC>
__device__ __forceinline__ float mlp16_lowp(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                            int nh, float fr, float x, float y, float z, uint32_t tmask, bool cl) {
    if constexpr (PREC == NR_PRECISION_BF16) {
        if (cl) return mlp16_lowp_cl<PREC, true>(lp, fl, in0, nh, fr, x, y, z, tmask);
    }
    return mlp16_lowp_cl<PREC, false>(lp, fl, in0, nh, fr, x, y, z, tmask);
}

// ---- fp32x3: fp32-class hidden layers on the fp16 matrix core (NR_PRECISION_FP32X3).
// Each activation a (f32, scaled: nr_pack.cpp pack_x3_32) is split into ah = rtz_f16(a) and
// al = rne_f16(a - ah), each weight into wh + wl (host side), and every hidden layer takes three
// K = 32 products per tile, a.w ~ al.wh + ah.wl + ah.wh (6 v_mfma_f32_32x32x16_f16, f32
// accumulate, the bias as the accumulator init).  The dropped al.wl and the 22-bit operands
// leave ~2-3x the error of the f32 fmaf chain against an exact evaluation (tests/
// test_gpu_fp32x3.py).  Per tile and layer the split is 8 v_cvt_pkrtz +
// 8 v_pk_max_i16 (the hi words' ReLU: a negative a has a non-positive ah) + 16
// v_fma_mix{lo,hi}_f16 with the clamp bit (the residual: a - ah has a's sign and, below 1 by the
// pack's scaling, the clamp to [0, 1] is its ReLU) -- 32 VALU against 6 MFMAs of 32 cycles.
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef short s16x2v __attribute__((ext_vector_type(2)));

// accumulator registers 8s..8s+7 -> ReLU'd hi / residual B operands of k-step s.
// m1 = -1.0f read from the pack: with a run-time multiplier the compiler forms the residual
// as one v_fma_mix (a literal -1 folds to a subtract of the widened hi, 3 instructions)
__device__ __forceinline__ void split_x3(const f32x16 &c, int s, float m1, f16x8 &hi, f16x8 &lo) {
    u32x4 hw, lw;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float v0 = c[8 * s + 2 * q], v1 = c[8 * s + 2 * q + 1];
        const f16x2v h = __builtin_bit_cast(f16x2v, __builtin_amdgcn_cvt_pkrtz(v0, v1));
        const _Float16 l0 = __builtin_amdgcn_fmed3h((_Float16)__builtin_fmaf((float)h[0], m1, v0), (_Float16)0.0f,
                                                    (_Float16)1.0f);
        const _Float16 l1 = __builtin_amdgcn_fmed3h((_Float16)__builtin_fmaf((float)h[1], m1, v1), (_Float16)0.0f,
                                                    (_Float16)1.0f);
        lw[q] = __builtin_bit_cast(uint32_t, (f16x2v){l0, l1});
        hw[q] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2v, h), (s16x2v){0, 0}));
    }
    hi = __builtin_bit_cast(f16x8, hw);
    lo = __builtin_bit_cast(f16x8, lw);
}

struct X3W {
    f16x8 h0, h1, l0, l1;  // hi / residual A operands of k-steps 0, 1
    f32x16 b;
};
__device__ __forceinline__ X3W x3_load(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int jl) {
    const int lane = lane_id(), h = lane >> 5;
    const f16x8 *A = reinterpret_cast<const f16x8 *>(lp + X3_HID + jl * X3_HSTRIDE);
    return X3W{A[lane], A[64 + lane], A[128 + lane], A[192 + lane], load_bias16(fl + 32 + 32 * jl + 16 * h)};
}

template <int NT>
__device__ __forceinline__ void hidden_x3(const X3W &w, f32x16 (&acc)[NT], float m1) {
    f16x8 hi[NT][2], lo[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) split_x3(acc[t], s, m1, hi[t][s], lo[t][s]);
    // small terms first (the bias, then the residual products), the hi.hi product last
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.h0, lo[t][0], w.b, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.h1, lo[t][1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.l0, hi[t][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.l1, hi[t][1], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.h0, hi[t][0], d, 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.h1, hi[t][1], d, 0, 0, 0);
    }
}

template <int NT, int NH>
__device__ __forceinline__ float mlp32_x3_nt(const uint16_t *__restrict__ lp, const float *__restrict__ fl, int in0,
                                             int nh_rt, float fr, float x, float y, float z) {
    constexpr int P = NR_PRECISION_FP16;
    const int nh = NH > 0 ? NH : nh_rt;
    const int lane = lane_id(), h = lane >> 5;
    const float *F = fl + x3_final(nh);
    const float m1 = F[33];
    f32x16 acc[NT];
    {
        // layer 0 as the reduced-precision MLP's (mlp32_lowp_nt) on the inputs scaled by
        // 2^X3_XYZ_SHIFT (exact): hi/lo fp16 split, one K = 16 MFMA per tile
        const float sx = F[34];
        x *= sx; y *= sx; z *= sx;
        const uint32_t p0 = cvt2<P>(x, y);
        const float dx = x - lo16f<P>(p0), dy = y - hi16f<P>(p0);
        const uint32_t q = cvt2<P>(z, dx);
        const uint32_t r = cvt2<P>(dy, z - lo16f<P>(q));
        uint32_t f = 0;
        if (in0 == 4) {
            const uint32_t f0 = cvt2<P>(fr, 0.0f);
            f = cvt2<P>(fr, fr - lo16f<P>(f0));
        }
        const uint32_t qf = (q & 0xffffu) | (f << 16);
        const auto w0 = __builtin_amdgcn_permlane32_swap(p0, p0, false, false);
        const auto w1 = __builtin_amdgcn_permlane32_swap(q, qf, false, false);
        const auto w2 = __builtin_amdgcn_permlane32_swap(r, 0u, false, false);
        const auto w3 = __builtin_amdgcn_permlane32_swap(f, 0u, false, false);
        const f16x8 A = reinterpret_cast<const f16x8 *>(lp)[lane];
        const f32x16 b0 = load_bias16(fl + 16 * h);
#pragma unroll
        for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, __builtin_bit_cast(f16x8, (u32x4){w0[t], w1[t], w2[t], w3[t]}),
                                                            b0, 0, 0, 0);
    }
    if constexpr (NH > 0) {
#pragma unroll
        for (int jl = 0; jl < NH; ++jl) hidden_x3<NT>(x3_load(lp, fl, jl), acc, m1);
    } else {
        for (int jl = 0; jl < nh; ++jl) hidden_x3<NT>(x3_load(lp, fl, jl), acc, m1);
    }
    // final 32 -> 1 layer in f32 on the VALU: lane l holds 16 of point (l & 31)'s units, the
    // pack holds their (scaled-back) weights in register order; the halves' partial sums are
    // joined by one v_permlane32_swap (tile 1 to lanes 32-63 on the way)
    const float4 *W4 = reinterpret_cast<const float4 *>(F + 16 * h);
    const float4 wa = W4[0], wb = W4[1], wc = W4[2], wd = W4[3];
    const float wf[16] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w, wc.x, wc.y, wc.z, wc.w, wd.x, wd.y, wd.z, wd.w};
    float zt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        float a = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) a = __builtin_fmaf(wf[i], fmaxf(acc[t][i], 0.0f), a);
        zt[t] = a;
    }
    float z0, z1;
    if constexpr (NT == 1) {
        half_views(zt[0], z0, z1);
    } else {
        const auto rr = __builtin_amdgcn_permlane32_swap(__float_as_uint(zt[0]), __float_as_uint(zt[1]), false, false);
        z0 = __uint_as_float(rr[0]);
        z1 = __uint_as_float(rr[1]);
    }
    return (z0 + z1) + F[32];
}

__device__ __forceinline__ float mlp16_x3_split(const MlpArgs &M, const uint16_t *lp, const float *fl, float fr, float x,
                                                float y, float z, uint32_t tmask) {
    if (M.nh == 7) {
        if (tmask & 0xcu) return mlp32_x3_nt<2, 7>(lp, fl, M.in0, M.nh, fr, x, y, z);
        return mlp32_x3_nt<1, 7>(lp, fl, M.in0, M.nh, fr, x, y, z);
    }
    if (tmask & 0xcu) return mlp32_x3_nt<2, 0>(lp, fl, M.in0, M.nh, fr, x, y, z);
    return mlp32_x3_nt<1, 0>(lp, fl, M.in0, M.nh, fr, x, y, z);
}

// fp32x3 per point: a point whose inputs are within the pack's bounds gets the split, any other
// point the fp32 MLP (bit-exact, from the fp32 pack) -- whatever else its wave holds, so a point's
// value never depends on its batch or chunk.  A wave of in-bound points runs the split
// alone, a wave of out-of-bound points the fp32 MLP alone, a mixed wave both (each point's column
// of the products is its own: the other lanes' inputs cannot reach it).  ok = M.lp_clamp: the pack
// exists (otherwise every point takes the fp32 MLP).
__device__ __forceinline__ float mlp16_x3(const MlpArgs &M, const float *s32, const uint16_t *lp, const float *fl,
                                          float fr, float x, float y, float z, uint32_t tmask, bool ok) {
    if (!ok) return mlp16_fp32(M, s32, fr, x, y, z, tmask);
    // the frame is an input only of a 4-input network (a 3-input network's single-frame tracer
    // passes A.frame here too: ADVICE r4)
    const bool in = __builtin_fabsf(x) <= X3_INPUT_BOUND && __builtin_fabsf(y) <= X3_INPUT_BOUND &&
                    __builtin_fabsf(z) <= X3_INPUT_BOUND && (M.in0 != 4 || __builtin_fabsf(fr) <= X3_FRAME_BOUND);
    const uint64_t out = __ballot(!in), live = __ballot(in);
    if (out == 0) return mlp16_x3_split(M, lp, fl, fr, x, y, z, tmask);
    const float v32 = mlp16_fp32(M, s32, fr, x, y, z, tmask);
    if (live == 0) return v32;
    const float v3 = mlp16_x3_split(M, lp, fl, fr, x, y, z, tmask);
    return in ? v3 : v32;
}

// The fp32 MLP as a call: the bf16/fp16 tracers' normals for points outside the x3 pack's input
// bounds (never the bundled scenes' hit points).  Out of line, so that the fallback adds nothing
// to the tracer's register demand at the shading site (inlined beside the split: 86 spilled VGPRs
// in the bf16 tracer against 28).  s: LDS, read through the generic address space here.
__device__ __noinline__ float mlp16_fp32_call(const float *s, int in0, int nh, float fr, float x, float y, float z,
                                              uint32_t tmask, bool cl) {
    return mlp16_fp32(s, in0, nh, fr, x, y, z, tmask, cl);
}

// bf16/fp16 tracers' normals (M.x3n): per point, the fp32x3 split for inputs within the x3 pack's
// bounds, the fp32 MLP otherwise -- the same per-point rule as the fp32x3 precision (mlp16_x3), so
// a normal never depends on the other rays of its wave.  Oracle: nr_oracle.c mlp_point_gpu_x3.
// ONE: 64 points as two one-tile passes (the shading site's register budget); otherwise one
// two-tile pass.
template <bool ONE = true>
__device__ __forceinline__ float mlp16_x3_normal(const MlpArgs &M, const float *s32, const uint16_t *lp,
                                                 const float *fl, float fr, float x, float y, float z, uint32_t tmask) {
    const bool in = __builtin_fabsf(x) <= X3_INPUT_BOUND && __builtin_fabsf(y) <= X3_INPUT_BOUND &&
                    __builtin_fabsf(z) <= X3_INPUT_BOUND && (M.in0 != 4 || __builtin_fabsf(fr) <= X3_FRAME_BOUND);
    float v = 0.0f;
    if (__builtin_expect(__ballot(!in) != 0, 0))
        v = mlp16_fp32_call(s32, M.in0, M.nh, fr, x, y, z, tmask, M.f32_clamp && inputs_in_bound_f32(x, y, z, fr));
    if (__ballot(in) != 0) {
        float v3;
        if (ONE && (tmask & 0xcu)) {
            // two one-tile passes instead of one two-tile pass (fewer live registers at the
            // shading site: 28 -> 9 spilled VGPRs in the bf16 batch tracer, C3 -1.7 %,
            // profiles/r4_ab_x3_tiles.txt): the second on tile 1's points moved to lanes 0-31
            v3 = mlp16_x3_split(M, lp, fl, fr, x, y, z, 0x3u);
            float a0, a1, b0, b1, c0, c1, d0, d1;
            half_views(x, a0, a1);
            half_views(y, b0, b1);
            half_views(z, c0, c1);
            half_views(fr, d0, d1);
            const bool lo = lane_id() < 32;
            const float v1 = mlp16_x3_split(M, lp, fl, lo ? d1 : d0, lo ? a1 : a0, lo ? b1 : b0, lo ? c1 : c0, 0x3u);
            v3 = lo ? v3 : v1;
        } else {
            v3 = mlp16_x3_split(M, lp, fl, fr, x, y, z, tmask);
        }
        v = in ? v3 : v;
    }
    return v;
}

// cl: see mlp16_lowp (ignored in fp32); fp32x3: the pack is valid (M.lp_clamp), the inputs are
// checked here
__device__ __forceinline__ float mlp16(const MlpArgs &M, const float *s32, const uint16_t *slp, const float *sfl,
                                       int prec, float fr, float x, float y, float z, uint32_t tmask, bool cl) {
    if (prec == NR_PRECISION_BF16) return mlp16_lowp<NR_PRECISION_BF16>(slp, sfl, M.in0, M.nh, fr, x, y, z, tmask, cl);
    if (prec == NR_PRECISION_FP16) return mlp16_lowp<NR_PRECISION_FP16>(slp, sfl, M.in0, M.nh, fr, x, y, z, tmask, cl);
    if (prec == NR_PRECISION_FP32X3) return mlp16_x3(M, s32, slp, sfl, fr, x, y, z, tmask, M.lp_clamp != 0);
    return mlp16_fp32<true>(M, s32, fr, x, y, z, tmask);
}

// wave-uniform: every lane's inputs are within LP_INPUT_BOUND (NaN is not)
__device__ __forceinline__ bool inputs_in_bound(float x, float y, float z, float f) {
    const bool ok = __builtin_fabsf(x) <= LP_INPUT_BOUND && __builtin_fabsf(y) <= LP_INPUT_BOUND &&
                    __builtin_fabsf(z) <= LP_INPUT_BOUND && __builtin_fabsf(f) <= LP_INPUT_BOUND;
    return __ballot(!ok) == 0;
}

// the 16-lane tiles of lane mask m that hold a set lane -- on the 32-bit halves: as a 64-bit test,
// m >> 48 != 0 became a compare against the constant 2^48, which the compiler kept in a VGPR pair
// for the tracer's whole life (and spilled)
__device__ __forceinline__ uint32_t tiles_of(uint64_t m) {
    const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    return ((lo & 0xffffu) ? 1u : 0u) | ((lo >> 16) ? 2u : 0u) | ((hi & 0xffffu) ? 4u : 0u) | ((hi >> 16) ? 8u : 0u);
}

// LDS staging of the 16-wide packs (dynamic shared memory, block-wide 16-byte copies)
extern __shared__ __attribute__((aligned(16))) unsigned char nr_smem16[];

struct Smem16 {
    float *s32;       // fp32 16-wide pack
    uint16_t *slp;    // bf16/fp16 A operands
    float *sfl;       // float side of the low-precision pack
};

// Stages the packs a kernel of precision PREC reads into LDS.  A reduced-precision kernel
// that also evaluates fp32 normals (NEED32: k_trace) reads the fp32 pack from global memory
// (30 KB, L2-resident): normal passes are ~5% of its MLP work, and without the fp32 pack a
// workgroup's LDS (16.5 KB pack + stash + frames) lets 3 workgroups share a CU instead of 2
// (bf16 C3 batch 2.09 -> 1.81 ms/frame, profiles/r2_lowp_clamp_lds_ab.txt).
// smem16_bytes() is the matching dynamic-LDS size.
template <int PREC, bool NEED32>
__device__ __forceinline__ Smem16 stage16(const MlpArgs &M) {
    constexpr bool lds32 = PREC == NR_PRECISION_FP32;
    Smem16 S;
    const int off = lds32 ? M.pk_bytes : 0;
    S.s32 = lds32 ? reinterpret_cast<float *>(nr_smem16) : const_cast<float *>(M.pk);
    S.slp = reinterpret_cast<uint16_t *>(nr_smem16 + off);
    S.sfl = reinterpret_cast<float *>(nr_smem16 + off + M.lp_bytes);
    if constexpr (lds32) {
        const int4 *src = reinterpret_cast<const int4 *>(M.pk);
        int4 *dst = reinterpret_cast<int4 *>(S.s32);
        for (int i = threadIdx.x; i < M.pk_bytes / 16; i += blockDim.x) dst[i] = src[i];
    }
    if constexpr (PREC != NR_PRECISION_FP32) {
        const int4 *src = reinterpret_cast<const int4 *>(M.lp);
        int4 *dst = reinterpret_cast<int4 *>(S.slp);
        for (int i = threadIdx.x; i < M.lp_bytes / 16; i += blockDim.x) dst[i] = src[i];
        src = reinterpret_cast<const int4 *>(M.lpf);
        dst = reinterpret_cast<int4 *>(S.sfl);
        for (int i = threadIdx.x; i < M.lpf_bytes / 16; i += blockDim.x) dst[i] = src[i];
    }

    __syncthreads();
    return S;
}

// The fp32x3 pack copied into dynamic LDS after the 16-bit pack (the endgame instances with
// NR_EG_WAVES > 4, whose fine passes and normals read it there); before stage16, whose
// __syncthreads completes it.  Returns the LDS copies of M.x3lp / M.x3fl.
template <int PREC>
__device__ __forceinline__ void stage_x3(const MlpArgs &M, int x3lp_bytes, int x3fl_bytes, const uint16_t *&xl,
                                         const float *&xf) {
    const int off = (PREC == NR_PRECISION_FP32 ? M.pk_bytes : 0) + M.lp_bytes + M.lpf_bytes;
    uint16_t *l = reinterpret_cast<uint16_t *>(nr_smem16 + off);
    float *f = reinterpret_cast<float *>(nr_smem16 + off + x3lp_bytes);
    const int4 *src = reinterpret_cast<const int4 *>(M.x3lp);
    int4 *dst = reinterpret_cast<int4 *>(l);
    for (int i = threadIdx.x; i < x3lp_bytes / 16; i += blockDim.x) dst[i] = src[i];
    src = reinterpret_cast<const int4 *>(M.x3fl);
    dst = reinterpret_cast<int4 *>(f);
    for (int i = threadIdx.x; i < x3fl_bytes / 16; i += blockDim.x) dst[i] = src[i];
    xl = l;
    xf = f;
}

// host side: the dynamic LDS stage16<prec, need32> uses
inline int smem16_bytes(const MlpArgs &M, int prec, bool need32, int x3_bytes = 0) {
    (void)need32;
    const bool lds32 = prec == NR_PRECISION_FP32;
    return (lds32 ? M.pk_bytes : 0) + (prec != NR_PRECISION_FP32 ? M.lp_bytes + M.lpf_bytes : 0) +
           x3_bytes;
}

}  // namespace nr
