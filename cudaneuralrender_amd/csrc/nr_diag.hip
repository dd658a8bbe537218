// nr_diag.hip -- diagnostics that are not part of the render path.  Built with the MFMA
// operands forced into VGPRs (Makefile), the form k_trace compiles to, so the latencies
// measured here are the ones the tracer sees.
#include "nr_mlp16.h"

namespace nr {

extern __shared__ __attribute__((aligned(16))) unsigned char nr_smem_diag[];

// Latency of the fp32 MLP on NT tiles for one wave alone on its SIMD (nr_set_debug
// bit 6): `reps` back-to-back evaluations, each input depending on the previous output.
// Y[0] = shader cycles per evaluation, Y[1..64] = the last outputs.  PART: see
// mlp16_fp32_nt.  CL: the clamped ReLU form (the tracer's, on the scaled pack); NH: unrolled
// for 7 hidden layers.
// (at most 128 VGPRs, the tracers' budget, so that the register allocation -- how far ahead the
// unrolled form can request weights -- is theirs)
template <int NT, int PART, bool CL = false, int NH = 0>
__global__ __launch_bounds__(64, 4) void k_mlp_latency(MlpArgs M, const float *__restrict__ X, float *__restrict__ Y,
                                                    int reps) {
    float *s32 = reinterpret_cast<float *>(nr_smem_diag);
    const int4 *src = reinterpret_cast<const int4 *>(M.pk);
    for (int i = threadIdx.x; i < M.pk_bytes / 16; i += blockDim.x) reinterpret_cast<int4 *>(s32)[i] = src[i];
    __syncthreads();
    const int lane = lane_id();
    float x = X[3 * lane], y = X[3 * lane + 1], z = X[3 * lane + 2], v = 0.0f;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) v = mlp16_fp32_nt<NT, PART, CL, NH>(s32, M.in0, M.nh, 0.0f, x + v * 1e-30f, y, z);
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) Y[0] = (float)(t1 - t0) / (float)reps;
    Y[1 + lane] = v;
}

// The same for the 16-bit MLP on 128 points (k_mlp16's form, mlp32_lowp_128; 7 hidden layers):
// PART 0 = the whole evaluation (the stream if M.lp_stream, else the builtin form), PART 1 = the
// pipelined stream alone (nr_mlp16_asm.h), its outputs fed back as its inputs; and on the
// tracer's 64 points (mlp16_lowp, one point per lane): PART 2 = two 32-point tiles, PART 3 = one.  Y[0] = shader cycles per evaluation.
template <int PREC, int PART>
__global__ __launch_bounds__(64) void k_mlp_latency_lp(MlpArgs M, const float *__restrict__ X, float *__restrict__ Y,
                                                       int reps) {
    uint16_t *slp = reinterpret_cast<uint16_t *>(nr_smem_diag);
    float *sfl = reinterpret_cast<float *>(nr_smem_diag + M.lp_bytes);
    for (int i = threadIdx.x; i < M.lp_bytes / 16; i += blockDim.x)
        reinterpret_cast<int4 *>(slp)[i] = reinterpret_cast<const int4 *>(M.lp)[i];
    for (int i = threadIdx.x; i < M.lpf_bytes / 16; i += blockDim.x)
        reinterpret_cast<int4 *>(sfl)[i] = reinterpret_cast<const int4 *>(M.lpf)[i];
    __syncthreads();
    const int lane = lane_id();
    constexpr bool CL = PREC == NR_PRECISION_BF16;
    float x[2] = {X[3 * lane], X[3 * lane + 3]}, y[2] = {X[3 * lane + 1], X[3 * lane + 4]};
    float z[2] = {X[3 * lane + 2], X[3 * lane + 5]}, fr[2] = {0.0f, 0.0f}, v[2] = {0.0f, 0.0f};
    u32x4 kk[4][2];
    for (int t = 0; t < 4; ++t) kk[t][0] = (u32x4){__float_as_uint(x[0]), __float_as_uint(y[0]), 0u, 0u};
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if constexpr (PART == 0) {
            const float xr[2] = {x[0] + v[0] * 1e-30f, x[1] + v[1] * 1e-30f};
            mlp32_lowp_128<PREC, 7, CL>(slp, sfl, M.in0, 7, fr, xr, y, z, v, M.lp_stream != 0);
        } else if constexpr (PART >= 2) {
            v[0] = mlp16_lowp<PREC>(slp, sfl, M.in0, 7, 0.0f, x[0] + v[0] * 1e-30f, y[0], z[0], PART == 2 ? 0xfu : 0x3u, CL);
        } else {
            mlp7_x4_stream<PREC, CL>(slp, sfl, kk);
            for (int t = 0; t < 4; ++t) kk[t][0] = kk[t][1] & 0x3f003f00u;
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) Y[0] = (float)(t1 - t0) / (float)reps;
    Y[1 + lane] = PART == 0 ? v[0] + v[1] : PART >= 2 ? v[0] : __uint_as_float(kk[0][0][0] ^ kk[3][1][3]);
}

template <int PART, bool CL = false, int NH = 0>
static void launch_lat(const MlpArgs &M, const float *X, float *Y, int reps, int nt, hipStream_t st) {
    const int sm = M.pk_bytes;
    if (nt <= 1) hipLaunchKernelGGL((k_mlp_latency<1, PART, CL, NH>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
    else if (nt == 2) hipLaunchKernelGGL((k_mlp_latency<2, PART, CL, NH>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
    else if (nt == 3) hipLaunchKernelGGL((k_mlp_latency<3, PART, CL, NH>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
    else hipLaunchKernelGGL((k_mlp_latency<4, PART, CL, NH>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
}

hipError_t launch_mlp_latency(const MlpArgs &M, int prec, const float *X, float *Y, int reps, int nt, int part,
                              hipStream_t st) {
    if (prec == NR_PRECISION_BF16 || prec == NR_PRECISION_FP16) {
        if (M.nh != 7 || M.in0 != 3 || !M.lp) return hipErrorInvalidValue;
        const int sm = M.lp_bytes + M.lpf_bytes;
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(1), dim3(64), sm, st, M, X, Y, reps); };
        // nt <= 2: the tracer's 64-point form on nt 32-point tiles; else k_mlp16's 128 points
        const int pt = (part & 1) ? 1 : nt == 1 ? 3 : nt == 2 ? 2 : 0;
        if (prec == NR_PRECISION_BF16) {
            if (pt == 0) go(k_mlp_latency_lp<NR_PRECISION_BF16, 0>);
            else if (pt == 1) go(k_mlp_latency_lp<NR_PRECISION_BF16, 1>);
            else if (pt == 2) go(k_mlp_latency_lp<NR_PRECISION_BF16, 2>);
            else go(k_mlp_latency_lp<NR_PRECISION_BF16, 3>);
        } else {
            if (pt == 0) go(k_mlp_latency_lp<NR_PRECISION_FP16, 0>);
            else if (pt == 1) go(k_mlp_latency_lp<NR_PRECISION_FP16, 1>);
            else if (pt == 2) go(k_mlp_latency_lp<NR_PRECISION_FP16, 2>);
            else go(k_mlp_latency_lp<NR_PRECISION_FP16, 3>);
        }
        return hipGetLastError();
    }
    // part bit 0: no final layer; bit 1: the clamped form (needs the scaled pack); bit 2: unrolled
    // for 7 hidden layers (needs nh == 7)
    if (((part & 2) && !M.f32_clamp) || ((part & 4) && M.nh != 7)) return hipErrorInvalidValue;
    switch (part & 7) {
        case 0: launch_lat<0>(M, X, Y, reps, nt, st); break;
        case 1: launch_lat<1>(M, X, Y, reps, nt, st); break;
        case 2: launch_lat<0, true>(M, X, Y, reps, nt, st); break;
        case 3: launch_lat<1, true>(M, X, Y, reps, nt, st); break;
        case 4: launch_lat<0, false, 7>(M, X, Y, reps, nt, st); break;
        case 5: launch_lat<1, false, 7>(M, X, Y, reps, nt, st); break;
        case 6: launch_lat<0, true, 7>(M, X, Y, reps, nt, st); break;
        default: launch_lat<1, true, 7>(M, X, Y, reps, nt, st); break;
    }
    return hipGetLastError();
}

}  // namespace nr
