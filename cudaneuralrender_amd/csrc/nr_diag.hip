// nr_diag.hip -- diagnostics that are not part of the render path.  Built with the MFMA
// operands forced into VGPRs (Makefile), the form k_trace compiles to, so the latencies
// measured here are the ones the tracer sees.
#include "nr_mlp16.h"

namespace nr {

extern __shared__ __attribute__((aligned(16))) unsigned char nr_smem_diag[];

// Latency of the fp32 MLP on NT tiles for one wave alone on its SIMD (nr_set_debug
// bit 6): `reps` back-to-back evaluations, each input depending on the previous output.
// Y[0] = shader cycles per evaluation, Y[1..64] = the last outputs.  PART: see
// mlp16_fp32_nt.
template <int NT, int PART>
__global__ __launch_bounds__(64) void k_mlp_latency(MlpArgs M, const float *__restrict__ X, float *__restrict__ Y,
                                                    int reps) {
    float *s32 = reinterpret_cast<float *>(nr_smem_diag);
    const int4 *src = reinterpret_cast<const int4 *>(M.pk);
    for (int i = threadIdx.x; i < M.pk_bytes / 16; i += blockDim.x) reinterpret_cast<int4 *>(s32)[i] = src[i];
    __syncthreads();
    const int lane = lane_id();
    float x = X[3 * lane], y = X[3 * lane + 1], z = X[3 * lane + 2], v = 0.0f;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) v = mlp16_fp32_nt<NT, PART>(s32, M.in0, M.nh, 0.0f, x + v * 1e-30f, y, z);
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) Y[0] = (float)(t1 - t0) / (float)reps;
    Y[1 + lane] = v;
}

template <int PART>
static void launch_lat(const MlpArgs &M, const float *X, float *Y, int reps, int nt, hipStream_t st) {
    const int sm = M.pk_bytes;
    if (nt <= 1) hipLaunchKernelGGL((k_mlp_latency<1, PART>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
    else if (nt == 2) hipLaunchKernelGGL((k_mlp_latency<2, PART>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
    else if (nt == 3) hipLaunchKernelGGL((k_mlp_latency<3, PART>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
    else hipLaunchKernelGGL((k_mlp_latency<4, PART>), dim3(1), dim3(64), sm, st, M, X, Y, reps);
}

hipError_t launch_mlp_latency(const MlpArgs &M, const float *X, float *Y, int reps, int nt, int part, hipStream_t st) {
    if (part) launch_lat<1>(M, X, Y, reps, nt, st);
    else launch_lat<0>(M, X, Y, reps, nt, st);
    return hipGetLastError();
}

}  // namespace nr
