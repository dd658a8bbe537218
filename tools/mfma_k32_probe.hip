// Diagnostic: one v_mfma_f32_16x16x32_{f16,bf16} per 16x16 matrix, for tools/mfma_k32_check.py:
// is the K = 32 instruction's sum the same as two chained K = 16 steps of the matrix core's
// summation model (oracle/nr_oracle.c mfma_sum_e, fitted on v_mfma_f32_32x32x16 in round 4)?  If it
// is, a 16x16x32 form of the 16-bit MLP gives the current form's values bit for bit.
//   A: n x [16 rows][32 k] 16-bit, B: n x [32 k][16 cols] 16-bit, C, D: n x [16][16] f32.
// Operand layout (16x16x32): lane l holds A row l % 16, k = 8 (l / 16) + e; B column l % 16, the
// same k; D register i of lane l = row 4 (l / 16) + i, column l % 16.
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC mfma_k32_probe.hip -o bin/libmfma_k32_probe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <bool BF16>
__global__ __launch_bounds__(64) void k_probe32(const uint16_t *A, const uint16_t *B, const float *C, float *D) {
    const int m = blockIdx.x, l = threadIdx.x, r = l & 15, g = l >> 4;
    const uint16_t *a = A + (size_t)m * 512, *b = B + (size_t)m * 512;
    uint16_t av[8], bv[8];
    for (int e = 0; e < 8; ++e) {
        av[e] = a[r * 32 + 8 * g + e];
        bv[e] = b[(8 * g + e) * 16 + r];
    }
    f32x4 c;
    for (int i = 0; i < 4; ++i) c[i] = C[(size_t)m * 256 + (4 * g + i) * 16 + r];
    f32x4 d;
    if constexpr (BF16) {
        bf16x8 x, y;
        __builtin_memcpy(&x, av, 16);
        __builtin_memcpy(&y, bv, 16);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, c, 0, 0, 0);
    } else {
        f16x8 x, y;
        __builtin_memcpy(&x, av, 16);
        __builtin_memcpy(&y, bv, 16);
        d = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i) D[(size_t)m * 256 + (4 * g + i) * 16 + r] = d[i];
}

extern "C" int mfma_k32_probe(const uint16_t *A, const uint16_t *B, const float *C, float *D, int n, int bf16) {
    uint16_t *dA, *dB;
    float *dC, *dD;
    if (hipMalloc(&dA, (size_t)n * 1024) != hipSuccess || hipMalloc(&dB, (size_t)n * 1024) != hipSuccess ||
        hipMalloc(&dC, (size_t)n * 1024) != hipSuccess || hipMalloc(&dD, (size_t)n * 1024) != hipSuccess)
        return -1;
    hipMemcpy(dA, A, (size_t)n * 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, (size_t)n * 1024, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, (size_t)n * 1024, hipMemcpyHostToDevice);
    if (bf16) hipLaunchKernelGGL(k_probe32<true>, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD);
    else hipLaunchKernelGGL(k_probe32<false>, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD);
    const hipError_t e = hipDeviceSynchronize();
    hipMemcpy(D, dD, (size_t)n * 1024, hipMemcpyDeviceToHost);
    hipFree(dA);
    hipFree(dB);
    hipFree(dC);
    hipFree(dD);
    return e == hipSuccess ? 0 : -2;
}
