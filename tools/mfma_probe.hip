// Diagnostic: one v_mfma_f32_32x32x16_{f16,bf16} per 32x32 matrix, for tools/mfma_model.py's
// rounding-model fit (which order / grouping / rounding the matrix core sums its 16 products and
// the accumulator in).  Built by tools/mfma_model.py into tools/bin/libmfma_probe.so.
//   A: n x [32 rows][16 k] 16-bit, B: n x [16 k][32 cols] 16-bit, C, D: n x [32][32] f32.
// Operand layout (CDNA3/4 32x32x16): lane l holds A row l % 32, k = 8 (l / 32) + e; B column
// l % 32, the same k; D register i of lane l = row (i & 3) + 8 (i >> 2) + 4 (l / 32), column l % 32.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <bool BF16>
__global__ __launch_bounds__(64) void k_probe(const uint16_t *A, const uint16_t *B, const float *C, float *D) {
    const int m = blockIdx.x, l = threadIdx.x, r = l & 31, h = l >> 5;
    const uint16_t *a = A + (size_t)m * 512, *b = B + (size_t)m * 512;
    uint16_t av[8], bv[8];
    for (int e = 0; e < 8; ++e) {
        av[e] = a[r * 16 + 8 * h + e];
        bv[e] = b[(8 * h + e) * 32 + r];
    }
    f32x16 c;
    for (int i = 0; i < 16; ++i) c[i] = C[(size_t)m * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
    f32x16 d;
    if constexpr (BF16) {
        bf16x8 x, y;
        __builtin_memcpy(&x, av, 16);
        __builtin_memcpy(&y, bv, 16);
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, c, 0, 0, 0);
    } else {
        f16x8 x, y;
        __builtin_memcpy(&x, av, 16);
        __builtin_memcpy(&y, bv, 16);
        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, c, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) D[(size_t)m * 1024 + ((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = d[i];
}

extern "C" int mfma_probe(const uint16_t *A, const uint16_t *B, const float *C, float *D, int n, int bf16) {
    uint16_t *dA, *dB;
    float *dC, *dD;
    const size_t s16 = (size_t)n * 512 * 2, s32 = (size_t)n * 1024 * 4;
    if (hipMalloc(&dA, s16) || hipMalloc(&dB, s16) || hipMalloc(&dC, s32) || hipMalloc(&dD, s32)) return 1;
    hipMemcpy(dA, A, s16, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, s16, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, s32, hipMemcpyHostToDevice);
    if (bf16)
        hipLaunchKernelGGL(k_probe<true>, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD);
    else
        hipLaunchKernelGGL(k_probe<false>, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD);
    int rc = hipDeviceSynchronize() != hipSuccess;
    hipMemcpy(D, dD, s32, hipMemcpyDeviceToHost);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
    return rc;
}
