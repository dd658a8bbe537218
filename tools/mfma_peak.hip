// mfma_peak.hip -- sustained rate of back-to-back independent v_mfma_f32_16x16x4_f32 (the
// fp32 MLP's instruction) and v_mfma_f32_32x32x16_bf16, waves per SIMD 1..4, no VALU work:
// the practical ceiling the MLP kernels are measured against.  Prints TFLOP/s.
// build: hipcc --offload-arch=gfx950 -O3 mfma_peak.hip -o bin/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ void k_f32(float *out, int iters, float a0, float b0) {
    f32x4 c[8];
    for (int i = 0; i < 8; ++i) c[i] = f32x4{0, 0, 0, 0};
    const float a = a0 + threadIdx.x * 1e-9f, b = b0;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the same f32 MFMA stream with NV independent v_add_f32 after every MFMA (the VALU work an
// MLP epilogue or a marching phase adds to the issue port)
template <int NV>
__global__ void k_f32_valu(float *out, int iters, float a0, float b0) {
    f32x4 c[8];
    for (int i = 0; i < 8; ++i) c[i] = f32x4{0, 0, 0, 0};
    const float a = a0 + threadIdx.x * 1e-9f, b = b0;
    float v[8];
    for (int i = 0; i < 8; ++i) v[i] = a * (float)(i + 1);
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[i], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < NV; ++q) asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[(i + q) & 7]) : "v"(b));
        }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][3] + v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_bf16(float *out, int iters, float a0, float b0) {
    f32x16 c[4];
    for (int i = 0; i < 4; ++i) c[i] = f32x16{};
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(a0 + threadIdx.x * 1e-3f); b[i] = (__bf16)b0; }
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < 4; ++i) s += c[i][0] + c[i][15];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0)) return 1;
    const int cus = prop.multiProcessorCount;
    float *out;
    if (hipMalloc(&out, (size_t)cus * 16 * 256 * 4)) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) || hipEventCreate(&e1)) return 1;
    for (int kind = 0; kind < 2; ++kind)
        for (int wps = 1; wps <= 4; ++wps) {
            const int iters = kind == 0 ? 4096 : 8192;
            const int grid = cus * wps;  // 256 threads = 4 waves = one per SIMD, wps blocks per CU
            auto launch = [&]() {
                if (kind == 0) hipLaunchKernelGGL(k_f32, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f);
                else hipLaunchKernelGGL(k_bf16, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f);
            };
            launch();
            if (hipDeviceSynchronize()) return 1;
            if (hipEventRecord(e0, 0)) return 1;
            for (int r = 0; r < 5; ++r) launch();
            if (hipEventRecord(e1, 0) || hipEventSynchronize(e1)) return 1;
            float ms = 0;
            if (hipEventElapsedTime(&ms, e0, e1)) return 1;
            ms /= 5;
            const double flop = (double)grid * 4 * iters * (kind == 0 ? 8.0 * 2 * 16 * 16 * 4 : 4.0 * 2 * 32 * 32 * 16);
            const double tf = flop / (ms * 1e-3) / 1e12;
            printf("%s  waves/SIMD %d: %.3f ms  %.1f TF/s  (%.3f of %s)\n", kind == 0 ? "16x16x4 f32  " : "32x32x16 bf16", wps,
                   ms, tf, tf / (kind == 0 ? 157.3 : 2516.6), kind == 0 ? "157.3" : "2516.6");
        }
    for (int nv = 1; nv <= 6; ++nv)
        for (int wps = 1; wps <= 3; wps += 2) {
            const int iters = 4096, grid = cus * wps;
            auto launch = [&]() {
                switch (nv) {
                    case 1: hipLaunchKernelGGL(k_f32_valu<1>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f); break;
                    case 2: hipLaunchKernelGGL(k_f32_valu<2>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f); break;
                    case 3: hipLaunchKernelGGL(k_f32_valu<3>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f); break;
                    case 4: hipLaunchKernelGGL(k_f32_valu<4>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f); break;
                    case 5: hipLaunchKernelGGL(k_f32_valu<5>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f); break;
                    default: hipLaunchKernelGGL(k_f32_valu<6>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f, 1e-3f); break;
                }
            };
            launch();
            if (hipDeviceSynchronize()) return 1;
            if (hipEventRecord(e0, 0)) return 1;
            for (int r = 0; r < 5; ++r) launch();
            if (hipEventRecord(e1, 0) || hipEventSynchronize(e1)) return 1;
            float ms = 0;
            if (hipEventElapsedTime(&ms, e0, e1)) return 1;
            ms /= 5;
            const double tf = (double)grid * 4 * iters * 8.0 * 2 * 16 * 16 * 4 / (ms * 1e-3) / 1e12;
            printf("16x16x4 f32 + %d v_add_f32 per MFMA, waves/SIMD %d: %.1f TF/s (%.3f of 157.3)\n", nv, wps, tf, tf / 157.3);
        }
    return 0;
}
