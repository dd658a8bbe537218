// sqrt_exhaustive.hip -- which cheap square roots equal the correctly rounded sqrtf on
// every non-negative float?  Exhaustive over all 2^31 bit patterns 0x00000000-0x7fffffff
// (denormals, infinity and NaNs included); counts mismatches (NaN == NaN).
//   raw32: v_sqrt_f32 alone                (__builtin_amdgcn_sqrtf)
//   raw64: f32(v_sqrt_f64(f64(x)))         (__builtin_amdgcn_sqrt on double)
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off sqrt_exhaustive.hip -o bin/sqrt_exhaustive
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(unsigned long long *bad, unsigned *first) {
    const unsigned stride = gridDim.x * blockDim.x;
    unsigned long long b32 = 0, b64 = 0;
    for (unsigned u = blockIdx.x * blockDim.x + threadIdx.x; u < 0x80000000u; u += stride) {
        const float x = __uint_as_float(u);
        const float ref = sqrtf(x);  // correctly rounded expansion (-fno-fast-math)
        const float r32 = __builtin_amdgcn_sqrtf(x);
        const float r64 = (float)__builtin_amdgcn_sqrt((double)x);
        const bool e32 = __float_as_uint(r32) == __float_as_uint(ref) || (r32 != r32 && ref != ref);
        const bool e64 = __float_as_uint(r64) == __float_as_uint(ref) || (r64 != r64 && ref != ref);
        if (!e32) { ++b32; atomicMin(first + 0, u); }
        if (!e64) { ++b64; atomicMin(first + 1, u); }
    }
    atomicAdd(bad + 0, b32);
    atomicAdd(bad + 1, b64);
}

int main() {
    unsigned long long *db; unsigned *df;
    if (hipMalloc(&db, 16) || hipMalloc(&df, 8)) return 1;
    if (hipMemset(db, 0, 16) || hipMemset(df, 0xff, 8)) return 1;
    hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, db, df);
    unsigned long long b[2]; unsigned f[2];
    if (hipMemcpy(b, db, 16, hipMemcpyDeviceToHost) || hipMemcpy(f, df, 8, hipMemcpyDeviceToHost)) return 1;
    printf("raw v_sqrt_f32:          %llu mismatches of 2^31 (first 0x%08x)\n", b[0], f[0]);
    printf("f32(v_sqrt_f64(f64 x)):  %llu mismatches of 2^31 (first 0x%08x)\n", b[1], f[1]);
    return 0;
}
