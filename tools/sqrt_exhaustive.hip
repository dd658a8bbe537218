// sqrt_exhaustive.hip -- which cheap square roots equal the correctly rounded sqrtf on
// every non-negative float?  Exhaustive over all 2^31 bit patterns 0x00000000-0x7fffffff
// (denormals, infinity and NaNs included); counts mismatches (NaN == NaN).
//   raw32: v_sqrt_f32 alone                (__builtin_amdgcn_sqrtf)
//   raw64: f32(v_sqrt_f64(f64(x)))         (__builtin_amdgcn_sqrt on double)
//   rn:    nr_device.h sqrt_rn_normal (v_sqrt_f32 + the two-FMA rounding correction, without
//          the denormal scaling and the class check) on its domain [2^-96, FLT_MAX]
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off sqrt_exhaustive.hip -o bin/sqrt_exhaustive
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../cudaneuralrender_amd/csrc/nr_device.h"

__global__ void k(unsigned long long *bad, unsigned *first) {
    const unsigned stride = gridDim.x * blockDim.x;
    unsigned long long b32 = 0, b64 = 0, brn = 0;
    for (unsigned u = blockIdx.x * blockDim.x + threadIdx.x; u < 0x80000000u; u += stride) {
        const float x = __uint_as_float(u);
        const float ref = sqrtf(x);  // correctly rounded expansion (-fno-fast-math)
        const float r32 = __builtin_amdgcn_sqrtf(x);
        const float r64 = (float)__builtin_amdgcn_sqrt((double)x);
        const bool e32 = __float_as_uint(r32) == __float_as_uint(ref) || (r32 != r32 && ref != ref);
        const bool e64 = __float_as_uint(r64) == __float_as_uint(ref) || (r64 != r64 && ref != ref);
        if (!e32) { ++b32; atomicMin(first + 0, u); }
        if (!e64) { ++b64; atomicMin(first + 1, u); }
        if (u >= 0x0f800000u && u <= 0x7f7fffffu && __float_as_uint(nr::sqrt_rn_normal(x)) != __float_as_uint(ref)) {
            ++brn;
            atomicMin(first + 2, u);
        }
    }
    atomicAdd(bad + 0, b32);
    atomicAdd(bad + 1, b64);
    atomicAdd(bad + 2, brn);
}

int main() {
    unsigned long long *db; unsigned *df;
    if (hipMalloc(&db, 24) || hipMalloc(&df, 12)) return 1;
    if (hipMemset(db, 0, 24) || hipMemset(df, 0xff, 12)) return 1;
    hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, db, df);
    unsigned long long b[3]; unsigned f[3];
    if (hipMemcpy(b, db, 24, hipMemcpyDeviceToHost) || hipMemcpy(f, df, 12, hipMemcpyDeviceToHost)) return 1;
    printf("raw v_sqrt_f32:          %llu mismatches of 2^31 (first 0x%08x)\n", b[0], f[0]);
    printf("f32(v_sqrt_f64(f64 x)):  %llu mismatches of 2^31 (first 0x%08x)\n", b[1], f[1]);
    printf("sqrt_rn_normal on [2^-96, FLT_MAX]: %llu mismatches (first 0x%08x)\n", b[2], f[2]);
    return 0;
}
