// permlane_probe.hip -- lane movement of v_permlane16_swap / v_permlane32_swap (gfx950):
// vdst = lane id, src = 100 + lane id; prints which source value each lane holds after.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(unsigned *o) {
    const unsigned l = threadIdx.x;
    const auto r16 = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
    const auto r32 = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
    o[l] = r16[0]; o[64 + l] = r16[1]; o[128 + l] = r32[0]; o[192 + l] = r32[1];
}

int main() {
    unsigned *d, h[256];
    if (hipMalloc(&d, 1024)) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost)) return 1;
    const char *nm[4] = {"permlane16 vdst", "permlane16 src ", "permlane32 vdst", "permlane32 src "};
    for (int v = 0; v < 4; ++v) {
        printf("%s:", nm[v]);
        for (int g = 0; g < 4; ++g) printf("  lanes %2d-%2d <- %u..%u", 16 * g, 16 * g + 15, h[64 * v + 16 * g], h[64 * v + 16 * g + 15]);
        printf("\n");
    }
    return 0;
}
