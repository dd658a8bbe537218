// Probe (GPU box): does a 16-bit-result VALU conversion on gfx950 zero the high half of
// its destination VGPR, as the compiler's fp16 operand packing assumes?
//   hipcc --offload-arch=gfx950 -O2 tools/cvt_high_probe.hip -o tools/bin/cvt_high_probe
// Each case pre-loads the destination with 0xDEADBEEF, converts 1.5f, and prints the
// full 32-bit register: 0x00003e00 = high half zeroed, 0xdead3e00 = preserved
// (the v_add_f16 case: 0x00004200 / 0xdead4200).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned *out, float x) {
    unsigned r0 = 0xDEADBEEFu, r1 = 0xDEADBEEFu, r2 = 0xDEADBEEFu, r3 = 0xDEADBEEFu, r4 = 0xDEADBEEFu;
    asm volatile("v_cvt_f16_f32_e32 %0, %1" : "+v"(r0) : "v"(x));
    asm volatile("v_cvt_f16_f32_e64 %0, %1" : "+v"(r1) : "v"(x));
    asm volatile("v_cvt_f16_f32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:DWORD" : "+v"(r2) : "v"(x));
    asm volatile("v_cvt_f16_f32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(r3) : "v"(x));
    asm volatile("v_add_f16_e32 %0, %1, %1" : "+v"(r4) : "v"(0x3e00u));
    if (threadIdx.x == 0) { out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3; out[4] = r4; }
}

int main() {
    unsigned *d, h[5];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 1.5f);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *names[5] = {"v_cvt_f16_f32_e32", "v_cvt_f16_f32_e64", "sdwa WORD_1 UNUSED_PAD",
                            "sdwa WORD_1 UNUSED_PRESERVE", "v_add_f16_e32 (1.5+1.5)"};
    for (int i = 0; i < 5; ++i) printf("%-28s 0x%08x\n", names[i], h[i]);
    hipFree(d);
    return 0;
}
