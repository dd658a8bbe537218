// cvt_clamp_probe.hip -- what the VOP3 clamp bit does on v_cvt_pk_bf16_f32 and
// v_cvt_pk_f16_f32 (gfx950): prints each input pair and the two packed 16-bit results.
// build: hipcc --offload-arch=gfx950 -O2 cvt_clamp_probe.hip -o bin/cvt_clamp_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__global__ void k(const float *a, unsigned *o) {
    const int i = threadIdx.x;
    unsigned r, s;
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2 clamp" : "=v"(r) : "v"(a[2 * i]), "v"(a[2 * i + 1]));
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2 clamp" : "=v"(s) : "v"(a[2 * i]), "v"(a[2 * i + 1]));
    o[i] = r;
    o[64 + i] = s;
}

static float bf(unsigned h) { unsigned u = h << 16; float f; memcpy(&f, &u, 4); return f; }
static float hf(unsigned h) {
    _Float16 x; unsigned short s = (unsigned short)h; memcpy(&x, &s, 2); return (float)x;
}

int main() {
    const int n = 8;
    float h[2 * n] = {-1.0f, 0.5f, 2.0f, 1e30f, -0.0f, 0.0f, 1e-30f, -1e-30f, 0.999f, 1.0f,
                      __builtin_nanf(""), -__builtin_nanf(""), 3e-39f, 0.25f, -5.f, 7.f};
    float *da; unsigned *dout;
    if (hipMalloc(&da, sizeof h) || hipMalloc(&dout, 128 * 4)) return 1;
    if (hipMemcpy(da, h, sizeof h, hipMemcpyHostToDevice)) return 1;
    k<<<1, n>>>(da, dout);
    unsigned o[128];
    if (hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost)) return 1;
    for (int i = 0; i < n; ++i)
        printf("in (%g, %g)  bf16 clamp %08x = (%g, %g)  f16 clamp %08x = (%g, %g)\n", h[2 * i], h[2 * i + 1], o[i],
               bf(o[i] & 0xffff), bf(o[i] >> 16), o[64 + i], hf(o[64 + i] & 0xffff), hf(o[64 + i] >> 16));
    return 0;
}
