// Probe (GPU box): do packed-FP32 VALU ops (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32) give
// wrong lanes while another wave on the same SIMD runs MFMAs?
//   hipcc --offload-arch=gfx950 -O2 tools/pk_mfma_probe.hip -o tools/bin/pk_mfma_probe
//   tools/bin/pk_mfma_probe
// Workgroups of 8 waves (2 per SIMD).  Even waves run a chain of MFMAs of kind K; odd waves
// evaluate the same products twice, once with packed-FP32 instructions and once with plain
// v_mul_f32 / v_add_f32 / v_fma_f32, and count lanes where the two disagree (by quarter-wave).
// K: 0 no MFMA (odd and even waves both run the packed check), 1 v_mfma_f32_32x32x16_f16,
// 2 v_mfma_f32_32x32x16_bf16, 3 v_mfma_f32_16x16x4_f32, 4 v_mfma_f32_16x16x32_f16,
// 5 v_mfma_f32_16x16x32_bf16.  OP: 0 v_pk_mul_f32 (op_sel) + v_pk_fma_f32, 1 v_pk_mul_f32,
// 2 v_pk_add_f32, 3 v_pk_fma_f32, 4 v_pk_mov_b32 (op_sel), each checked against plain VALU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 2048;

template <int K, int OP>
__global__ __launch_bounds__(512) void probe(unsigned *bad, float *sink, unsigned seed) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned h = seed * 2654435761u + (blockIdx.x * 512 + threadIdx.x) * 40503u;
    if (K != 0 && (wave & 1) == 0) {
        f16v acc = {};
        f4 acc4 = {};
        h8 a, b;
        b8 ab, bb;
        for (int i = 0; i < 8; ++i) {
            a[i] = (_Float16)(float)((h >> i) & 3);
            b[i] = (_Float16)(float)((h >> (i + 2)) & 3);
            ab[i] = (__bf16)(float)((h >> i) & 3);
            bb[i] = (__bf16)(float)((h >> (i + 2)) & 3);
        }
        for (int it = 0; it < ITERS / 4; ++it) {
            if constexpr (K == 1) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
            else if constexpr (K == 2) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, acc, 0, 0, 0);
            else if constexpr (K == 4) acc4 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc4, 0, 0, 0);
            else if constexpr (K == 5) acc4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, acc4, 0, 0, 0);
            else acc4 = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(h & 7), (float)lane, acc4, 0, 0, 0);
        }
        sink[blockIdx.x * 512 + threadIdx.x] = acc[0] + acc[15] + acc4[0];
        return;
    }
    f2 x = {1.0f + (float)(h & 1023) / 1024.0f, 0.5f + (float)((h >> 10) & 1023) / 512.0f};
    f2 y = {0.75f + (float)lane / 64.0f, 1.25f - (float)lane / 128.0f};
    unsigned nbad[4] = {0, 0, 0, 0};
    for (int it = 0; it < ITERS; ++it) {
        f2 p, q;
        float s0, s1;
        if constexpr (OP == 0) {  // p = x * y.yx (op_sel), q = fma(p, x, y)
            asm volatile("v_pk_mul_f32 %0, %2, %3 op_sel:[0,1] op_sel_hi:[1,0]\n\t"
                         "v_pk_fma_f32 %1, %0, %2, %3"
                         : "=&v"(p), "=&v"(q) : "v"(x), "v"(y));
            s0 = __builtin_fmaf(x.x * y.y, x.x, y.x);
            s1 = __builtin_fmaf(x.y * y.x, x.y, y.y);
        } else if constexpr (OP == 1) {
            asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(q) : "v"(x), "v"(y));
            s0 = x.x * y.x; s1 = x.y * y.y;
        } else if constexpr (OP == 2) {
            asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(q) : "v"(x), "v"(y));
            s0 = x.x + y.x; s1 = x.y + y.y;
        } else if constexpr (OP == 3) {
            asm volatile("v_pk_fma_f32 %0, %1, %2, %1" : "=v"(q) : "v"(x), "v"(y));
            s0 = __builtin_fmaf(x.x, y.x, x.x); s1 = __builtin_fmaf(x.y, y.y, x.y);
        } else {
            asm volatile("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(q) : "v"(x), "v"(y));
            s0 = x.y; s1 = y.x;
        }
        asm volatile("" : "+v"(s0), "+v"(s1));
        if (__float_as_uint(q.x) != __float_as_uint(s0) || __float_as_uint(q.y) != __float_as_uint(s1)) ++nbad[lane >> 4];
        (void)p;
        x.x = 1.0f + (float)((__float_as_uint(s0) >> 5) & 1023) / 1024.0f;
        x.y = 0.5f + (float)((__float_as_uint(s1) >> 7) & 1023) / 512.0f;
    }
    for (int k = 0; k < 4; ++k)
        if (nbad[k]) atomicAdd(bad + k, nbad[k]);
}

template <int K, int OP>
static void check(const char *name) {
    unsigned *bad;
    float *sink;
    const int blocks = 256 * 2;
    if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&sink, (size_t)blocks * 512 * 4) != hipSuccess) exit(1);
    unsigned tot[4] = {0, 0, 0, 0};
    for (unsigned seed = 1; seed <= 8; ++seed) {
        (void)hipMemset(bad, 0, 16);
        hipLaunchKernelGGL((probe<K, OP>), dim3(blocks), dim3(512), 0, 0, bad, sink, seed);
        unsigned hb[4];
        if (hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost) != hipSuccess) exit(1);
        for (int k = 0; k < 4; ++k) tot[k] += hb[k];
    }
    printf("%-36s packed != scalar: lanes 0-15 %u, 16-31 %u, 32-47 %u, 48-63 %u\n", name, tot[0], tot[1], tot[2], tot[3]);
    (void)hipFree(bad);
    (void)hipFree(sink);
}

template <int OP>
static void all(const char *op) {
    printf("-- %s\n", op);
    check<0, OP>("no MFMA waves");
    check<1, OP>("beside v_mfma_f32_32x32x16_f16");
    check<2, OP>("beside v_mfma_f32_32x32x16_bf16");
    check<4, OP>("beside v_mfma_f32_16x16x32_f16");
    check<5, OP>("beside v_mfma_f32_16x16x32_bf16");
    check<3, OP>("beside v_mfma_f32_16x16x4_f32");
}

int main() {
    all<0>("v_pk_mul_f32 op_sel + v_pk_fma_f32");
    all<1>("v_pk_mul_f32");
    all<2>("v_pk_add_f32");
    all<3>("v_pk_fma_f32");
    all<4>("v_pk_mov_b32 op_sel");
    return 0;
}
