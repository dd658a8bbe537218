// mix_bench.hip -- experiment: can the f32 VALU evaluate part of the MLP beside the
// matrix cores?  On gfx950 the f32 matrix rate (v_mfma_f32_16x16x4_f32) and the f32
// VALU rate (v_pk_fma_f32) are both 64 FLOP/clk/SIMD and the two pipes are separate
// (MI355X_MICROARCH.md, "Wave scheduling"), so an MFMA wave and a VALU wave on one SIMD
// could in principle add up.  Both paths compute the same k-ordered fmaf chains, so
// their outputs must agree bit for bit (checked here).
//
// Roles per wave (block of 4 * nwaves_per_simd waves; wave w runs on SIMD w % 4):
//   MFMA role: mlp16_fp32_nt<4> on 64 points (nr_mlp16.h, the k_trace MLP)
//   VALU role: 2 points per lane (128 per wave) in packed f32, weights wave-uniform
//              (LDS broadcast reads or scalar loads, -DVALU_SGPR)
// Work is dealt in 128-point chunks from one atomic counter (a MFMA wave runs two tiles
// sets of 64 per chunk), so the faster role takes more.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off mix_bench.hip ../cudaneuralrender_amd/csrc/nr_pack.cpp -o bin/mix_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../cudaneuralrender_amd/csrc/nr_mlp16.h"

using namespace nr;

typedef float f32x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// VALU pack (floats): layer 0 W0T [k 4][m 32], b0 [32]; hidden j: WT [k 32][m 32], b [32];
// final: w [32], b [1] (+3 pad).  WT[k][m] = W[m][k] (in-major), so one k step reads 32
// consecutive floats = 8 broadcast float4.
constexpr int VP_L0 = 0, VP_L0B = 128, VP_HID = 160, VP_HSTRIDE = 1024 + 32;
__host__ __device__ inline int vp_final(int nh) { return VP_HID + nh * VP_HSTRIDE; }
__host__ __device__ inline int vp_floats(int nh) { return vp_final(nh) + 36; }

__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

template <bool SG>
__device__ __forceinline__ f32x2 valu_mlp(const float *__restrict__ w, int nh, f32x2 x, f32x2 y, f32x2 z) {
    f32x2 a[32], c[32];
    // layer 0: fma chain over x, y, z from +0, then + bias, ReLU
#pragma unroll
    for (int m = 0; m < 32; ++m) {
        const float w0 = w[VP_L0 + m], w1 = w[VP_L0 + 32 + m], w2 = w[VP_L0 + 64 + m], b = w[VP_L0B + m];
        f32x2 acc = pfma((f32x2){w0, w0}, x, (f32x2){0.0f, 0.0f});
        acc = pfma((f32x2){w1, w1}, y, acc);
        acc = pfma((f32x2){w2, w2}, z, acc);
        acc = acc + (f32x2){b, b};
        a[m] = __builtin_elementwise_max(acc, (f32x2){0.0f, 0.0f});
    }
    for (int jl = 0; jl < nh; ++jl) {
        const float *L = w + VP_HID + jl * VP_HSTRIDE;
#pragma unroll
        for (int m = 0; m < 32; ++m) c[m] = (f32x2){0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < 32; ++k) {
#pragma unroll
            for (int m4 = 0; m4 < 8; ++m4) {
                const float4 wv = reinterpret_cast<const float4 *>(L + k * 32)[m4];
                c[4 * m4 + 0] = pfma((f32x2){wv.x, wv.x}, a[k], c[4 * m4 + 0]);
                c[4 * m4 + 1] = pfma((f32x2){wv.y, wv.y}, a[k], c[4 * m4 + 1]);
                c[4 * m4 + 2] = pfma((f32x2){wv.z, wv.z}, a[k], c[4 * m4 + 2]);
                c[4 * m4 + 3] = pfma((f32x2){wv.w, wv.w}, a[k], c[4 * m4 + 3]);
            }
        }
#pragma unroll
        for (int m = 0; m < 32; ++m) {
            const float b = L[1024 + m];
            a[m] = __builtin_elementwise_max(c[m] + (f32x2){b, b}, (f32x2){0.0f, 0.0f});
        }
    }
    const float *F = w + vp_final(nh);
    f32x2 acc = {0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 32; ++k) acc = pfma((f32x2){F[k], F[k]}, a[k], acc);
    return acc + (f32x2){F[32], F[32]};
}

// One point per lane (the k_trace ray layout): two outputs per v_pk_fma_f32, the
// activation broadcast to both halves.
__device__ __forceinline__ float valu_mlp1(const float *__restrict__ w, int nh, float x, float y, float z) {
    float a[32];
    f32x2 c[16];
#pragma unroll
    for (int m = 0; m < 32; ++m) {
        float acc = __builtin_fmaf(w[VP_L0 + m], x, 0.0f);
        acc = __builtin_fmaf(w[VP_L0 + 32 + m], y, acc);
        acc = __builtin_fmaf(w[VP_L0 + 64 + m], z, acc);
        a[m] = fmaxf(acc + w[VP_L0B + m], 0.0f);
    }
    for (int jl = 0; jl < nh; ++jl) {
        const float *L = w + VP_HID + jl * VP_HSTRIDE;
#pragma unroll
        for (int q = 0; q < 16; ++q) c[q] = (f32x2){0.0f, 0.0f};
        // weights of step k+1 are read while step k computes; the scheduling barriers keep
        // the compiler from hoisting all 32 steps' reads (256 VGPRs)
        float4 wb[2][8];
#pragma unroll
        for (int q = 0; q < 8; ++q) wb[0][q] = reinterpret_cast<const float4 *>(L)[q];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (k + 1 < 32) {
#pragma unroll
                for (int q = 0; q < 8; ++q) wb[(k + 1) & 1][q] = reinterpret_cast<const float4 *>(L + (k + 1) * 32)[q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float4 wv = wb[k & 1][q];
                c[2 * q] = pfma((f32x2){wv.x, wv.y}, (f32x2){a[k], a[k]}, c[2 * q]);
                c[2 * q + 1] = pfma((f32x2){wv.z, wv.w}, (f32x2){a[k], a[k]}, c[2 * q + 1]);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const f32x2 v = __builtin_elementwise_max(c[q] + (f32x2){L[1024 + 2 * q], L[1024 + 2 * q + 1]},
                                                      (f32x2){0.0f, 0.0f});
            a[2 * q] = v.x;
            a[2 * q + 1] = v.y;
        }
    }
    const float *F = w + vp_final(nh);
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; ++k) acc = __builtin_fmaf(F[k], a[k], acc);
    return acc + F[32];
}

struct Args {
    MlpArgs M;
    const float *vpk;  // VALU pack (global)
    int vp_bytes;
    const float *X;
    float *Y;
    long n;            // points (multiple of 128)
    unsigned *ctr;     // [0] chunk counter, [1] chunks done by MFMA waves, [2] by VALU waves
    int valu_mask;     // wave w of the block is a VALU wave iff (valu_mask >> w) & 1
    int valu_mode;     // 1: two points per lane (valu_mlp), 2: one point per lane (valu_mlp1)
};

extern __shared__ __attribute__((aligned(16))) unsigned char smem_mix[];

template <int MODE>  // 0: valu_mlp, weights in LDS; 1: valu_mlp, weights global; 2: valu_mlp1
__global__ __launch_bounds__(768) void k_mix(Args P) {
    constexpr bool SG = MODE == 1;
    float *s32 = reinterpret_cast<float *>(smem_mix);
    float *svp = reinterpret_cast<float *>(smem_mix + P.M.pk_bytes);
    for (int i = threadIdx.x; i < P.M.pk_bytes / 16; i += blockDim.x)
        reinterpret_cast<int4 *>(s32)[i] = reinterpret_cast<const int4 *>(P.M.pk)[i];
    for (int i = threadIdx.x; i < P.vp_bytes / 16; i += blockDim.x)
        reinterpret_cast<int4 *>(svp)[i] = reinterpret_cast<const int4 *>(P.vpk)[i];
    __syncthreads();
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    const bool valu = (P.valu_mask >> wid) & 1;
    const long nchunks = P.n / 128;
    unsigned done = 0;
    while (true) {
        unsigned c = 0;
        if (lane == 0) c = atomicAdd(P.ctr, 1u);
        c = __shfl(c, 0);
        if ((long)c >= nchunks) break;
        const long base = (long)c * 128;
        if (MODE == 2 && valu) {
#pragma unroll 1
            for (int h = 0; h < 2; ++h) {
                const float *p = P.X + (base + 64 * h + lane) * 3;
                P.Y[base + 64 * h + lane] = valu_mlp1(svp, P.M.nh, p[0], p[1], p[2]);
            }
        } else if (MODE != 2 && valu) {
            const float *p0 = P.X + (base + lane) * 3, *p1 = P.X + (base + 64 + lane) * 3;
            const f32x2 x = {p0[0], p1[0]}, y = {p0[1], p1[1]}, z = {p0[2], p1[2]};
            const f32x2 v = valu_mlp<SG>(SG ? P.vpk : svp, P.M.nh, x, y, z);
            P.Y[base + lane] = v.x;
            P.Y[base + 64 + lane] = v.y;
        } else {
#pragma unroll 1
            for (int h = 0; h < 2; ++h) {
                const float *p = P.X + (base + 64 * h + lane) * 3;
                const float v = mlp16_fp32_nt<4>(s32, P.M.in0, P.M.nh, 0.0f, p[0], p[1], p[2]);
                P.Y[base + 64 * h + lane] = v;
            }
        }
        ++done;
    }
    if (lane == 0) atomicAdd(P.ctr + (valu ? 2 : 1), done);
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : (1l << 22);
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const int nh = 7;
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(-0.5f, 0.5f);
    std::vector<int> dims = {3, 32, 32, 32, 32, 32, 32, 32, 32, 1};
    std::vector<std::vector<float>> K(9), B(9);
    for (int l = 0; l < 9; ++l) {
        K[l].resize(dims[l] * dims[l + 1]);
        B[l].resize(dims[l + 1]);
        for (auto &v : K[l]) v = U(rng);
        for (auto &v : B[l]) v = U(rng) * 0.2f;
    }
    std::vector<float> pk;
    if (!pack_fp32_16(dims, K, B, pk)) { fprintf(stderr, "pack failed\n"); return 1; }
    std::vector<float> vp(vp_floats(nh), 0.0f);
    for (int k = 0; k < 3; ++k)
        for (int m = 0; m < 32; ++m) vp[VP_L0 + k * 32 + m] = K[0][k * 32 + m];  // Keras (in x out): K[k][m]
    for (int m = 0; m < 32; ++m) vp[VP_L0B + m] = B[0][m];
    for (int j = 0; j < nh; ++j) {
        for (int k = 0; k < 32; ++k)
            for (int m = 0; m < 32; ++m) vp[VP_HID + j * VP_HSTRIDE + k * 32 + m] = K[j + 1][k * 32 + m];
        for (int m = 0; m < 32; ++m) vp[VP_HID + j * VP_HSTRIDE + 1024 + m] = B[j + 1][m];
    }
    for (int k = 0; k < 32; ++k) vp[vp_final(nh) + k] = K[8][k];
    vp[vp_final(nh) + 32] = B[8][0];

    std::vector<float> X(n * 3);
    std::uniform_real_distribution<float> UX(-1.0f, 1.0f);
    for (auto &v : X) v = UX(rng);
    float *dpk, *dvp, *dX, *dY, *dY2;
    unsigned *dctr;
    CK(hipMalloc(&dpk, pk.size() * 4));
    CK(hipMalloc(&dvp, vp.size() * 4));
    CK(hipMalloc(&dX, n * 12));
    CK(hipMalloc(&dY, n * 4));
    CK(hipMalloc(&dY2, n * 4));
    CK(hipMalloc(&dctr, 64));
    CK(hipMemcpy(dpk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dvp, vp.data(), vp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dX, X.data(), n * 12, hipMemcpyHostToDevice));
    Args P{};
    P.M.pk = dpk;
    P.M.pk_bytes = (int)((pk.size() * 4 + 15) / 16 * 16);
    P.M.in0 = 3;
    P.M.nh = nh;
    P.vpk = dvp;
    P.vp_bytes = (int)((vp.size() * 4 + 15) / 16 * 16);
    P.X = dX;
    P.n = n;
    P.ctr = dctr;
    const int smem = P.M.pk_bytes + P.vp_bytes;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    CK(hipFuncSetAttribute((const void *)k_mix<0>, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    CK(hipFuncSetAttribute((const void *)k_mix<1>, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
    CK(hipFuncSetAttribute((const void *)k_mix<2>, hipFuncAttributeMaxDynamicSharedMemorySize, smem));

    struct Cfg { const char *name; int threads, valu_mask, bpc; bool sg; int mode = 1; };
    const Cfg cfgs[] = {
        {"mfma 4w x2", 256, 0x0, 2, false},      {"mfma 4w x3", 256, 0x0, 3, false},
        {"mfma 8w x1", 512, 0x00, 1, false},
        {"valu-lds 4w x2", 256, 0xf, 2, false},   {"valu-lds 4w x3", 256, 0xf, 3, false},
        {"valu-sgpr 4w x2", 256, 0xf, 2, true},
        {"mix-lds 4m+4v x1", 512, 0xf0, 1, false}, {"mix-lds 8m+4v x1", 768, 0xf00, 1, false},
        {"mix-sgpr 4m+4v x1", 512, 0xf0, 1, true}, {"mix-sgpr 8m+4v x1", 768, 0xf00, 1, true},
        {"mix-lds 4m+4v x2 (2 blocks)", 512, 0xf0, 2, false},
        {"valu1 4w x2", 256, 0xf, 2, false, 2},  {"valu1 4w x3", 256, 0xf, 3, false, 2},
        {"mix-valu1 4m+4v x1", 512, 0xf0, 1, false, 2}, {"mix-valu1 8m+4v x1", 768, 0xf00, 1, false, 2},
    };
    std::vector<float> Yref(n), Yv(n);
    bool have_ref = false;
    for (const Cfg &c : cfgs) {
        P.valu_mask = c.valu_mask;
        P.valu_mode = c.mode;
        P.Y = dY;
        auto launch = [&]() {
            CK(hipMemsetAsync(dctr, 0, 64, 0));
            if (c.mode == 2) hipLaunchKernelGGL(k_mix<2>, dim3(ncu * c.bpc), dim3(c.threads), smem, 0, P);
            else if (c.sg) hipLaunchKernelGGL(k_mix<1>, dim3(ncu * c.bpc), dim3(c.threads), smem, 0, P);
            else hipLaunchKernelGGL(k_mix<0>, dim3(ncu * c.bpc), dim3(c.threads), smem, 0, P);
            CK(hipGetLastError());
        };
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        unsigned ctr[3];
        CK(hipMemcpy(ctr, dctr, 12, hipMemcpyDeviceToHost));
        CK(hipMemcpy(Yv.data(), dY, n * 4, hipMemcpyDeviceToHost));
        long diff = 0;
        if (!have_ref) { Yref = Yv; have_ref = true; }
        else for (long i = 0; i < n; ++i) diff += memcmp(&Yv[i], &Yref[i], 4) != 0;
        const double tf = (double)n * 14592 / (ms * 1e-3) / 1e12;
        printf("%-30s %8.3f ms  %7.2f TF/s (%.3f of 157.3)  chunks mfma %u valu %u  diff %ld\n", c.name, ms, tf,
               tf / 157.3, ctr[1], ctr[2], diff);
        fflush(stdout);
    }
    return 0;
}
