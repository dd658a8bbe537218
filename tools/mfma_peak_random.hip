// mfma_peak_random.hip -- the 16-bit matrix core's sustained rate on RANDOM operands, with the
// clock the chip holds while it runs (r1_mfma_peak.txt used constant operands,
// which hold ~2.4 GHz and hide the DVFS give-back, MI355X_MICROARCH.md "DVFS give-back" 1, 6, 7).
//
// Per shape (v_mfma_f32_32x32x16_{bf16,f16}, v_mfma_f32_16x16x32_{bf16,f16}) and waves per SIMD
// (1..4): back-to-back independent MFMAs whose A/B operands are four different random register
// sets per wave (uniform in [-1, 1), every lane and register different), ~20 ms per launch, after
// >= 2 s of back-to-back launches of the same kernel.  Each wave stamps s_memtime and
// s_memrealtime around its loop into a buffer of its own; the clock is the median over waves of
// delta(s_memtime) / delta(s_memrealtime) x 100 MHz.  Prints wall TF/s, the fraction of the
// 2.5166 PF spec peak (2.4 GHz), the clock, and TF/s per GHz.
// build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 mfma_peak_random.hip -o bin/mfma_peak_random
// (the VGPR form: in the default AGPR form hipcc shuffled the 16x16x32 loop's accumulators between
// every trip, v_accvgpr_read/write/mov, which halved that loop's rate)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float rnd(uint32_t &s) {
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    return (float)(s >> 8) * (2.0f / 16777216.0f) - 1.0f;
}

template <typename V>
__device__ __forceinline__ V rnd8(uint32_t &s) {
    V v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (decltype(v[0] + 0))rnd(s);
    return v;
}

// SHAPE 0: 32x32x16 (32768 FLOP, 4 accumulators), 1: 16x16x32 (16384 FLOP, 8 accumulators)
template <int SHAPE, bool BF>
__global__ __launch_bounds__(256) void k_peak(float *out, unsigned long long *st, int iters, uint32_t seed) {
    typedef typename std::conditional<BF, bf16x8, f16x8>::type V;
    uint32_t s = seed ^ (blockIdx.x * 7919u + threadIdx.x * 104729u + 12345u);
    for (int i = 0; i < 4; ++i) rnd(s);
    V a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = rnd8<V>(s); b[i] = rnd8<V>(s); }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float sum = 0.0f;
    if constexpr (SHAPE == 0) {
        f32x16 c[4] = {};
        // four iterations per trip, so that every operand index is a constant (a run-time rotation
        // became select chains over the whole register array)
        for (int it = 0; it < iters; it += 4)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if constexpr (BF) c[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[(i + r) & 3], c[i], 0, 0, 0);
                    else c[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[(i + r) & 3], c[i], 0, 0, 0);
                }
        for (int i = 0; i < 4; ++i) sum += c[i][0] + c[i][15];
    } else {
        f32x4 c[8] = {};
        for (int it = 0; it < iters; it += 4)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if constexpr (BF) c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 3], b[(i + r) & 3], c[i], 0, 0, 0);
                    else c[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i & 3], b[(i + r) & 3], c[i], 0, 0, 0);
                }
        for (int i = 0; i < 8; ++i) sum += c[i][0] + c[i][3];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = sum;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        st[2 * w] = t1 - t0;
        st[2 * w + 1] = r1 - r0;
    }
}

int main() {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0)) return 1;
    const int cus = prop.multiProcessorCount;
    float *out;
    unsigned long long *st;
    if (hipMalloc(&out, (size_t)cus * 4 * 256 * 4) || hipMalloc(&st, (size_t)cus * 16 * 2 * 8)) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) || hipEventCreate(&e1)) return 1;
    printf("# random operands, %d CUs; spec peak 2516.6 TF/s (16-bit dense, 2.4 GHz)\n", cus);
    for (int kind = 0; kind < 4; ++kind) {
        const int shape = kind >> 1;
        const bool bf = (kind & 1) == 0;
        const double flop_per = shape == 0 ? 32768.0 : 16384.0;
        const int per_it = shape == 0 ? 4 : 8;
        for (int wps = 1; wps <= 4; ++wps) {
            const int grid = cus * wps;
            // ~20 ms per launch at ~1.8 GHz: 3.6e7 cycles / (32 cycles per MFMA-slot of the SIMD)
            const int iters = ((int)(3.6e7 / 32.0 / per_it / wps) * (shape == 0 ? 1 : 2)) & ~3;
            auto launch = [&]() {
                const uint32_t seed = 0x9e3779b9u;
                if (kind == 0) hipLaunchKernelGGL((k_peak<0, true>), dim3(grid), dim3(256), 0, 0, out, st, iters, seed);
                else if (kind == 1) hipLaunchKernelGGL((k_peak<0, false>), dim3(grid), dim3(256), 0, 0, out, st, iters, seed);
                else if (kind == 2) hipLaunchKernelGGL((k_peak<1, true>), dim3(grid), dim3(256), 0, 0, out, st, iters, seed);
                else hipLaunchKernelGGL((k_peak<1, false>), dim3(grid), dim3(256), 0, 0, out, st, iters, seed);
            };
            // >= 2 s of back-to-back launches first (the clock settles under load)
            for (int r = 0; r < 100; ++r) launch();
            if (hipDeviceSynchronize()) return 1;
            const int reps = 10;
            if (hipEventRecord(e0, 0)) return 1;
            for (int r = 0; r < reps; ++r) launch();
            if (hipEventRecord(e1, 0) || hipEventSynchronize(e1)) return 1;
            float ms = 0;
            if (hipEventElapsedTime(&ms, e0, e1)) return 1;
            ms /= reps;
            std::vector<unsigned long long> h((size_t)grid * 4 * 2);
            if (hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost)) return 1;
            std::vector<double> clk, cyc;
            for (int w = 0; w < grid * 4; ++w) {
                clk.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);  // GHz
                cyc.push_back((double)h[2 * w]);
            }
            std::sort(clk.begin(), clk.end());
            std::sort(cyc.begin(), cyc.end());
            const double ghz = clk[clk.size() / 2];
            const double flop = (double)grid * 4 * iters * per_it * flop_per;
            const double tf = flop / (ms * 1e-3) / 1e12;
            // the median wave's loop cycles per MFMA of its own (wps waves share a SIMD: divided by wps
            // when they overlap for the whole loop, which the resident grid does not guarantee)
            const double cpm = cyc[cyc.size() / 2] / ((double)iters * per_it);
            printf("%s %s  waves/SIMD %d: %7.3f ms  %7.1f TF/s  %.3f of spec  clock %.3f GHz (p10 %.3f p90 %.3f)  "
                   "%.1f TF/s per GHz  wave %.2f cyc/MFMA\n",
                   shape == 0 ? "32x32x16" : "16x16x32", bf ? "bf16" : "f16 ", wps, ms, tf, tf / 2516.6, ghz,
                   clk[clk.size() / 10], clk[clk.size() * 9 / 10], tf / ghz, cpm);
            fflush(stdout);
        }
    }
    return 0;
}
