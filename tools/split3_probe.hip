// split3_probe.hip -- diagnostic for DESIGN.md section 9 item 0: fp32-class hidden layers on the
// 16-bit matrix core by a three-term split (a = ah + al, w = wh + wl, a.w ~ ah.wh + ah.wl + al.wh,
// f32 accumulate) against one 16-bit term, on the plane_1 shape (7 hidden 32x32 ReLU layers).
// Not product code: it measures throughput (2^22 points) and the error against an fp64 chain
// and an f32 sequential-fma chain (the fp32 mode's arithmetic) on the CPU.
// Inputs are generated in-kernel (24-bit integer hashes, exact in f32 on both sides), so the
// timing is the MLP alone.  Layout as the product's reduced-precision MLP (nr_mlp16.h): a
// wave's 64 points form two 32-point tiles of v_mfma_f32_32x32x16_{f16,bf16}; the f32 result
// is its own next B operand (registers 8s..8s+7 = k-step s; the weights' columns are permuted
// to match on the host).
// build: hipcc --offload-arch=gfx950 -O3 split3_probe.hip -o bin/split3_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int NL = 7;  // hidden 32x32 layers

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

// input unit k of point p: a 24-bit integer hash scaled by 2^-24 (exact in f32)
__host__ __device__ inline float input_of(uint32_t p, uint32_t k) {
    uint32_t h = p * 2654435761u + k * 40503u + 0x9e3779b9u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}
// output row of accumulator register r in lane half h (v_mfma_f32_32x32x16 D layout)
__host__ __device__ inline int row_of(int r, int h) { return (r / 4) * 8 + 4 * h + (r % 4); }
// input unit of k-step s, lane half h, slot i: the row the previous layer left in register 8s+i
__host__ __device__ inline int col_of(int s, int h, int i) { return row_of(8 * s + i, h); }

// MODE 0: one f16 term; 1: f16 three-term split; 2: bf16 three-term split; 3: one bf16 term
template <int MODE>
__global__ __launch_bounds__(256, 4) void k_probe(const uint4 *__restrict__ Ah, const uint4 *__restrict__ Al,
                                                  const float *__restrict__ bias, float *__restrict__ out, long n, int nl) {
    constexpr bool BF = MODE >= 2;
    typedef typename std::conditional<BF, bf16x8, f16x8>::type v8;
    typedef typename std::conditional<BF, __bf16, _Float16>::type e16;
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    for (long c = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); c * 64 < n; c += nw) {
        f32x16 acc[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t p = (uint32_t)(c * 64 + 32 * t + (lane & 31));
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = input_of(p, row_of(r, h));
        }
#pragma unroll 1
        for (int ll = 0; ll < nl; ++ll) {
            const int l = ll % NL;  // nl > NL repeats the layers: the marginal cost of a layer
            v8 wh[2], wl[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                wh[s] = __builtin_bit_cast(v8, Ah[(l * 2 + s) * 64 + lane]);
                wl[s] = __builtin_bit_cast(v8, Al[(l * 2 + s) * 64 + lane]);
            }
            f32x16 b;
#pragma unroll
            for (int r = 0; r < 16; ++r) b[r] = bias[l * 32 + row_of(r, h)];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                v8 xh[2], xl[2];
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const float a = ll == 0 ? acc[t][8 * s + i] : fmaxf(acc[t][8 * s + i], 0.0f);
                        const e16 hi = (e16)a;
                        xh[s][i] = hi;
                        if (MODE == 1 || MODE == 2) xl[s][i] = (e16)(a - (float)hi);
                    }
                f32x16 d = b;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    if constexpr (BF) {
                        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[s], xh[s], d, 0, 0, 0);
                        if (MODE == 2) {
                            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh[s], xl[s], d, 0, 0, 0);
                            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl[s], xh[s], d, 0, 0, 0);
                        }
                    } else {
                        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[s], xh[s], d, 0, 0, 0);
                        if (MODE == 1) {
                            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[s], xl[s], d, 0, 0, 0);
                            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl[s], xh[s], d, 0, 0, 0);
                        }
                    }
                }
                acc[t] = d;
            }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            float sum = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) sum += fmaxf(acc[t][r], 0.0f);
            sum += __shfl_xor(sum, 32);
            const long p = c * 64 + 32 * t + (lane & 31);
            if (h == 0 && p < n) out[p] = sum;
        }
    }
}

// A tuned f16 variant (closer to k_mlp16's code shape): A operands and the D-layout biases
// staged in LDS, NLT layers (repeating the NL weight sets; unrolling them spills the hoisted weights),
// packed conversions (v_cvt_pk_f16_f32 pairs; the split's residual from the unpacked high
// halves).  SPLIT: the three-term split; otherwise one f16 term.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool SPLIT, int NLT>
__global__ __launch_bounds__(256, 4) void k_tuned(const uint4 *__restrict__ Ah, const uint4 *__restrict__ Al,
                                                  const float *__restrict__ biasD, float *__restrict__ out, long n) {
    __shared__ uint4 sAh[NL * 2 * 64], sAl[NL * 2 * 64];
    __shared__ f32x16 sB[NL * 2];
    for (int i = threadIdx.x; i < NL * 2 * 64; i += blockDim.x) {
        sAh[i] = Ah[i];
        if (SPLIT) sAl[i] = Al[i];
    }
    for (int i = threadIdx.x; i < NL * 2 * 16; i += blockDim.x) reinterpret_cast<float *>(sB)[i] = biasD[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    for (long c = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); c * 64 < n; c += nw) {
        f32x16 acc[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t p = (uint32_t)(c * 64 + 32 * t + (lane & 31));
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = input_of(p, row_of(r, h));
        }
#pragma unroll 1
        for (int ll = 0; ll < NLT; ++ll) {
            const int l = ll % NL;
            f16x8 wh[2], wl[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                wh[s] = __builtin_bit_cast(f16x8, sAh[(l * 2 + s) * 64 + lane]);
                if (SPLIT) wl[s] = __builtin_bit_cast(f16x8, sAl[(l * 2 + s) * 64 + lane]);
            }
            const f32x16 b = sB[l * 2 + h];
            f16x8 xh[2][2], xl[2][2];
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    u32x4 hw, lw;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        f32x2 v = {acc[t][8 * s + 2 * q], acc[t][8 * s + 2 * q + 1]};
                        if (ll > 0) v = __builtin_elementwise_max(v, (f32x2){0.0f, 0.0f});
                        const f16x2 hi = __builtin_convertvector(v, f16x2);
                        hw[q] = __builtin_bit_cast(uint32_t, hi);
                        if (SPLIT) lw[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v - __builtin_convertvector(hi, f32x2), f16x2));
                    }
                    xh[t][s] = __builtin_bit_cast(f16x8, hw);
                    if (SPLIT) xl[t][s] = __builtin_bit_cast(f16x8, lw);
                }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                f32x16 d = b;
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[s], xh[t][s], d, 0, 0, 0);
                    if (SPLIT) {
                        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[s], xl[t][s], d, 0, 0, 0);
                        d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl[s], xh[t][s], d, 0, 0, 0);
                    }
                }
                acc[t] = d;
            }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            float sum = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) sum += fmaxf(acc[t][r], 0.0f);
            sum += __shfl_xor(sum, 32);
            const long p = c * 64 + 32 * t + (lane & 31);
            if (h == 0 && p < n) out[p] = sum;
        }
    }
}

static uint16_t f16_bits(float v) {
    _Float16 x = (_Float16)v;
    uint16_t b;
    memcpy(&b, &x, 2);
    return b;
}
static float f16_val(uint16_t b) {
    _Float16 x;
    memcpy(&x, &b, 2);
    return (float)x;
}
static uint16_t bf16_bits(float v) {  // round to nearest even
    uint32_t u;
    memcpy(&u, &v, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static float bf16_val(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float v;
    memcpy(&v, &u, 4);
    return v;
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : (1l << 22);
    const int reps = 10, ncheck = 8192;
    // weights ~ U(-0.35, 0.35), biases ~ U(-0.05, 0.05): activations stay O(1) over 7 layers
    std::vector<float> W(NL * 32 * 32), B(NL * 32);
    uint64_t st = 12345;
    auto rnd = [&]() {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        return (float)((st >> 40) & 0xffffff) / 16777216.0f;
    };
    for (auto &w : W) w = (rnd() - 0.5f) * 0.7f;
    for (auto &b : B) b = (rnd() - 0.5f) * 0.1f;
    // A operands: lane l, k-step s, slot i = W[l & 31][col_of(s, l >> 5, i)] as hi / lo
    std::vector<uint16_t> ah[2], al[2];  // [0] f16, [1] bf16
    for (int f = 0; f < 2; ++f) {
        ah[f].resize(NL * 2 * 64 * 8);
        al[f].resize(NL * 2 * 64 * 8);
    }
    for (int l = 0; l < NL; ++l)
        for (int s = 0; s < 2; ++s)
            for (int ln = 0; ln < 64; ++ln)
                for (int i = 0; i < 8; ++i) {
                    const float w = W[(l * 32 + (ln & 31)) * 32 + col_of(s, ln >> 5, i)];
                    const size_t o = ((size_t)(l * 2 + s) * 64 + ln) * 8 + i;
                    ah[0][o] = f16_bits(w);
                    al[0][o] = f16_bits(w - f16_val(ah[0][o]));
                    ah[1][o] = bf16_bits(w);
                    al[1][o] = bf16_bits(w - bf16_val(ah[1][o]));
                }
    // CPU references on the first ncheck points: fp64, and the f32 sequential-fma chain
    std::vector<double> ref(ncheck);
    std::vector<float> ref32(ncheck);
    for (int p = 0; p < ncheck; ++p) {
        double x[32], y[32];
        float xf[32], yf[32];
        for (int k = 0; k < 32; ++k) xf[k] = input_of((uint32_t)p, (uint32_t)k), x[k] = xf[k];
        for (int l = 0; l < NL; ++l) {
            for (int m = 0; m < 32; ++m) {
                double a = 0;
                float af = 0.0f;
                for (int k = 0; k < 32; ++k) {
                    const double in = l == 0 ? x[k] : std::max(x[k], 0.0);
                    const float inf = l == 0 ? xf[k] : std::max(xf[k], 0.0f);
                    a += (double)W[(l * 32 + m) * 32 + k] * in;
                    af = std::fma(W[(l * 32 + m) * 32 + k], inf, af);
                }
                y[m] = a + B[l * 32 + m];
                yf[m] = af + B[l * 32 + m];
            }
            memcpy(x, y, sizeof x);
            memcpy(xf, yf, sizeof xf);
        }
        double s = 0;
        float sf = 0.0f;
        for (int m = 0; m < 32; ++m) s += std::max(x[m], 0.0), sf += std::max(xf[m], 0.0f);
        ref[p] = s;
        ref32[p] = sf;
    }
    double e32 = 0, mag = 0;
    for (int p = 0; p < ncheck; ++p) e32 = std::max(e32, std::fabs(ref32[p] - ref[p])), mag = std::max(mag, std::fabs(ref[p]));
    printf("points %ld, hidden layers %d, max |ref| %.4f; f32 sequential-fma chain: max abs err %.3e\n", n, NL, mag, e32);

    uint4 *dAh[2], *dAl[2];
    float *dB, *dOut;
    for (int f = 0; f < 2; ++f) {
        CHECK(hipMalloc(&dAh[f], ah[f].size() * 2));
        CHECK(hipMalloc(&dAl[f], al[f].size() * 2));
        CHECK(hipMemcpy(dAh[f], ah[f].data(), ah[f].size() * 2, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dAl[f], al[f].data(), al[f].size() * 2, hipMemcpyHostToDevice));
    }
    std::vector<float> BD(NL * 2 * 16);  // biases in the D layout: [layer][half][register]
    for (int l = 0; l < NL; ++l)
        for (int hh = 0; hh < 2; ++hh)
            for (int r = 0; r < 16; ++r) BD[(l * 2 + hh) * 16 + r] = B[l * 32 + row_of(r, hh)];
    float *dBD;
    CHECK(hipMalloc(&dBD, BD.size() * 4));
    CHECK(hipMemcpy(dBD, BD.data(), BD.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dB, B.size() * 4));
    CHECK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dOut, n * 4));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount * 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char *names[6] = {"f16 x1", "f16 x3 split", "bf16 x3 split", "bf16 x1", "f16 x1 tuned", "f16 x3 tuned"};
    std::vector<float> out(ncheck);
    for (int mode = 0; mode < 6; ++mode) {
        const int f = (mode == 2 || mode == 3) ? 1 : 0;
        auto launch = [&](int nl) {
            if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dB, dOut, n, nl);
            if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dB, dOut, n, nl);
            if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dB, dOut, n, nl);
            if (mode == 3) hipLaunchKernelGGL(k_probe<3>, dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dB, dOut, n, nl);
            if (mode == 4 && nl == NL) hipLaunchKernelGGL((k_tuned<false, NL>), dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dBD, dOut, n);
            if (mode == 4 && nl != NL) hipLaunchKernelGGL((k_tuned<false, 2 * NL>), dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dBD, dOut, n);
            if (mode == 5 && nl == NL) hipLaunchKernelGGL((k_tuned<true, NL>), dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dBD, dOut, n);
            if (mode == 5 && nl != NL) hipLaunchKernelGGL((k_tuned<true, 2 * NL>), dim3(grid), dim3(256), 0, 0, dAh[f], dAl[f], dBD, dOut, n);
        };
        float ms2 = 0.0f, ms = 0.0f;
        for (int nl : {2 * NL, NL}) {  // the last pass (NL layers) is the one checked
            launch(nl);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) launch(nl);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            if (nl == 2 * NL) { ms2 = ms; continue; }
        }
        CHECK(hipMemcpy(out.data(), dOut, ncheck * 4, hipMemcpyDeviceToHost));
        double err = 0;
        for (int p = 0; p < ncheck; ++p) err = std::max(err, std::fabs((double)out[p] - ref[p]));
        const double tf = (double)n * NL * 2 * 32 * 32 / (ms * 1e-3) / 1e12;
        const double tfm = (double)n * NL * 2 * 32 * 32 / ((ms2 - ms) * 1e-3) / 1e12;
        printf("%-14s %8.4f ms  %7.1f TFLOP/s (hidden-layer FLOP)  max abs err vs fp64 %.3e;  %d layers %.4f ms: marginal %.1f TFLOP/s per added layer\n",
               names[mode], ms, tf, err, 2 * NL, ms2, tfm);
    }
    return 0;
}
