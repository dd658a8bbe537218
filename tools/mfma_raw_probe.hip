// Probe (GPU box): wait states around v_mfma_f32_32x32x16_{f16,bf16} under full-chip contention.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_raw_probe.hip -o tools/bin/mfma_raw_probe
//   tools/bin/mfma_raw_probe [blocks_per_cu]
// hipcc pads 12 wait states between an 8-pass XDL MFMA and a VALU that reads or writes its
// destination, and 2 between a VALU write and an MFMA that reads it.  Each mode runs a chain
// of MFMAs per wave (accumulator pinned to v[0:15]) and, with exactly N wait states,
//   R: reads every result register with VALU (v_xor_b32 pairs at N, N+1, ... N+7),
//   W: overwrites result registers v0 and v15 with VALU (does a late write-back undo it?),
//   B: issues the MFMA N states after a VALU write of its B operand,
// and compares every lane's samples with the same program padded to 40 wait states.  A
// nonzero count means N wait states are not enough on this chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 64;
constexpr int NOUT = 24;  // per lane: 16 accumulator words + 8 sample words

#define N1 "s_nop 0\n\t"
#define N2 "s_nop 1\n\t"
#define N10 "s_nop 9\n\t"
#define N11 "s_nop 10\n\t"
#define N12 "s_nop 11\n\t"
#define N14 "s_nop 13\n\t"
#define N40 "s_nop 15\n\ts_nop 15\n\ts_nop 7\n\t"
#define SETTLE "s_nop 15\n\ts_nop 15\n\ts_nop 15\n\t"

#define PRELUDE                                                                                   \
    const unsigned h = seed * 2654435761u + (blockIdx.x * 256 + threadIdx.x) * 40503u;            \
    f16x8 A, B;                                                                                   \
    for (int i = 0; i < 8; ++i) {                                                                 \
        A[i] = (_Float16)(int)(((h >> (i * 3)) % 5) - 2);                                         \
        B[i] = (_Float16)(int)(((h >> (i * 3 + 1)) % 5) - 2);                                     \
    }                                                                                             \
    const u32x4 a = __builtin_bit_cast(u32x4, A), b = __builtin_bit_cast(u32x4, B);               \
    f32x16 acc = {};                                                                              \
    unsigned smp[8] = {0, 0, 0, 0, 0, 0, 0, 0};

#define EPILOGUE                                                                                  \
    float *o = out + ((size_t)blockIdx.x * 256 + threadIdx.x) * NOUT;                             \
    for (int i = 0; i < 16; ++i) o[i] = acc[i];                                                   \
    for (int i = 0; i < 8; ++i) o[16 + i] = __uint_as_float(smp[i]);

// R: VALU reads of the result, the first N wait states after the MFMA
#define KERNEL_R(NAME, OP, NOPS)                                                                  \
    __global__ __launch_bounds__(256) void NAME(float *out, unsigned seed) {                      \
        PRELUDE                                                                                   \
        for (int it = 0; it < ITERS; ++it) {                                                      \
            unsigned r[8];                                                                        \
            asm volatile("s_nop 4\n\t" OP " v[0:15], %9, %10, v[0:15]\n\t" NOPS                    \
                         "v_xor_b32 %0, v0, v1\n\tv_xor_b32 %1, v2, v3\n\t"                        \
                         "v_xor_b32 %2, v4, v5\n\tv_xor_b32 %3, v6, v7\n\t"                        \
                         "v_xor_b32 %4, v8, v9\n\tv_xor_b32 %5, v10, v11\n\t"                      \
                         "v_xor_b32 %6, v12, v13\n\tv_xor_b32 %7, v14, v15\n\t" SETTLE             \
                         : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]),        \
                           "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]), "+{v[0:15]}"(acc)                \
                         : "v"(a), "v"(b));                                                       \
            for (int i = 0; i < 8; ++i) smp[i] = smp[i] * 31u + r[i];                             \
        }                                                                                         \
        EPILOGUE                                                                                  \
    }

// W: VALU writes of result registers v0 and v15 N wait states after the MFMA
#define KERNEL_W(NAME, OP, NOPS)                                                                  \
    __global__ __launch_bounds__(256) void NAME(float *out, unsigned seed) {                      \
        PRELUDE                                                                                   \
        for (int it = 0; it < ITERS; ++it) {                                                      \
            unsigned r0, r1;                                                                      \
            asm volatile("s_nop 4\n\t" OP " v[0:15], %3, %4, v[0:15]\n\t" NOPS                    \
                         "v_mov_b32 v15, %5\n\tv_mov_b32 v0, %5\n\t" SETTLE                        \
                         "v_mov_b32 %0, v15\n\tv_mov_b32 %1, v0\n\t"                               \
                         : "=&v"(r0), "=&v"(r1), "+{v[0:15]}"(acc)                                 \
                         : "v"(a), "v"(b), "v"((float)(it & 7)));                                 \
            smp[0] = smp[0] * 31u + r0;                                                           \
            smp[1] = smp[1] * 31u + r1;                                                           \
        }                                                                                         \
        EPILOGUE                                                                                  \
    }

// B: the MFMA N wait states after a VALU write of its B operand (b alternates with b')
#define KERNEL_B(NAME, OP, NOPS)                                                                  \
    __global__ __launch_bounds__(256) void NAME(float *out, unsigned seed) {                      \
        PRELUDE                                                                                   \
        const unsigned b2 = b.x ^ 0x00010001u; /* flips the low mantissa bit of both halves */    \
        for (int it = 0; it < ITERS; ++it) {                                                      \
            u32x4 bb = b;                                                                         \
            asm volatile(SETTLE "v_mov_b32 v20, %3\n\t" NOPS OP " v[0:15], %2, v[20:23], v[0:15]\n\t" \
                         SETTLE "v_mov_b32 v20, %4\n\t" N2                                         \
                         : "+{v[0:15]}"(acc), "+{v[20:23]}"(bb)                                    \
                         : "v"(a), "v"((it & 1) ? b2 : b.x), "v"(b.x));                           \
        }                                                                                         \
        EPILOGUE                                                                                  \
    }

#define F16 "v_mfma_f32_32x32x16_f16"
#define BF16 "v_mfma_f32_32x32x16_bf16"
KERNEL_R(r_f16_40, F16, N40)
KERNEL_R(r_f16_10, F16, N10)
KERNEL_R(r_f16_11, F16, N11)
KERNEL_R(r_f16_12, F16, N12)
KERNEL_R(r_f16_14, F16, N14)
KERNEL_R(r_bf16_40, BF16, N40)
KERNEL_R(r_bf16_12, BF16, N12)
KERNEL_W(w_f16_40, F16, N40)
KERNEL_W(w_f16_10, F16, N10)
KERNEL_W(w_f16_11, F16, N11)
KERNEL_W(w_f16_12, F16, N12)
KERNEL_W(w_bf16_40, BF16, N40)
KERNEL_W(w_bf16_12, BF16, N12)
KERNEL_B(b_f16_40, F16, N40)
KERNEL_B(b_f16_1, F16, N1)
KERNEL_B(b_f16_2, F16, N2)
KERNEL_B(b_bf16_40, BF16, N40)
KERNEL_B(b_bf16_2, BF16, N2)

typedef void (*kfn)(float *, unsigned);

static std::vector<float> run(kfn k, int blocks, unsigned seed) {
    float *d;
    const size_t n = (size_t)blocks * 256 * NOUT;
    if (hipMalloc(&d, n * 4) != hipSuccess) exit(1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, seed);
    std::vector<float> h(n);
    if (hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) exit(1);
    (void)hipFree(d);
    return h;
}

static void cmp(const char *name, kfn ref, kfn x, int blocks) {
    size_t badw = 0, waves = 0;
    for (unsigned seed = 1; seed <= 3; ++seed) {
        const auto r = run(ref, blocks, seed), v = run(x, blocks, seed);
        const size_t nw = r.size() / (64 * NOUT);
        waves += nw;
        for (size_t w = 0; w < nw; ++w) {
            bool bad = false;
            for (size_t i = w * 64 * NOUT; i < (w + 1) * 64 * NOUT; ++i)
                bad |= __builtin_bit_cast(unsigned, r[i]) != __builtin_bit_cast(unsigned, v[i]);
            badw += bad;
        }
    }
    printf("%-40s %zu of %zu waves differ from the 40-state reference\n", name, badw, waves);
}

int main(int argc, char **argv) {
    const int blocks = 256 * (argc > 1 ? atoi(argv[1]) : 4);
    cmp("R f16: reference again", r_f16_40, r_f16_40, blocks);
    cmp("R f16: VALU read at 10", r_f16_40, r_f16_10, blocks);
    cmp("R f16: VALU read at 11", r_f16_40, r_f16_11, blocks);
    cmp("R f16: VALU read at 12", r_f16_40, r_f16_12, blocks);
    cmp("R f16: VALU read at 14", r_f16_40, r_f16_14, blocks);
    cmp("R bf16: VALU read at 12", r_bf16_40, r_bf16_12, blocks);
    cmp("W f16: VALU write at 10", w_f16_40, w_f16_10, blocks);
    cmp("W f16: VALU write at 11", w_f16_40, w_f16_11, blocks);
    cmp("W f16: VALU write at 12", w_f16_40, w_f16_12, blocks);
    cmp("W bf16: VALU write at 12", w_bf16_40, w_bf16_12, blocks);
    cmp("B f16: MFMA 1 state after B write", b_f16_40, b_f16_1, blocks);
    cmp("B f16: MFMA 2 states after B write", b_f16_40, b_f16_2, blocks);
    cmp("B bf16: MFMA 2 states after B write", b_bf16_40, b_bf16_2, blocks);
    return 0;
}
