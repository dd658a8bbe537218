// Probe (GPU box): forwarding between ordinary VALU and packed-FP32 VALU (v_pk_*_f32) on gfx950
// under full-chip contention.
//   hipcc --offload-arch=gfx950 -O2 tools/pk_hazard_probe.hip -o tools/bin/pk_hazard_probe
//   tools/bin/pk_hazard_probe [blocks_per_cu]
// Each case runs a producer -> consumer pair back to back (no wait states) inside one asm
// statement, ITERS times per wave, with lane-dependent data, and folds the consumer's result
// into a per-lane checksum; the same pair separated by 8 wait states is the reference.
// Reported: waves whose checksum differs, and which quarter-waves (lanes 0-15, 16-31, 32-47,
// 48-63) the differing lanes were in.  Every case also runs with EXEC limited to lanes 48-63,
// 32-63 and a random mask per iteration (the producer/consumer pair of a divergent region).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int ITERS = 256;
#define PAD "s_nop 7\n\t"

// CASE bodies, registers pinned: out = v[12:13], a = v[10:11], b = v14
#define C0 "v_add_f32 v10, v10, v14\n\t"                               // VALU writes lo of pair
#define C0USE "v_pk_add_f32 v[12:13], v[10:11], v[10:11]\n\t"          // pk reads the pair
#define C1 "v_add_f32 v11, v11, v14\n\t"                               // VALU writes hi of pair
#define C2 "v_pk_mul_f32 v[10:11], v[10:11], v[10:11]\n\t"             // pk writes the pair
#define C2USE "v_add_f32 v12, v11, v10\n\tv_mov_b32 v13, v10\n\t"     // VALU reads both halves
#define C3 "v_div_fixup_f32 v10, v10, v14, v11\n\t"                    // the gen_ray pattern
#define C3USE "v_pk_add_f32 v[12:13], v[10:11], v[10:11]\n\t"

#define C4 "v_rcp_f32 v10, v10\n\ts_nop 0\n\t"                       // TRANS producer, 1 state
#define C4USE "v_fma_f32 v12, v10, v14, v11\n\tv_mov_b32 v13, v10\n\t"
#define C5 "v_sqrt_f32 v10, v10\n\ts_nop 0\n\t"
#define C5USE "v_add_u32 v12, -1, v10\n\tv_fma_f32 v13, -v12, v10, v11\n\t"
#define C6 "v_mul_f32 v11, v11, v14\n\t"                               // VALU writes hi, pk_mul op_sel reads it
#define C6USE "v_pk_mul_f32 v[12:13], v[10:11], v[10:11] op_sel_hi:[1,0]\n\t"

// the gen_ray sequence of the batched fp16 k_trace (v[26:27] = (u, v), v[20:21] = (rinv, -),
// v[4:5] = (M4, M5), v[14:15] = (M8, M9), v[8:9] = (M0, M1)): out = v[26:27] at the end
#define C7 "v_pk_mul_f32 v[22:23], v[26:27], v[20:21] op_sel_hi:[1,0]\n\t"                    \
           "v_pk_mov_b32 v[26:27], v[4:5], v[14:15] op_sel:[1,0]\n\t"                          \
           "v_mov_b32_e32 v5, v15\n\t"                                                          \
           "v_mul_f32_e32 v20, -2.0, v20\n\t"                                                   \
           "v_pk_mul_f32 v[24:25], v[8:9], v[22:23]\n\t"                                        \
           "v_pk_mul_f32 v[26:27], v[26:27], v[22:23] op_sel:[0,1] op_sel_hi:[1,0]\n\t"
#define C7P "v_pk_mul_f32 v[22:23], v[26:27], v[20:21] op_sel_hi:[1,0]\n\t" PAD                \
            "v_pk_mov_b32 v[26:27], v[4:5], v[14:15] op_sel:[1,0]\n\t" PAD                      \
            "v_mov_b32_e32 v5, v15\n\t" PAD                                                     \
            "v_mul_f32_e32 v20, -2.0, v20\n\t" PAD                                              \
            "v_pk_mul_f32 v[24:25], v[8:9], v[22:23]\n\t" PAD                                   \
            "v_pk_mul_f32 v[26:27], v[26:27], v[22:23] op_sel:[0,1] op_sel_hi:[1,0]\n\t"
// only the v_pk_mov_b32 op_sel read of v5 followed by the v5 overwrite
#define C8 "v_pk_mov_b32 v[26:27], v[4:5], v[14:15] op_sel:[1,0]\n\tv_mov_b32_e32 v5, v15\n\t"
#define C8P "v_pk_mov_b32 v[26:27], v[4:5], v[14:15] op_sel:[1,0]\n\t" PAD "v_mov_b32_e32 v5, v15\n\t"

#define ENTER "s_mov_b64 s[40:41], exec\n\ts_mov_b64 exec, %3\n\t"
#define ENTER5 "s_mov_b64 s[40:41], exec\n\ts_mov_b64 exec, %5\n\t"
#define LEAVE "s_mov_b64 exec, s[40:41]\n\t"
#define BODY(P, U) ENTER PAD P U PAD LEAVE
#define BODYP(P, U) ENTER PAD P PAD U PAD LEAVE
#define RUN(P, U)                                                                                 \
    if constexpr (PADDED) asm volatile(BODYP(P, U) : "+{v[12:13]}"(o), "+{v[10:11]}"(a) : "{v14}"(b), "s"(m) : "s40", "s41"); \
    else asm volatile(BODY(P, U) : "+{v[12:13]}"(o), "+{v[10:11]}"(a) : "{v14}"(b), "s"(m) : "s40", "s41");

// MASK: 0 full wave, 1 lanes 48-63, 2 lanes 32-63, 3 a pseudo-random mask per iteration
template <int CASE, bool PADDED, int MASK>
__global__ __launch_bounds__(256) void probe(unsigned *out, unsigned seed) {
    const unsigned lane = threadIdx.x & 63;
    const unsigned h = seed * 2654435761u + (blockIdx.x * 256 + threadIdx.x) * 40503u;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a = {1.0f + (float)(h & 255) / 256.0f, 2.0f + (float)((h >> 8) & 255) / 128.0f};
    const float b = 0.5f + (float)lane / 64.0f;
    unsigned sum = 0;
    unsigned long long rs = (unsigned long long)seed * 0x9E3779B97F4A7C15ull + blockIdx.x * 977u + (threadIdx.x >> 6);
    for (int it = 0; it < ITERS; ++it) {
        f2 o = {0.0f, 0.0f};
        rs = rs * 6364136223846793005ull + 1442695040888963407ull;
        unsigned long long m = MASK == 0 ? ~0ull : MASK == 1 ? 0xffff000000000000ull
                             : MASK == 2 ? 0xffffffff00000000ull : (rs ^ (rs >> 29)) | 1ull;
        m ^= (unsigned long long)(seed >> 24) << 63 >> 63;  // opaque (seed < 2^24): an SGPR, not a literal
        m = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(m >> 32)) << 32) |
            (unsigned)__builtin_amdgcn_readfirstlane((int)m);  // wave-uniform
        if constexpr (CASE == 0) { RUN(C0, C0USE) }
        else if constexpr (CASE == 1) { RUN(C1, C0USE) }
        else if constexpr (CASE == 2) { RUN(C2, C2USE) }
        else if constexpr (CASE == 3) { RUN(C3, C3USE) }
        else if constexpr (CASE == 4) { RUN(C4, C4USE) }
        else if constexpr (CASE == 5) { RUN(C5, C5USE) }
        else if constexpr (CASE == 6) { RUN(C6, C6USE) }
        else {
            // registers: v[26:27] (u, v), v[20:21], v[4:5], v[14:15], v[8:9] from lane data
            typedef float f2v __attribute__((ext_vector_type(2)));
            f2v uv = a, rr = {b, 0.0f}, m45 = {a.x * 0.5f, a.y - 1.0f}, m89 = {b * 3.0f, a.x + b}, m01 = {a.y, b};
            if constexpr (CASE == 7) {
                if constexpr (PADDED)
                    asm volatile(ENTER5 PAD C7P PAD LEAVE : "+{v[26:27]}"(uv), "+{v[20:21]}"(rr), "+{v[4:5]}"(m45)
                                 : "{v[14:15]}"(m89), "{v[8:9]}"(m01), "s"(m) : "s40", "s41", "v22", "v23", "v24", "v25");
                else
                    asm volatile(ENTER5 PAD C7 PAD LEAVE : "+{v[26:27]}"(uv), "+{v[20:21]}"(rr), "+{v[4:5]}"(m45)
                                 : "{v[14:15]}"(m89), "{v[8:9]}"(m01), "s"(m) : "s40", "s41", "v22", "v23", "v24", "v25");
            } else {
                if constexpr (PADDED)
                    asm volatile(ENTER PAD C8P PAD LEAVE : "+{v[26:27]}"(uv), "+{v[4:5]}"(m45)
                                 : "{v[14:15]}"(m89), "s"(m) : "s40", "s41");
                else
                    asm volatile(ENTER PAD C8 PAD LEAVE : "+{v[26:27]}"(uv), "+{v[4:5]}"(m45)
                                 : "{v[14:15]}"(m89), "s"(m) : "s40", "s41");
            }
            o = uv + m45 + rr;
        }
        sum = sum * 31u + __float_as_uint(o.x) + 7u * __float_as_uint(o.y);
        a.x = 1.0f + (float)((__float_as_uint(o.x) >> 7) & 255) / 256.0f + (float)lane / 128.0f;
        a.y = 2.0f + (float)((__float_as_uint(o.y) >> 9) & 255) / 128.0f;
    }
    out[blockIdx.x * 256 + threadIdx.x] = sum;
}

template <int CASE, bool PADDED, int MASK>
static std::vector<unsigned> run(int blocks, unsigned seed) {
    unsigned *d;
    if (hipMalloc(&d, (size_t)blocks * 256 * 4) != hipSuccess) exit(1);
    hipLaunchKernelGGL((probe<CASE, PADDED, MASK>), dim3(blocks), dim3(256), 0, 0, d, seed);
    std::vector<unsigned> h((size_t)blocks * 256);
    if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) exit(1);
    (void)hipFree(d);
    return h;
}

template <int CASE, int MASK>
static void check1(const char *name, int blocks) {
    size_t badw = 0, waves = 0, q[4] = {0, 0, 0, 0};
    for (unsigned seed = 1; seed <= 4; ++seed) {
        const auto r = run<CASE, true, MASK>(blocks, seed), v = run<CASE, false, MASK>(blocks, seed);
        for (size_t w = 0; w < r.size() / 64; ++w) {
            bool bad = false;
            for (int l = 0; l < 64; ++l)
                if (r[w * 64 + l] != v[w * 64 + l]) { bad = true; ++q[l >> 4]; }
            badw += bad;
            ++waves;
        }
    }
    static const char *mn[4] = {"full", "48-63", "32-63", "random"};
    printf("%-46s exec %-6s %zu of %zu waves differ; lanes per quarter %zu %zu %zu %zu\n", name, mn[MASK], badw,
           waves, q[0], q[1], q[2], q[3]);
}

template <int CASE>
static void check(const char *name, int blocks) {
    check1<CASE, 0>(name, blocks);
    check1<CASE, 1>(name, blocks);
    check1<CASE, 2>(name, blocks);
    check1<CASE, 3>(name, blocks);
}

int main(int argc, char **argv) {
    const int blocks = 256 * (argc > 1 ? atoi(argv[1]) : 4);
    check<0>("VALU writes lo -> v_pk_add reads pair", blocks);
    check<1>("VALU writes hi -> v_pk_add reads pair", blocks);
    check<2>("v_pk_mul writes pair -> VALU reads hi/lo", blocks);
    check<3>("v_div_fixup writes lo -> v_pk_add reads pair", blocks);
    check<4>("v_rcp (1 state) -> v_fma", blocks);
    check<5>("v_sqrt (1 state) -> v_add_u32/v_fma", blocks);
    check<6>("VALU writes hi -> v_pk_mul op_sel_hi reads", blocks);
    check<7>("gen_ray sequence (pk_mul, pk_mov op_sel, WAR v5)", blocks);
    check<8>("v_pk_mov_b32 op_sel read, then v5 overwrite", blocks);
    return 0;
}
