// lowp_lane_test.hip -- does the bf16 32-point-tile MLP (nr_mlp16.h mlp16_lowp) give a
// point the same value whatever the other lanes hold and whichever tiles are marked live?
// Each configuration evaluates 64 points with some lanes "dead" (garbage / NaN / huge
// coordinates, tile bits cleared) and compares the live lanes with a full evaluation.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off lowp_lane_test.hip
//        ../cudaneuralrender_amd/csrc/nr_pack.cpp -o bin/lowp_lane_test
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../cudaneuralrender_amd/csrc/nr_mlp16.h"

using namespace nr;

__global__ void k(MlpArgs M, const float *X, const unsigned long long *live, int mode, float *Y) {
    Smem16 S = stage16(M, NR_PRECISION_BF16);
    const int lane = lane_id();
    const int cfg = blockIdx.x;
    const unsigned long long lm = live[cfg];
    const bool lv = (lm >> lane) & 1ull;
    float x = X[3 * lane], y = X[3 * lane + 1], z = X[3 * lane + 2];
    if (!lv) {  // dead lane garbage
        if (mode == 1) { x = __builtin_nanf(""); y = 1e30f; z = -1e30f; }
        else if (mode == 2) { x = 3.0e38f; y = -7.0f; z = __builtin_inff(); }
        else { x = 0.5f * (float)lane; y = -0.25f; z = 9.0f; }
    }
    uint32_t tmask = tiles_of(lm);
    const float v = mlp16(M, S.s32, S.slp, S.sfl, NR_PRECISION_BF16, 0.0f, x, y, z, tmask);
    if (threadIdx.x < 64) Y[cfg * 64 + lane] = v;
}

int main() {
    std::mt19937 rng(3);
    std::uniform_real_distribution<float> U(-0.5f, 0.5f), UX(-1.0f, 1.0f);
    std::vector<int> dims = {3, 32, 32, 32, 32, 32, 32, 32, 32, 1};
    std::vector<std::vector<float>> K(9), B(9);
    for (int l = 0; l < 9; ++l) {
        K[l].resize(dims[l] * dims[l + 1]);
        B[l].resize(dims[l + 1]);
        for (auto &v : K[l]) v = U(rng);
        for (auto &v : B[l]) v = U(rng) * 0.2f;
    }
    std::vector<float> pk;
    std::vector<uint16_t> lp;
    std::vector<float> lpf;
    if (!pack_fp32_16(dims, K, B, pk) || !pack_lowp_32(dims, K, B, NR_PRECISION_BF16, lp, lpf)) return 1;
    auto pad16 = [](size_t b) { return (b + 15) / 16 * 16; };
    std::vector<unsigned long long> lives = {~0ull, 0xffff0000ull, 0xffff0000ffff0000ull, 0xffff000000000000ull,
                                             0x0000ffff00000000ull, 0x00000000ffffffffull, 0xffffffff00000000ull,
                                             0x5555555555555555ull, 0x0000000000ff0000ull, 0xf0f0f0f0f0f0f0f0ull};
    const int ncfg = (int)lives.size();
    std::vector<float> X(64 * 3);
    for (auto &v : X) v = UX(rng);
    float *dpk, *dlpf, *dX, *dY; uint16_t *dlp; unsigned long long *dlive;
    if (hipMalloc(&dpk, pad16(pk.size() * 4)) || hipMalloc(&dlp, pad16(lp.size() * 2)) ||
        hipMalloc(&dlpf, pad16(lpf.size() * 4)) || hipMalloc(&dX, X.size() * 4) || hipMalloc(&dY, ncfg * 64 * 4) ||
        hipMalloc(&dlive, ncfg * 8)) return 1;
    if (hipMemcpy(dpk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dlp, lp.data(), lp.size() * 2, hipMemcpyHostToDevice) ||
        hipMemcpy(dlpf, lpf.data(), lpf.size() * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(dlive, lives.data(), ncfg * 8, hipMemcpyHostToDevice)) return 1;
    MlpArgs M{};
    M.pk = dpk; M.lp = dlp; M.lpf = dlpf;
    M.pk_bytes = (int)pad16(pk.size() * 4); M.lp_bytes = (int)pad16(lp.size() * 2); M.lpf_bytes = (int)pad16(lpf.size() * 4);
    M.in0 = 3; M.nh = 7;
    const int sm = M.pk_bytes + M.lp_bytes + M.lpf_bytes;
    std::vector<float> Y(ncfg * 64);
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL(k, dim3(ncfg), dim3(64), sm, 0, M, dX, dlive, mode, dY);
        if (hipDeviceSynchronize()) return 1;
        if (hipMemcpy(Y.data(), dY, Y.size() * 4, hipMemcpyDeviceToHost)) return 1;
        for (int c = 1; c < ncfg; ++c) {
            int bad = 0, first = -1;
            for (int l = 0; l < 64; ++l)
                if (((lives[c] >> l) & 1ull) && memcmp(&Y[c * 64 + l], &Y[l], 4)) { ++bad; if (first < 0) first = l; }
            printf("mode %d live %016llx: %d live lanes differ from the full evaluation (first lane %d)\n", mode,
                   lives[c], bad, first);
        }
    }
    return 0;
}
