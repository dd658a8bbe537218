// scene_bench.hip -- cost of the scene SDF (manySphere, nr_device.h) per wave call, alone on
// the chip: one wave per SIMD, points sampled along bench-like rays (most spheres far);
// prints shader cycles per call from s_memtime around 64 chained calls.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scene_bench.hip -o bin/scene_bench
#include <cstdio>
#include <vector>

#include "../cudaneuralrender_amd/csrc/nr_device.h"

using namespace nr;

__global__ void k(const float4 *pts, float *out, unsigned long long *cyc, double zoff, int reps, int mode) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float4 q = pts[i];
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        float v;
        if (mode == 0) v = many_sphere(mk3(q.x, q.y, q.z), q.w, zoff);
        else if (mode == 1) v = nr_tanh(q.w);
        else v = many_sphere(mk3(q.x, q.y, q.z), -0.1f + 1e-4f * q.w, zoff);  // T ~ 0.011: all far
        acc += v;
        q.w = v * 0.999f + 1e-3f;  // chained: the next call depends on this one
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[i] = acc;
    if ((threadIdx.x & 63) == 0) cyc[i >> 6] = t1 - t0;
}

int main() {
    const int waves = 1024, n = waves * 64, reps = 64;
    std::vector<float4> h(n);
    unsigned s = 1;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0f / 16777216.0f); };
    for (auto &p : h) {  // points on rays from the eye (0,0,2) through the unit box, t in [0.8, 2.8]
        const float u = rnd() * 2 - 1, v = rnd() * 2 - 1, t = 0.8f + 2.0f * rnd();
        const float dx = u, dy = v, dz = -2.0f, l = sqrtf(dx * dx + dy * dy + dz * dz);
        p = make_float4(dx / l * t, dy / l * t, 2.0f + dz / l * t, 0.05f + 0.3f * rnd());
    }
    {   // host: fraction of points with at least one sphere inside s + 0.1111, mean count
        long anyn = 0, cnt = 0;
        for (auto &p : h) {
            int c = 0;
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    const float cx = p.x - (-0.5f + 0.4f * a), cy = p.y - (0.2f - 0.4f * b), cz = p.z - 0.7f;
                    c += sqrtf(cx * cx + cy * cy + cz * cz) <= p.w + 0.1111f;
                }
            anyn += c > 0; cnt += c;
        }
        printf("points with a near sphere: %.3f, near spheres per point %.3f\n", (double)anyn / n, (double)cnt / n);
    }
    float4 *dp; float *dout; unsigned long long *dc;
    if (hipMalloc(&dp, n * 16) || hipMalloc(&dout, n * 4) || hipMalloc(&dc, waves * 8)) return 1;
    if (hipMemcpy(dp, h.data(), n * 16, hipMemcpyHostToDevice)) return 1;
    for (int mode = 0; mode < 3; ++mode) {
        for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k, dim3(waves / 4), dim3(256), 0, 0, dp, dout, dc, -0.7, reps, mode);
        if (hipDeviceSynchronize()) return 1;
        std::vector<unsigned long long> c(waves);
        if (hipMemcpy(c.data(), dc, waves * 8, hipMemcpyDeviceToHost)) return 1;
        std::vector<float> o(n);
        if (hipMemcpy(o.data(), dout, n * 4, hipMemcpyDeviceToHost)) return 1;
        double sum = 0;
        for (auto v : c) sum += (double)v;
        printf("%s: %.0f cycles per wave call (one wave per SIMD, %d chained calls)\n",
               mode == 0 ? "manySphere" : (mode == 1 ? "nr_tanh" : "manySphere, all spheres far"), sum / waves / reps, reps);
    }
    return 0;
}
