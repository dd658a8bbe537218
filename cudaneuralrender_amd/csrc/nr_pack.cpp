// nr_pack.cpp -- host-side weight packing for the fused MFMA MLP, and the camera.
//
// Input: Keras Dense kernels (in x out, row-major) as HighFive hands them to the
// DenseLayer constructor (reference src/layers/denseLayer.cu:180-227, which
// transposes them to out-major W[out][in]).  Output: register-layout-ready packs
// for the 16-point-tile MLP (nr_mlp16.h; layout documented in nr_internal.h and
// DESIGN.md §4).
#include "nr_internal.h"

#include <cmath>
#include <cstring>

namespace nr {

bool fused_shape_ok(const std::vector<int> &dims) {
    int nl = (int)dims.size() - 1;
    if (nl < 2 || nl - 2 > MAX_HIDDEN) return false;
    if (dims[0] != 3 && dims[0] != 4) return false;
    for (int l = 1; l < nl; ++l) if (dims[l] != 32) return false;
    return dims[nl] == 1;
}

namespace {
uint16_t f2bf16(float x) {
    uint32_t u; memcpy(&u, &x, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

uint16_t f2fp16(float x) {
    uint32_t u; memcpy(&u, &x, 4);
    uint32_t sign = (u >> 16) & 0x8000u;
    float ax = std::fabs(x);
    if (std::isnan(x)) return (uint16_t)(sign | 0x7e00u);
    if (ax >= 65520.0f) return (uint16_t)(sign | 0x7c00u);
    if (ax < 6.103515625e-05f) {                       // subnormal half
        float q = std::nearbyint(ax / 5.9604644775390625e-08f);   // RNE (default rounding mode)
        return (uint16_t)(sign | (uint32_t)q);
    }
    int e; float m = std::frexp(ax, &e);                // ax = m 2^e, m in [0.5,1)
    float mant = std::nearbyint((m * 2.0f - 1.0f) * 1024.0f);
    int exp = e - 1 + 15;
    if (mant >= 1024.0f) { mant = 0; exp += 1; }
    if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
    return (uint16_t)(sign | (uint32_t)exp << 10 | (uint32_t)mant);
}
}  // namespace

// ---- 16-point tiles (nr_mlp16.h).  Lane (j, g): point j, unit group g; register k.
namespace {
// fp32: unit held by (g, k): next layer MFMA -> 4k + g (ascending f32 chain over the
// 8 k-steps x 4 lane groups); next layer final VALU -> 8g + k (chain hops 3 times).
inline int unit16(int g, int k, bool final_consumer) { return final_consumer ? 8 * g + k : 4 * k + g; }
// low precision: the MFMA C layout as is: register k = 4mt + r of group g = row 16mt + 4g + r
inline int row16(int g, int k) { return 16 * (k >> 2) + 4 * g + (k & 3); }
}  // namespace

bool pack_fp32_16(const std::vector<int> &dims, const std::vector<std::vector<float>> &K,
                  const std::vector<std::vector<float>> &B, std::vector<float> &pack) {
    if (!fused_shape_ok(dims)) return false;
    int nl = (int)dims.size() - 1, nh = nl - 2, in0 = dims[0];
    pack.assign(pk_floats(nh), 0.0f);
    // layer 0 as one 16x16x4 MFMA per row tile: A[row 16mt + i][k = input kk]
    for (int mt = 0; mt < 2; ++mt)
        for (int lane = 0; lane < 64; ++lane) {
            int i = lane & 15, kk = lane >> 4, gp = i >> 2, rp = i & 3;
            int uout = (nh == 0) ? 8 * gp + 4 * mt + rp : 16 * mt + 4 * rp + gp;
            pack[PK_L0W + mt * 64 + lane] = (kk < in0) ? K[0][(size_t)kk * 32 + uout] : 0.0f;
        }
    for (int g = 0; g < 4; ++g)
        for (int k = 0; k < 8; ++k) pack[PK_L0B + g * 8 + k] = B[0][unit16(g, k, nh == 0)];
    for (int j = 0; j < nh; ++j) {
        const std::vector<float> &Kj = K[j + 1];
        bool fin = (j == nh - 1);
        int base = PK_HID + j * PK_HID_STRIDE;
        for (int st = 0; st < 8; ++st)
            for (int mt = 0; mt < 2; ++mt) {
                int m = 2 * st + mt;
                for (int lane = 0; lane < 64; ++lane) {
                    int i = lane & 15, kk = lane >> 4;
                    int gp = i >> 2, rp = i & 3;
                    int uout = fin ? 8 * gp + 4 * mt + rp : 16 * mt + 4 * rp + gp;
                    int uin = 4 * st + kk;
                    pack[base + ((m >> 2) * 64 + lane) * 4 + (m & 3)] = Kj[(size_t)uin * 32 + uout];
                }
            }
        for (int g = 0; g < 4; ++g)
            for (int k = 0; k < 8; ++k) pack[base + 1024 + g * 8 + k] = B[j + 1][unit16(g, k, fin)];
    }
    int fo = pk_final(nh);
    for (int g = 0; g < 4; ++g)
        for (int k = 0; k < 8; ++k) pack[fo + g * 8 + k] = K[nl - 1][8 * g + k];
    pack[fo + 32] = B[nl - 1][0];
    return true;
}

bool pack_lowp_16(const std::vector<int> &dims, const std::vector<std::vector<float>> &K,
                  const std::vector<std::vector<float>> &B, int precision, std::vector<uint16_t> &a_ops,
                  std::vector<float> &fl) {
    if (!fused_shape_ok(dims)) return false;
    int nl = (int)dims.size() - 1, nh = nl - 2, in0 = dims[0];
    auto cvt = [&](float v) { return precision == NR_PRECISION_BF16 ? f2bf16(v) : f2fp16(v); };
    a_ops.assign((size_t)nh * LP_A_ELEMS, 0);
    fl.assign(160 + 32 * nh + 36, 0.0f);
    // layer 0: f32 16x16x4 MFMA A operand, rows in natural unit order
    for (int mt = 0; mt < 2; ++mt)
        for (int lane = 0; lane < 64; ++lane) {
            int i = lane & 15, kk = lane >> 4;
            fl[mt * 64 + lane] = (kk < in0) ? K[0][(size_t)kk * 32 + 16 * mt + i] : 0.0f;
        }
    for (int g = 0; g < 4; ++g)
        for (int k = 0; k < 8; ++k) fl[128 + g * 8 + k] = B[0][row16(g, k)];
    for (int j = 0; j < nh; ++j) {
        const std::vector<float> &Kj = K[j + 1];
        for (int mt = 0; mt < 2; ++mt)
            for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                    int i = lane & 15, gg = lane >> 4;
                    int uin = row16(gg, e);       // B operand element e of group gg = that unit
                    int uout = 16 * mt + i;
                    a_ops[(size_t)j * LP_A_ELEMS + (mt * 64 + lane) * 8 + e] = cvt(Kj[(size_t)uin * 32 + uout]);
                }
        for (int g = 0; g < 4; ++g)
            for (int k = 0; k < 8; ++k) fl[160 + 32 * j + g * 8 + k] = B[j + 1][row16(g, k)];
    }
    int fo = 160 + 32 * nh;
    for (int g = 0; g < 4; ++g)
        for (int k = 0; k < 8; ++k) fl[fo + g * 8 + k] = K[nl - 1][row16(g, k)];
    fl[fo + 32] = B[nl - 1][0];
    return true;
}

// updateViewMatrices (reference src/main.cpp:207-222), evaluated in double and
// rounded to float once (the reference uses Eigen float arithmetic).
void camera_matrices(float rx, float ry, float zoom, float tx, float ty, float inv_view[12], float normal[16]) {
    const double pi = 3.14159265358979323846;
    double ax = -(double)rx * pi / 180.0, ay = -(double)ry * pi / 180.0;
    double cx = std::cos(ax), sx = std::sin(ax), cy = std::cos(ay), sy = std::sin(ay);
    double Rx[3][3] = {{1, 0, 0}, {0, cx, -sx}, {0, sx, cx}};
    double Ry[3][3] = {{cy, 0, sy}, {0, 1, 0}, {-sy, 0, cy}};
    double R[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            R[i][j] = 0;
            for (int k = 0; k < 3; ++k) R[i][j] += Rx[i][k] * Ry[k][j];
        }
    // viewTranslation = (tx, ty, -zoom); modelView.translate(-viewTranslation)
    double t[3] = {-(double)tx, -(double)ty, (double)zoom};
    double T[3];
    for (int i = 0; i < 3; ++i) T[i] = R[i][0] * t[0] + R[i][1] * t[1] + R[i][2] * t[2];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) inv_view[4 * i + j] = (float)R[i][j];
        inv_view[4 * i + 3] = (float)T[i];
    }
    // inverse of [R | T; 0 1] = [R^T | -R^T T; 0 1]
    for (int i = 0; i < 3; ++i) {
        double acc = 0;
        for (int j = 0; j < 3; ++j) {
            normal[4 * i + j] = (float)R[j][i];
            acc += R[j][i] * T[j];
        }
        normal[4 * i + 3] = (float)(-acc);
    }
    normal[12] = normal[13] = normal[14] = 0.0f;
    normal[15] = 1.0f;
}

}  // namespace nr
