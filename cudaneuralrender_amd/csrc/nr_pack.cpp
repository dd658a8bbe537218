// nr_pack.cpp -- host-side weight packing for the fused MFMA MLP, and the camera.
//
// Input: Keras Dense kernels (in x out, row-major) as HighFive hands them to the
// DenseLayer constructor (reference src/layers/denseLayer.cu:180-227, which
// transposes them to out-major W[out][in]).  Output: register-layout-ready packs
// for the 16-point-tile MLP (nr_mlp16.h; layout documented in nr_internal.h and
// DESIGN.md §4).
#include "nr_internal.h"

#include <algorithm>
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

float bf16f(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f; memcpy(&f, &u, 4);
    return f;
}

float fp16f(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    const float sign = (h & 0x8000u) ? -1.0f : 1.0f;
    if (e == 31) return m ? NAN : sign * INFINITY;
    if (e == 0) return sign * std::ldexp((float)m, -24);
    return sign * std::ldexp((float)(1024 + m), e - 25);
}
}  // namespace

// Power-of-two scales for the clamped-ReLU packs: e[l] such that every ReLU layer l's
// activation, for network inputs within +-bound, is at most 2^e[l] / 2^margin.  Interval
// arithmetic in double over the exact f32 weights; the margin covers the rounding of the
// evaluation (bf16: 2 -- weights and activations rounded to bf16, relative 2^-9 each per
// layer, ~3% over 8 layers; fp32: 1 -- f32 chains, ~2^-19 relative).  The rounding error of a
// unit is relative to the sum of its terms' magnitudes S = |b| + sum |w| max(|lo|, |hi|), not to
// its value, so a unit whose bias cancels large products could round past the interval bound:
// the bound used is top + eps S (bf16 eps 2^-6, fp32 2^-19).  Returns false -- the
// unscaled pack, ReLU by max -- when a scale or a scaled weight would leave the range where
// power-of-two scaling is exact, or a nonzero weight or bias is below 2^-60 in magnitude (with
// such values the scaled chains could round differently from the unscaled ones near f32's
// subnormal range).
static bool clamp_scales(const std::vector<int> &dims, const std::vector<std::vector<float>> &K,
                         const std::vector<std::vector<float>> &B, std::vector<int> &e, double bound, int margin,
                         double eps) {
    const int nl = (int)dims.size() - 1;
    std::vector<double> lo(dims[0], -bound), hi(dims[0], bound);
    e.assign(nl - 1, 0);
    for (int l = 0; l < nl; ++l) {
        for (float w : K[l])
            if (w != 0.0f && std::fabs(w) < 0x1p-60f) return false;
        for (float b : B[l])
            if (b != 0.0f && std::fabs(b) < 0x1p-60f) return false;
    }
    for (int l = 0; l < nl - 1; ++l) {
        const int in = dims[l], out = dims[l + 1];
        std::vector<double> nlo(out), nhi(out);
        double top = 0.0;
        for (int u = 0; u < out; ++u) {
            double a = B[l][u], b = B[l][u], S = std::fabs((double)B[l][u]);
            for (int i = 0; i < in; ++i) {
                const double w = K[l][(size_t)i * out + u];
                a += std::min(w * lo[i], w * hi[i]);
                b += std::max(w * lo[i], w * hi[i]);
                S += std::fabs(w) * std::max(std::fabs(lo[i]), std::fabs(hi[i]));
            }
            nlo[u] = std::max(a, 0.0);  // ReLU
            nhi[u] = std::max(b, 0.0);
            top = std::max(top, nhi[u] + eps * S);
        }
        if (!std::isfinite(top)) return false;
        e[l] = top > 0.0 ? (int)std::ceil(std::log2(top)) + margin : 0;
        if (e[l] < -60 || e[l] > 100) return false;
        lo = nlo;
        hi = nhi;
    }
    // every scaled nonzero weight and bias must stay a normal bf16 / f32 well inside range
    for (int l = 0; l < nl; ++l) {
        const int sw = (l > 0 ? e[l - 1] : 0) - (l < nl - 1 ? e[l] : 0);
        const int sb = l < nl - 1 ? -e[l] : 0;
        for (float w : K[l])
            if (w != 0.0f && (std::fabs(std::ldexp((double)w, sw)) < 0x1p-110 || std::fabs(std::ldexp((double)w, sw)) > 0x1p110))
                return false;
        for (float b : B[l])
            if (b != 0.0f && (std::fabs(std::ldexp((double)b, sb)) < 0x1p-110 || std::fabs(std::ldexp((double)b, sb)) > 0x1p110))
                return false;
    }
    return true;
}

// Hard bounds on every ReLU layer's largest activation for xyz inputs within +-xyz_b (and a 4th
// input within +-f_b): the maximum of the interval bounds (double, over the exact f32 weights)
// over a grid of sub-boxes of the input box -- 16 per xyz axis; 8 per axis x 16 frame slabs for
// a 4th input.  Still a hard bound, 2-4 binades tighter than one interval pass over the whole box
// on the bundled networks (interval arithmetic ignores the correlation of a unit's inputs, and a
// small box leaves less of it).  Returns false on a non-finite bound.
static bool box_tops(const std::vector<int> &dims, const std::vector<std::vector<float>> &K,
                     const std::vector<std::vector<float>> &B, double xyz_b, double f_b, std::vector<double> &top) {
    const int nl = (int)dims.size() - 1, in0 = dims[0];
    const int mx = in0 == 4 ? 8 : 16, mf = in0 == 4 ? 16 : 1;
    bool ok = true;
    std::vector<double> lo, hi, nlo, nhi;
    top.assign(nl - 1, 0.0);
    for (int box = 0; box < mx * mx * mx * mf && ok; ++box) {
        lo.assign(in0, 0.0);
        hi.assign(in0, 0.0);
        for (int i = 0; i < in0; ++i) {
            const int m = i < 3 ? mx : mf, k = i < 3 ? (box / (i == 0 ? 1 : i == 1 ? mx : mx * mx)) % mx : box / (mx * mx * mx);
            const double b = i < 3 ? xyz_b : f_b;
            lo[i] = -b + 2.0 * b * k / m;
            hi[i] = k + 1 == m ? b : -b + 2.0 * b * (k + 1) / m;
        }
        for (int l = 0; l < nl - 1; ++l) {
            const int in = dims[l], out = dims[l + 1];
            nlo.assign(out, 0.0);
            nhi.assign(out, 0.0);
            for (int u = 0; u < out; ++u) {
                double a = B[l][u], b = B[l][u];
                for (int i = 0; i < in; ++i) {
                    const double w = K[l][(size_t)i * out + u];
                    a += std::min(w * lo[i], w * hi[i]);
                    b += std::max(w * lo[i], w * hi[i]);
                }
                if (!std::isfinite(a) || !std::isfinite(b)) ok = false;
                nlo[u] = std::max(a, 0.0);
                nhi[u] = std::max(b, 0.0);
                top[l] = std::max(top[l], nhi[u]);
            }
            lo.swap(nlo);
            hi.swap(nhi);
        }
    }
    return ok;
}

// Layer l's weights times 2^(e[l-1] - e[l]) and its bias times 2^-e[l] (e[-1] = 0, e[last]
// = 0): activations come out scaled by 2^-e[l] and the last layer's output unscaled.
static void apply_scales(const std::vector<int> &e, std::vector<std::vector<float>> &K,
                         std::vector<std::vector<float>> &B) {
    const int nl = (int)K.size();
    for (int l = 0; l < nl; ++l) {
        const int sw = (l > 0 ? e[l - 1] : 0) - (l < nl - 1 ? e[l] : 0);
        const int sb = l < nl - 1 ? -e[l] : 0;
        for (float &w : K[l]) w = std::ldexp(w, sw);
        for (float &b : B[l]) b = std::ldexp(b, sb);
    }
}

// ---- 16-point tiles (nr_mlp16.h).  Lane (j, g): point j, unit group g; register k.
namespace {
// fp32: unit held by (g, k): next layer MFMA -> 4k + g (ascending f32 chain over the
// 8 k-steps x 4 lane groups); next layer final VALU -> 8g + k (chain hops 3 times).
inline int unit16(int g, int k, bool final_consumer) { return final_consumer ? 8 * g + k : 4 * k + g; }
}  // namespace

// The fp32 pack is scaled like the bf16 clamped pack (clamp_scales, F32_INPUT_BOUND): each
// f32 product, fmaf chain and bias add then computes its unscaled value times 2^-e exactly
// (rounding is scale-invariant while values stay normal), so the network's output is the
// unscaled network's bit for bit, and ReLU activations stay <= 1/2 for inputs within the
// bound -- v_add_f32 with the clamp bit is then the bias add and the ReLU in one
// instruction (nr_mlp16.h).  A wave with an input beyond the bound runs the add + max form on
// the same pack: larger inputs make larger scaled values, still exact.  Precondition of the
// "bit for bit": no fmaf result of the unscaled evaluation lies in (0, 2^(e - 126)) in magnitude
// (e <= ~27 for the bundled networks: below ~10^-30), where the scaled evaluation would round a
// subnormal.  Sums that cancel are exact (Sterbenz), so such a result needs tiny operands:
// clamp_scales refuses networks with nonzero weights or biases below 2^-60, and inputs that
// small (tests/test_gpu_f32_clamp.py drives 1e-25) only reach it through a layer-0 unit whose
// bias is exactly 0 and whose products are all below ~2^-100.
bool pack_fp32_16(const std::vector<int> &dims, const std::vector<std::vector<float>> &Kin,
                  const std::vector<std::vector<float>> &Bin, std::vector<float> &pack, int *clamp) {
    if (!fused_shape_ok(dims)) return false;
    int nl = (int)dims.size() - 1, nh = nl - 2, in0 = dims[0];
    std::vector<int> e;
    const bool cl = clamp_scales(dims, Kin, Bin, e, (double)F32_INPUT_BOUND, 1, 0x1p-19);
    if (clamp) *clamp = cl ? 1 : 0;
    std::vector<std::vector<float>> K(Kin), B(Bin);
    if (cl) {
        apply_scales(e, K, B);
        // layer 0 keeps its f32 weights (the products of the raw inputs are the reference's);
        // its chain is scaled on the way out: fma(c, 2^-e0, b 2^-e0) = (c + b) 2^-e0
        K[0] = Kin[0];
    }
    pack.assign(pk_floats(nh), 0.0f);
    pack[pk_final(nh) + 33] = cl ? std::ldexp(1.0f, -e[0]) : 1.0f;
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

bool pack_lowp_32(const std::vector<int> &dims, const std::vector<std::vector<float>> &Kin,
                  const std::vector<std::vector<float>> &Bin, int precision, std::vector<uint16_t> &a_ops,
                  std::vector<float> &fl, int *clamp) {
    if (!fused_shape_ok(dims)) return false;
    const int nl = (int)dims.size() - 1, nh = nl - 2, in0 = dims[0];
    const bool bf = precision == NR_PRECISION_BF16;
    // bf16: layer l's weights scaled by 2^(e[l-1] - e[l]) and its bias by 2^-e[l] (e[-1] = 0,
    // e[last] = 0), so activations come out scaled by 2^-e[l] and the last layer's output is
    // unscaled: power-of-two scaling is exact in bf16 and f32, so the network computes the same
    // values as unscaled, and activations stay below 1 for the clamped ReLU (nr_mlp16.h)
    // (fp16 stays unscaled: its narrow exponent range turns the scaled activations -- held below
    // 1 by a hard interval bound that sits 7-10 binades above the actual values -- into
    // subnormals; measured round 3: +10 % MLP rate, C5 crops' coverage IoU vs the fp32 oracle
    // 0.98 -> 0.74-0.86.  DESIGN.md section 2.)
    std::vector<int> e;
    const bool cl = bf && clamp_scales(dims, Kin, Bin, e, (double)LP_INPUT_BOUND, 2, 0x1p-6);
    if (clamp) *clamp = cl ? 1 : 0;
    std::vector<std::vector<float>> K(Kin), B(Bin);
    if (cl) apply_scales(e, K, B);
    auto cvt = [&](float v) { return bf ? f2bf16(v) : f2fp16(v); };
    auto back = [&](uint16_t h) { return bf ? bf16f(h) : fp16f(h); };
    auto lo = [&](float v) { return cvt(v - back(cvt(v))); };  // the residual's 16-bit value
    auto crow = [](int h, int i) { return (i & 3) + 8 * (i >> 2) + 4 * h; };      // C/D row of register i
    auto kin = [](int s, int h, int e) { return 16 * s + 8 * (e >> 2) + 4 * h + (e & 3); };
    a_ops.assign((size_t)lp32_elems(nh), 0);
    fl.assign((size_t)lp32_floats(nh), 0.0f);
    // layer 0, K = 16: h = 0 slots {wh x3 . xh, wh x3 . xl, wh3 . frh, wh3 . frl},
    //                  h = 1 slots {wl x3 . xh, wl3 . frh, 0 x4}
    for (int lane = 0; lane < 64; ++lane) {
        const int m = lane & 31, h = lane >> 5;
        uint16_t *el = &a_ops[(size_t)lane * 8];
        for (int c = 0; c < 3; ++c) {
            const float w = K[0][(size_t)c * 32 + m];
            if (h == 0) el[c] = el[3 + c] = cvt(w);
            else el[c] = lo(w);
        }
        if (in0 == 4) {
            const float w = K[0][(size_t)3 * 32 + m];
            if (h == 0) el[6] = el[7] = cvt(w);
            else el[3] = lo(w);
        }
    }
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 16; ++i) fl[h * 16 + i] = B[0][crow(h, i)];
    for (int j = 0; j < nh; ++j) {
        const std::vector<float> &Kj = K[j + 1];
        for (int s = 0; s < 2; ++s)
            for (int lane = 0; lane < 64; ++lane)
                for (int k = 0; k < 8; ++k) {
                    const int m = lane & 31, h = lane >> 5;
                    a_ops[(size_t)LP32_HID + (size_t)j * LP32_HSTRIDE + (size_t)s * 512 + lane * 8 + k] =
                        cvt(Kj[(size_t)kin(s, h, k) * 32 + m]);
                }
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < 16; ++i) fl[32 + 32 * j + h * 16 + i] = B[j + 1][crow(h, i)];
    }
    for (int s = 0; s < 2; ++s)
        for (int h = 0; h < 2; ++h)
            for (int k = 0; k < 8; ++k)
                a_ops[(size_t)lp32_final(nh) + (s * 2 + h) * 8 + k] = cvt(K[nl - 1][kin(s, h, k)]);
    fl[32 + 32 * nh] = B[nl - 1][0];
    return true;
}

// The 16x16x32 layout (nr_internal.h pack_lowp_s16).  The 32x32x16 MLP sums every hidden unit's 32
// inputs as four 8-product blocks in the order B0 = {0-3, 8-11}, B1 = {4-7, 12-15}, B2 = {16-19,
// 24-27}, B3 = {20-23, 28-31} (unit = kin(s, h, e): k-step s, lane half h: block 2s + h); a
// v_mfma_f32_16x16x32 sums its K = 32 as lane groups g = 0..3 in that order, so group g's k-slots
// must hold block Bg: V(g, e) = base[g] + 8 (e >> 2) + (e & 3), base = {0, 4, 16, 20}.  A hidden
// layer's output rows (two MFMAs, half hf: rows 0-15 / 16-31; lane (j, g) receives rows 4g..4g+3
// of each) hold U(hf, r) = base[r >> 2] + 8 hf + (r & 3), so that they are the next layer's B
// operand as they lie.  The input layer stays a 32x32x16 MFMA; one v_permlane16_swap per word
// pair deals its (k-step s, lane half h) words to group s + 2h of a 16-point tile, so its row
// 16s + 8a + 4h + b computes unit base[s + 2h] + 8a + b.  The last hidden layer's rows take
// base {0, 16, 4, 20}, so that the swap back yields the 32x32x16 form's final-layer operands.
void pack_lowp_s16(const std::vector<uint16_t> &a32, const std::vector<float> &f32, int nh,
                   std::vector<uint16_t> &a16, std::vector<float> &f16) {
    static const int base[4] = {0, 4, 16, 20}, base_last[4] = {0, 16, 4, 20};
    auto ic = [](int u) { return 16 * ((u >> 2) & 1) + (u & 3) + 4 * (u >> 3); };        // crow^-1: fl index
    auto kslot = [](int k) { return 512 * (k >> 4) + 256 * ((k >> 2) & 1) + (k & 3) + 4 * ((k >> 3) & 1); };
    auto p0 = [&](int r) { return base[(r >> 4) + 2 * ((r >> 2) & 1)] + 8 * ((r >> 3) & 1) + (r & 3); };
    a16 = a32;
    f16 = f32;
    for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < 8; ++e) a16[(size_t)lane * 8 + e] = a32[(size_t)(p0(lane & 31) + 32 * (lane >> 5)) * 8 + e];
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 16; ++i) f16[(size_t)h * 16 + i] = f32[ic(p0((i & 3) + 8 * (i >> 2) + 4 * h))];
    for (int j = 0; j < nh; ++j) {
        const int *bj = j == nh - 1 ? base_last : base;
        const size_t A = (size_t)LP32_HID + (size_t)j * LP32_HSTRIDE;
        for (int hf = 0; hf < 2; ++hf)
            for (int lane = 0; lane < 64; ++lane) {
                const int r = lane & 15, g = lane >> 4;
                const int m = bj[r >> 2] + 8 * hf + (r & 3);                    // output unit
                for (int e = 0; e < 8; ++e) {
                    const int k = base[g] + 8 * (e >> 2) + (e & 3);             // input unit
                    // 32x32x16 element of (output m, input k): k-step s = k >> 4, lane m + 32 h
                    const int ks = kslot(k);
                    a16[A + (size_t)hf * 512 + (size_t)lane * 8 + e] =
                        a32[A + (size_t)(ks / 512) * 512 + (size_t)(m + 32 * ((ks / 256) & 1)) * 8 + (ks & 7)];
                }
            }
        for (int g = 0; g < 4; ++g)
            for (int hf = 0; hf < 2; ++hf)
                for (int i = 0; i < 4; ++i)
                    f16[32 + 32 * (size_t)j + g * 8 + hf * 4 + i] = f32[32 + 32 * (size_t)j + ic(bj[g] + 8 * hf + i)];
    }
}

// fp32x3 (nr_internal.h X3_*, nr_mlp16.h mlp32_x3_nt).  Interval bounds in double over the
// exact f32 weights for xyz within +-X3_INPUT_BOUND (and a 4th input within +-X3_FRAME_BOUND)
// give each ReLU layer's top activation; layer l's activations are scaled by 2^-e[l] with
// e[l] = ceil(log2(top)) - 10, so a scaled activation stays below 2^10 (x2 margin for the
// evaluation's rounding against the 2^11 the residual clamp needs).  Weights of layer l are
// scaled by 2^(e[l-1] - e[l]) and split into fp16 hi + residual; layer 0's xyz weights by
// 2^(-e[0] - X3_XYZ_SHIFT) (the kernel scales the inputs by 2^X3_XYZ_SHIFT), its 4th-input
// weights by 2^-e[0]; the final layer keeps f32 weights times 2^e[last].  Every scaling is by a
// power of two, so the split approximates the unscaled network; the fp16 range limits it
// (hi below 2^15), otherwise ok = 0 and the kernels run the fp32 MLP.
bool pack_x3_32(const std::vector<int> &dims, const std::vector<std::vector<float>> &K,
                const std::vector<std::vector<float>> &B, std::vector<uint16_t> &a_ops, std::vector<float> &fl,
                int *ok_out) {
    if (!fused_shape_ok(dims)) return false;
    const int nl = (int)dims.size() - 1, nh = nl - 2, in0 = dims[0];
    a_ops.assign((size_t)x3_elems(nh), 0);
    fl.assign((size_t)x3_floats(nh), 0.0f);
    bool ok = true;
    std::vector<int> e(nl - 1, 0);
    {
        // the scales from the sub-box interval bounds (box_tops): activations sit higher in the
        // window below 2^10, so fewer residuals al = a - ah fall into fp16's subnormal range,
        // which would cost them relative precision (emulated: mean error vs fp64 from 2.4-3.9x to
        // 1.8-2.4x the f32 chain's, a random 4-input network 5.8x -> 3.1x; tests/test_gpu_fp32x3.py)
        std::vector<double> top;
        ok = box_tops(dims, K, B, (double)X3_INPUT_BOUND, (double)X3_FRAME_BOUND, top);
        for (int l = 0; l < nl - 1 && ok; ++l) {
            if (!std::isfinite(top[l])) ok = false;
            e[l] = top[l] > 0.0 ? (int)std::ceil(std::log2(top[l])) - 10 : 0;
            if (e[l] < -100 || e[l] > 100) ok = false;
        }
    }
    const int ex = X3_XYZ_SHIFT;
    // fp16 hi / residual of a scaled weight; every hi must stay below 2^15
    auto split = [&](double ws, uint16_t &h, uint16_t &l) {
        if (!(std::fabs(ws) < 32768.0)) ok = false;
        const float w = (float)ws;  // exact: a power-of-two multiple of an f32 weight (range checked)
        h = f2fp16(w);
        l = f2fp16(w - fp16f(h));
    };
    auto crow = [](int h, int i) { return (i & 3) + 8 * (i >> 2) + 4 * h; };  // C/D row of register i
    auto kin = [](int s, int h, int k) { return 16 * s + 8 * (k >> 2) + 4 * h + (k & 3); };
    // layer 0, K = 16, as pack_lowp_32: h = 0 {wh x3 . xh, wh x3 . xl, wh3 . fh, wh3 . fl},
    //                                  h = 1 {wl x3 . xh, wl3 . fh, 0 x4}
    for (int lane = 0; lane < 64; ++lane) {
        const int m = lane & 31, h = lane >> 5;
        uint16_t *el = &a_ops[(size_t)lane * 8];
        for (int c = 0; c < in0; ++c) {
            const double ws = std::ldexp((double)K[0][(size_t)c * 32 + m], -e[0] - (c < 3 ? ex : 0));
            uint16_t wh, wl;
            split(ws, wh, wl);
            if (c < 3) {
                if (h == 0) el[c] = el[3 + c] = wh;
                else el[c] = wl;
            } else {
                if (h == 0) el[6] = el[7] = wh;
                else el[3] = wl;
            }
        }
    }
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 16; ++i) fl[h * 16 + i] = (float)std::ldexp((double)B[0][crow(h, i)], -e[0]);
    for (int j = 0; j < nh; ++j) {
        const std::vector<float> &Kj = K[j + 1];
        const int sw = e[j] - e[j + 1];
        for (int s = 0; s < 2; ++s)
            for (int lane = 0; lane < 64; ++lane)
                for (int k = 0; k < 8; ++k) {
                    const int m = lane & 31, h = lane >> 5;
                    const size_t o = (size_t)X3_HID + (size_t)j * X3_HSTRIDE + (size_t)s * 512 + lane * 8 + k;
                    split(std::ldexp((double)Kj[(size_t)kin(s, h, k) * 32 + m], sw), a_ops[o], a_ops[o + 1024]);
                }
        for (int h = 0; h < 2; ++h)
            for (int i = 0; i < 16; ++i) fl[32 + 32 * j + h * 16 + i] = (float)std::ldexp((double)B[j + 1][crow(h, i)], -e[j + 1]);
    }
    const int fo = x3_final(nh);
    for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 16; ++i) {
            const double w = std::ldexp((double)K[nl - 1][crow(h, i)], e[nl - 2]);
            if (K[nl - 1][crow(h, i)] != 0.0f && !(std::fabs(w) > 0x1p-120 && std::fabs(w) < 0x1p120)) ok = false;
            fl[fo + h * 16 + i] = (float)w;
        }
    fl[fo + 32] = B[nl - 1][0];
    fl[fo + 33] = -1.0f;
    fl[fo + 34] = std::ldexp(1.0f, ex);
    fl[fo + 35] = 1.0f;
    // scaled biases must stay normal f32 (power-of-two scaling exact)
    for (int l = 0; l < nl - 1; ++l)
        for (float b : B[l]) {
            const double bs = std::ldexp((double)b, -e[l]);
            if (b != 0.0f && !(std::fabs(bs) > 0x1p-120 && std::fabs(bs) < 0x1p120)) ok = false;
        }
    if (ok_out) *ok_out = ok ? 1 : 0;
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

// updateViewMatrices (main.cpp:207-222) in float, restating the scalar (non-vectorised) code
// paths of Eigen 3.3 that its expression takes (Eigen is not in this image: parity unpinned):
//   * the angles: -viewRotation.x * M_PI / 180 in double, rounded to float by AngleAxisf;
//   * AngleAxisf * AngleAxisf is a Quaternionf product (AngleAxis.h operator*): each factor
//     is (cos(a/2), sin(a/2) axis) (Quaternion.h operator=(AngleAxis)), the product the
//     generic quat_product (with one axis along x and the other along y, every term but one
//     of each component is a product with zero, so its rounding is that of a single product:
//     the SSE quat_product gives the same values);
//   * Matrix3f m = q: QuaternionBase::toRotationMatrix (tx = 2x, twx = tx w, ...);
//   * Affine3f::Identity().rotate(m): the linear part is I * m = m;
//   * .translate(v), v = -viewTranslation: translation = 0 + L v, each row a 3-term redux
//     in Eigen's unrolled order x0 + (x1 + x2);
//   * normalMatrix = modelView.matrix().inverse(): the generic 4x4 cofactor inverse
//     (InverseImpl.h compute_inverse_size4: cofactor_4x4 of general_det3_helper terms, then
//     division by det = (c0 + c1) + (c2 + c3)).  An SSE build of Eigen inverts 4x4 floats with
//     a different (Intel) sequence, so the last bits of the normal matrix are the part of this
//     restatement least likely to match a given reference build.
void camera_matrices_eigen(float rx, float ry, float zoom, float tx, float ty, float inv_view[12], float normal[16]) {
    const float ax = (float)((double)(-rx) * 3.14159265358979323846 / 180.0);
    const float ay = (float)((double)(-ry) * 3.14159265358979323846 / 180.0);
    // quaternions (w, x, y, z) of the two axis-angle rotations
    const float hx = 0.5f * ax, hy = 0.5f * ay;
    const float w1 = std::cos(hx), x1 = std::sin(hx) * 1.0f;  // axis UnitX
    const float w2 = std::cos(hy), y2 = std::sin(hy) * 1.0f;  // axis UnitY
    // generic quat_product: a = (w1, x1, 0, 0), b = (w2, 0, y2, 0), evaluated term by term
    const float z0 = 0.0f;
    const float qw = w1 * w2 - x1 * z0 - z0 * y2 - z0 * z0;
    const float qx = w1 * z0 + x1 * w2 + z0 * z0 - z0 * y2;
    const float qy = w1 * y2 + z0 * w2 + z0 * z0 - x1 * z0;
    const float qz = w1 * z0 + z0 * z0 + x1 * y2 - z0 * z0;
    // toRotationMatrix
    const float txq = 2.0f * qx, tyq = 2.0f * qy, tzq = 2.0f * qz;
    const float twx = txq * qw, twy = tyq * qw, twz = tzq * qw;
    const float txx = txq * qx, txy = tyq * qx, txz = tzq * qx;
    const float tyy = tyq * qy, tyz = tzq * qy, tzz = tzq * qz;
    float L[3][3];
    L[0][0] = 1.0f - (tyy + tzz); L[0][1] = txy - twz; L[0][2] = txz + twy;
    L[1][0] = txy + twz; L[1][1] = 1.0f - (txx + tzz); L[1][2] = tyz - twx;
    L[2][0] = txz - twy; L[2][1] = tyz + twx; L[2][2] = 1.0f - (txx + tyy);
    // translate(-viewTranslation), viewTranslation = (tx, ty, -zoom)
    const float v[3] = {-tx, -ty, -(-zoom)};
    float T[3];
    for (int i = 0; i < 3; ++i) T[i] = 0.0f + (L[i][0] * v[0] + (L[i][1] * v[1] + L[i][2] * v[2]));
    float M[4][4] = {{L[0][0], L[0][1], L[0][2], T[0]}, {L[1][0], L[1][1], L[1][2], T[1]},
                     {L[2][0], L[2][1], L[2][2], T[2]}, {0.0f, 0.0f, 0.0f, 1.0f}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) inv_view[4 * i + j] = M[i][j];
    auto det3 = [&](int i1, int i2, int i3, int j1, int j2, int j3) -> float {
        return M[i1][j1] * (M[i2][j2] * M[i3][j3] - M[i2][j3] * M[i3][j2]);
    };
    auto cof = [&](int i, int j) -> float {
        const int i1 = (i + 1) % 4, i2 = (i + 2) % 4, i3 = (i + 3) % 4;
        const int j1 = (j + 1) % 4, j2 = (j + 2) % 4, j3 = (j + 3) % 4;
        return det3(i1, i2, i3, j1, j2, j3) + det3(i2, i3, i1, j1, j2, j3) + det3(i3, i1, i2, j1, j2, j3);
    };
    float R[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) R[j][i] = ((i + j) & 1) ? -cof(i, j) : cof(i, j);
    const float det = (M[0][0] * R[0][0] + M[1][0] * R[0][1]) + (M[2][0] * R[0][2] + M[3][0] * R[0][3]);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) normal[4 * i + j] = R[i][j] / det;
}

}  // namespace nr
