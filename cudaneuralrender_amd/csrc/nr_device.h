// nr_device.h -- device-side building blocks shared by the march kernels
// (nr_kernels.hip: wavefront schedule, nr_trace.hip: persistent schedule).
//
// Restatement of the reference device helpers (helper_math.h:1248-1313,
// volumeRender_kernel.cu:38-61, :67-275, :361-413); the expression-by-expression
// float/double promotions mirror the CUDA source (double literals promote) and are
// kept in lock-step with oracle/nr_oracle.c.  Compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nr_internal.h"
#include "nr_kernels.h"

namespace nr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// ------------------------------------------------------------------ float math
// Restatement of the reference device helpers (helper_math.h:1248-1313,
// volumeRender_kernel.cu:67-275); the expression-by-expression promotions mirror
// the CUDA source (double literals promote).  Kept in lock-step with the oracle.

struct F3 { float x, y, z; };
__device__ __forceinline__ F3 mk3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ F3 add3(F3 a, F3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ F3 mul3s(F3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot3(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float length3(F3 v) { return sqrtf(dot3(v, v)); }
__device__ __forceinline__ F3 normalize3(F3 v) { float inv = 1.0f / sqrtf(dot3(v, v)); return mul3s(v, inv); }
__device__ __forceinline__ float dot4(float a0, float a1, float a2, float a3, const float *b) {
    return a0 * b[0] + a1 * b[1] + a2 * b[2] + a3 * b[3];
}
__device__ __forceinline__ float saturatef_(float x) {
    if (!(x > 0.0f)) return 0.0f;
    if (x > 1.0f) return 1.0f;
    return x;
}
__device__ __forceinline__ int f2i_rz(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}

// intersectSphere (volumeRender_kernel.cu:199-215) against the bounding sphere (c = 0,
// r = 1.2).  The reference forms b as (float)(2.0 * (double)dot) -- exact in f32 -- and
// each root as an f64 division rounded to f32; a single correctly rounded f32 division
// gives the same bits (innocuous double rounding: 53 >= 2*24 + 2), proven on the CPU by
// tests/test_oracle.py::test_intersect_sphere_f32_division_bit_exact.  Saves the two
// f64 divisions per generated ray.
__device__ __forceinline__ bool intersect_bounding(F3 o, F3 d, float &tnear, float &tfar) {
    const F3 Qv = mk3(o.x - 0.0f, o.y - 0.0f, o.z - 0.0f);
    const float a = dot3(d, d);
    const float b = 2.0f * dot3(Qv, d);
    const float cc = dot3(Qv, Qv) - 1.2f * 1.2f;
    const float disc = b * b - 4 * a * cc;
    if (!(disc > 0)) return false;
    const float sq = sqrtf(disc);
    const float a2 = 2.0f * a;
    tnear = (-b - sq) / a2;
    tfar = (-b + sq) / a2;
    return true;
}

static __constant__ float c_tet[12] = {1, -1, -1, -1, -1, 1, -1, 1, -1, 1, 1, 1};  // :38-43
#define NORMAL_EPSILON 0.00001f
#define MARCHING_EPSILON 0.000001f

// tanh from IEEE basic double operations (identical algorithm to the oracle).
__device__ double expm1_pos(double t) {
    if (t < 0.5) {
        const double inv_fact[19] = {
            1.0, 1.0 / 2.0, 1.0 / 6.0, 1.0 / 24.0, 1.0 / 120.0, 1.0 / 720.0,
            1.0 / 5040.0, 1.0 / 40320.0, 1.0 / 362880.0, 1.0 / 3628800.0,
            1.0 / 39916800.0, 1.0 / 479001600.0, 1.0 / 6227020800.0,
            1.0 / 87178291200.0, 1.0 / 1307674368000.0, 1.0 / 20922789888000.0,
            1.0 / 355687428096000.0, 1.0 / 6402373705728000.0,
            1.0 / 121645100408832000.0};
        double s = inv_fact[18];
#pragma unroll
        for (int i = 17; i >= 0; --i) s = s * t + inv_fact[i];
        return s * t;
    }
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    double kd = floor(t * 1.44269504088896338700 + 0.5);
    double r = (t - kd * ln2_hi) - kd * ln2_lo;
    const double c[18] = {
        1.0, 1.0, 1.0 / 2.0, 1.0 / 6.0, 1.0 / 24.0, 1.0 / 120.0, 1.0 / 720.0,
        1.0 / 5040.0, 1.0 / 40320.0, 1.0 / 362880.0, 1.0 / 3628800.0,
        1.0 / 39916800.0, 1.0 / 479001600.0, 1.0 / 6227020800.0,
        1.0 / 87178291200.0, 1.0 / 1307674368000.0, 1.0 / 20922789888000.0,
        1.0 / 355687428096000.0};
    double e = 1.0 / 6402373705728000.0;
#pragma unroll
    for (int i = 17; i >= 0; --i) e = e * r + c[i];
    e = ldexp(e, (int)kd);
    return e - 1.0;
}

__device__ float nr_tanh(float x) {
    if (x != x) return x;
    double ax = fabs((double)x);
    if (ax > 9.5) return x > 0 ? 1.0f : -1.0f;
    double em1 = expm1_pos(2.0 * ax);
    double t = em1 / (em1 + 2.0);
    float r = (float)t;
    return x < 0 ? -r : r;
}

__device__ __forceinline__ float smooth_union(float d1, float d2, float k) {  // :144-149
    // Reference: h = __saturatef(0.5 + 0.5*(d2-d1)/k); mix = d2*(1.0-h) + d1*h;
    // return mix - k*h*(1.0-h), with the double literals promoting to f64.
    // When |d2-d1| >= k the f64 quotient is >= 0.5 in magnitude (division and rounding
    // are monotone, 0.5 is representable), so h is exactly 1 or 0, and what remains is
    // exact in f32: h = 1 gives (d2*0 + d1) - (+0) = d2*0 + d1, h = 0 gives
    // (d2 + d1*0) - (+0) = d1*0 + d2 -- each one fmaf, since the product by 0 is exact
    // (signed zeros and NaN/inf operands included; proven on the CPU against the reference
    // form, tests/test_oracle.py).
    const float t = d2 - d1;
    if (t >= k) return __builtin_fmaf(d2, 0.0f, d1);
    if (t <= -k) return __builtin_fmaf(d1, 0.0f, d2);
    const float h = saturatef_((float)(0.5 + 0.5 * (double)t / (double)k));
    const float mix = (float)((double)d2 * (1.0 - (double)h) + (double)(d1 * h));
    return (float)((double)mix - (double)(k * h) * (1.0 - (double)h));
}

// z offset of the sphere grid in frame `frame` (cP.z += ..., :184), in f64 as the reference
__device__ __forceinline__ double sphere_zoff(int frame) { return -0.7 + ((double)(frame * 2) * 0.7 / 360.0); }

// sdfOpSmoothSubtraction (:137-142): h = __saturatef(0.5 - 0.5*(d1+d2)/k);
// mix = d1*(1.0-h) - d2*h; return mix + k*h*(1.0-h) -- the double literals promote.  As in
// smooth_union, |d1+d2| >= k makes the f64 quotient >= 0.5 in magnitude, so h is exactly
// 0 or 1 and only the division is skipped; the rest is the reference expression with that
// h (CPU proof: tests/test_oracle.py::test_smooth_subtraction_kernel_form_bit_exact).
__device__ __forceinline__ float smooth_sub_h(float d1, float d2, float k, float h) {
    const float mix = (float)((double)d1 * (1.0 - (double)h) - (double)(d2 * h));
    return (float)((double)mix + (double)(k * h) * (1.0 - (double)h));
}
__device__ __forceinline__ float smooth_subtraction(float d1, float d2, float k) {
    const float t = d1 + d2;
    float h;
    if (t >= k) h = 0.0f;
    else if (t <= -k) h = 1.0f;
    else h = saturatef_((float)(0.5 - 0.5 * (double)t / (double)k));
    return smooth_sub_h(d1, d2, k, h);
}

// sin from IEEE basic double operations (identical algorithm to the oracle's nr_sin_f):
// x - k pi/2 with a two-part pi/2, then the Taylor series of sin / cos to degree 21 / 22
// (|r| <= pi/4), rounded once to f32.  CUDA's sinf is not pinned; both sides need one
// definition (as for tanh).
__device__ float nr_sin(float xf) {
    if (xf != xf) return xf;
    if (xf == INFINITY || xf == -INFINITY) return __builtin_nanf("");
    const double x = (double)xf;
    const double kd = floor(x * 0.63661977236758134308 + 0.5);
    const double r = (x - kd * 1.57079632673412561417e+00) - kd * 6.07710050650619224932e-11;
    const double z = r * r;
    const double sc[11] = {1.0, -1.0 / 6.0, 1.0 / 120.0, -1.0 / 5040.0, 1.0 / 362880.0, -1.0 / 39916800.0,
                           1.0 / 6227020800.0, -1.0 / 1307674368000.0, 1.0 / 355687428096000.0,
                           -1.0 / 121645100408832000.0, 1.0 / 51090942171709440000.0};
    const double cc[12] = {1.0, -1.0 / 2.0, 1.0 / 24.0, -1.0 / 720.0, 1.0 / 40320.0, -1.0 / 3628800.0,
                           1.0 / 479001600.0, -1.0 / 87178291200.0, 1.0 / 20922789888000.0,
                           -1.0 / 6402373705728000.0, 1.0 / 2432902008176640000.0,
                           -1.0 / 1124000727777607680000.0};
    double ps = sc[10], pc = cc[11];
#pragma unroll
    for (int i = 9; i >= 0; --i) ps = ps * z + sc[i];
#pragma unroll
    for (int i = 10; i >= 0; --i) pc = pc * z + cc[i];
    const double sn = r * ps;
    const int q = (int)(kd - 4.0 * floor(kd * 0.25));  // k mod 4 in [0, 3]
    const double v = q == 0 ? sn : (q == 1 ? pc : (q == 2 ? -sn : -pc));
    return (float)v;
}

// The correctly rounded square root on [2^-96, FLT_MAX]: v_sqrt_f32 and the two-FMA rounding
// correction -- the sequence hipcc emits for sqrtf, without the denormal-range scaling and
// the zero / infinity / NaN class check that only inputs outside that range need (7 of its
// 16 VALU).  Equal to sqrtf on every float of the domain (tools/sqrt_exhaustive.hip).
__device__ __forceinline__ float sqrt_rn_normal(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    const float r = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : r;
}

__device__ float many_sphere(F3 p, float nsdf, double zoff) {  // :176-196
    // The reference walks cP through the 3x3 grid with f64 updates (cP.y -= 0.6,
    // cP.z += ..., per row cP.y += 0.4 and cP.x = p.x + 0.5, per sphere cP.x -= 0.4);
    // the x values repeat in every row, so the 3 x, 3 y and 1 z coordinates are formed
    // once with the same f64 operations and reused -- but for x0: p.x + 0.5 is exact in f64 for
    // |p.x| >= 2^-30 and rounds to 0.5 either way below, so the single f32 add gives the same
    // bits (tests/test_oracle.py::test_scene_x0_f32_add_equals_f64_form).
    const float x0 = p.x + 0.5f;
    const float x1 = (float)((double)x0 - 0.4);
    const float x2 = (float)((double)x1 - 0.4);
    const float ys = (float)((double)p.y - 0.6);
    const float y0 = (float)((double)ys + 0.4);
    const float y1 = (float)((double)y0 + 0.4);
    const float y2 = (float)((double)y1 + 0.4);
    const float zc = (float)((double)p.z + zoff);
    const float xx[3] = {x0 * x0, x1 * x1, x2 * x2};
    const float yy[3] = {y0 * y0, y1 * y1, y2 * y2};
    const float zz = zc * zc;
    // All 9 sphere distances first -- 9 independent correctly rounded square roots the
    // wave issues back to back -- then the sequential smooth-union chain, which is the
    // reference's loop in the reference's order (length(cP) = sqrtf(dot(cP, cP))).  In a
    // wave of scattered rays nearly every sphere has some lane near it, so skipping the
    // square roots of far spheres behind a branch cost more than it saved
    // (tools/scene_bench.hip).
    float q[9];
#pragma unroll
    for (int row = 0; row < 3; ++row)
#pragma unroll
        for (int col = 0; col < 3; ++col) q[3 * row + col] = (xx[col] + yy[row]) + zz;
    // Every q is >= zz, >= min xx and >= min yy, and <= (max xx + max yy) + zz (rounding is
    // monotone and the terms are non-negative): when the wave's bounds put all nine in
    // sqrt_rn_normal's domain (all but points within 1e-14 of a sphere centre, or non-finite
    // ones), the short sequence gives the same bits as sqrtf.
    const float lo = fmaxf(zz, fmaxf(fminf(fminf(xx[0], xx[1]), xx[2]), fminf(fminf(yy[0], yy[1]), yy[2])));
    const float hi = (fmaxf(fmaxf(xx[0], xx[1]), xx[2]) + fmaxf(fmaxf(yy[0], yy[1]), yy[2])) + zz;
    // Screening (round 3): smoothUnion(s, d, k) with d - s >= k is fmaf(d, 0, s) -- it does not
    // depend on d's value, only on that test (and on d's sign when s is +-0, where the test
    // already makes d >= k > 0).  The running union never exceeds the surface value nsdf
    // (smoothUnion(a, b) <= min(a, b)), so a sphere whose distance from the raw v_sqrt_f32 (within
    // 1 ulp of the correctly rounded root; tools/sqrt_exhaustive.hip) is beyond nsdf + k by more
    // than 2^-18 of the magnitudes involved (a thousand-fold margin over the rounding differences)
    // is beyond the running value + k in every lane: when that holds for the whole wave, the
    // sphere costs v_sqrt_f32 and the test instead of the correction, the sub and the union --
    // bit for bit the same result.  Spheres that some lane is near take the exact path.
    //
    // The test runs on the squared distance (round 3, later): sphere i is far when q[i] >= T2 =
    // max(T, 0)^2 with T = (nsdf + 0.11f) + (|nsdf| + 0.2f) 2^-16, all in f32.  Every rounding
    // between q and the union's test (T*T, the root, - 0.1f, - s) is monotone and within
    // 2^-24 of values of magnitude <= |nsdf| + 0.22 near the threshold, against a margin of
    // 2^-16 (|nsdf| + 0.2) -- sixty-fold; 0.11f - 0.1f falls short of 0.01f by 2e-9 of it.  With
    // T <= 0 every sphere passes (d >= -0.1f and -nsdf >= 0.11 + margin).  A NaN nsdf gives a NaN
    // T2 and the exact path.  A far sphere adds +0 to s (fmaf(d, 0, s) with d > 0 whenever s is
    // +-0), so neither its root nor d is formed: one compare per sphere instead of v_sqrt_f32
    // and five VALU.  tests/test_oracle.py::test_scene_far_screen_implies_union_test samples the
    // implication at and around the threshold.
    if (__ballot(!(lo >= 0x1p-96f && hi <= 0x1.fffffep127f)) == 0) {
        const float T = __builtin_fmaf(__builtin_fabsf(nsdf) + 0.2f, 0x1p-16f, nsdf + 0.11f);
        const float Tc = T < 0.0f ? 0.0f : T;
        const float T2 = Tc * Tc;
        float s = nsdf;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            if (__ballot(!(q[i] >= T2)) == 0) s = s + 0.0f;
            else s = smooth_union(s, sqrt_rn_normal(q[i]) - 0.1f, 0.01f);
        }
        return s;
    }
    float s = nsdf;
#pragma unroll
    for (int i = 0; i < 9; ++i) s = smooth_union(s, sqrtf(q[i]) - 0.1f, 0.01f);
    return s;
}

// manySphere(p, nSDF, false) (:176-196): the 9 spheres smooth-subtracted from the surface,
// the coordinates formed as in many_sphere
__device__ float many_sphere_sub(F3 p, float nsdf, double zoff) {
    const float x0 = p.x + 0.5f;  // = (float)((double)p.x + 0.5), see many_sphere
    const float x1 = (float)((double)x0 - 0.4);
    const float x2 = (float)((double)x1 - 0.4);
    const float ys = (float)((double)p.y - 0.6);
    const float y0 = (float)((double)ys + 0.4);
    const float y1 = (float)((double)y0 + 0.4);
    const float y2 = (float)((double)y1 + 0.4);
    const float zc = (float)((double)p.z + zoff);
    const float xx[3] = {x0 * x0, x1 * x1, x2 * x2};
    const float yy[3] = {y0 * y0, y1 * y1, y2 * y2};
    const float zz = zc * zc;
    float s = nsdf;
#pragma unroll
    for (int row = 0; row < 3; ++row)
#pragma unroll
        for (int col = 0; col < 3; ++col) s = smooth_subtraction(s, sqrtf((xx[col] + yy[row]) + zz) - 0.1f, 0.01f);
    return s;
}

// manyCylinderCut (:157-174): 300 cylinders (sdfCylinder :96-100, c = 0.02, infinite along
// z) in 15 rows of 20 smooth-subtracted from the surface; cP.y starts at p.y - 0.5 and
// every row adds 0.1 and resets cP.x = p.x + 0.9, every cylinder then steps cP.x by -0.1
// (f64 updates of f32 coordinates, as the reference's double literals make them)
__device__ float many_cylinder_cut(F3 p, float nsdf) {
    float s = nsdf;
    float cy = (float)((double)p.y - 0.5);
    for (int row = 0; row < 15; ++row) {
        cy = (float)((double)cy + 0.1);
        const float dy = cy - 0.02f;
        const float dyy = dy * dy;
        float cx = (float)((double)p.x + 0.9);
        for (int col = 0; col < 20; ++col) {
            const float dx = cx - 0.02f;
            s = smooth_subtraction(s, sqrtf(dx * dx + dyy) - 0.02f, 0.01f);
            cx = (float)((double)cx - 0.1);
        }
    }
    return s;
}

// displacementPattern (:151-154) = sdfOpDisplace(p, tanh(nSDF)) (:103-110):
// d += sin(5 p.x) sin(5 p.y) sin(5 p.z) * 0.05 (f32 products, the 0.05 promotes)
__device__ float displacement_pattern(F3 p, float nsdf) {
    const float d = nr_tanh(nsdf);
    const float w = nr_sin(5.0f * p.x) * nr_sin(5.0f * p.y) * nr_sin(5.0f * p.z);
    return (float)((double)d + (double)w * 0.05);
}

// The scenes sceneSDF's alternatives select (:217-230), out of line so that the inlined
// v1 / tanh paths of the march kernels keep their registers.
__device__ __noinline__ float scene_sdf_alt(F3 p, float nsdf, int scene, double zoff) {
    if (scene == NR_SCENE_SUBTRACT) return many_sphere_sub(p, nsdf, zoff);
    if (scene == NR_SCENE_CYLINDERS) return many_cylinder_cut(p, nsdf);
    if (scene == NR_SCENE_DISPLACE) return displacement_pattern(p, nsdf);
    return nr_tanh(nsdf) - 0.04f;  // NR_SCENE_ROUND: sdfOpRound(tanh(nSDF), 0.04) (:112-115, :221)
}

__device__ __forceinline__ float scene_sdf(F3 p, float nsdf, int scene, double zoff) {  // :217-230
    if (scene == NR_SCENE_V1) return many_sphere(p, nsdf, zoff);
    if (scene == NR_SCENE_TANH) return nr_tanh(nsdf);
    return scene_sdf_alt(p, nsdf, scene, zoff);
}

__device__ __forceinline__ uint32_t rgba_to_uint(float r, float g, float b, float a) {  // :266-274
    r = saturatef_(r); g = saturatef_(g); b = saturatef_(b); a = saturatef_(a);
    return ((uint32_t)(a * 255) << 24) | ((uint32_t)(b * 255) << 16) | ((uint32_t)(g * 255) << 8) |
           (uint32_t)(r * 255);
}

// nm: the frame's normal matrix (c_normalMatrix, row-major 4x4)
__device__ uint32_t shade_color(const RenderArgs &A, const float *nm, F3 n, F3 d) {
    if (A.color_type == NR_COLOR_FACING) {  // facingColor :380-384
        float dd = dot3(n, mk3(-d.x, -d.y, -d.z));
        float ratio = (dd > 0.0f) ? dd : 0.0f;
        return rgba_to_uint(ratio, ratio, ratio, 1.0f);
    }
    // matCapColor :387-413
    float ex = dot4(n.x, n.y, n.z, 0.0f, nm + 0);
    float ey = dot4(n.x, n.y, n.z, 0.0f, nm + 4);
    float ez = dot4(n.x, n.y, n.z, 0.0f, nm + 8);
    F3 ne = normalize3(mk3(ex, ey, ez));
    float fuvx = (float)((double)ne.x * 0.5 + 0.5);
    float fuvy = (float)((double)ne.y * 0.5 + 0.5);
    int uvx = f2i_rz(fuvx * (float)(A.mw - 1));
    int uvy = f2i_rz(fuvy * (float)(A.mh - 1));
    if (uvx > A.mw - 1) uvx = A.mw - 1;
    if (uvy > A.mh - 1) uvy = A.mh - 1;
    long index = (long)uvy * A.mw + uvx;
    if (index < 0) return 0u;
    return A.matcap[index];
}

// initMarcher's (x / (float)imageW) * 2 - 1 (:315-316); with a power-of-two divisor (rcp = 1/W, else 0)
// the quotient is the product by the exact reciprocal, bit for bit
__device__ __forceinline__ float pixel_uv(int x, int W, float rcp) {
    const float q = rcp != 0.0f ? (float)x * rcp : (float)x / (float)W;
    return q * 2.0f - 1.0f;
}

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// v of lane 4 * (l / 4) + Q of this lane's quad (DPP quad_perm: a VALU operand modifier, no LDS
// round trip and no per-lane address register)
template <int Q>
__device__ __forceinline__ float quad_bcast(float v) {
    constexpr int ctrl = Q | (Q << 2) | (Q << 4) | (Q << 6);
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, false));
}
__device__ __forceinline__ F3 quad_bcast3_1(const F3 &v) { return mk3(quad_bcast<1>(v.x), quad_bcast<1>(v.y), quad_bcast<1>(v.z)); }
__device__ __forceinline__ F3 quad_bcast3_2(const F3 &v) { return mk3(quad_bcast<2>(v.x), quad_bcast<2>(v.y), quad_bcast<2>(v.z)); }
__device__ __forceinline__ F3 quad_bcast3_3(const F3 &v) { return mk3(quad_bcast<3>(v.x), quad_bcast<3>(v.y), quad_bcast<3>(v.z)); }

__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// popcount(m & lanemask_lt()): the set lanes of m below this one, by v_mbcnt_lo / v_mbcnt_hi.
// (Formed from lanemask_lt(), the per-lane 64-bit mask is a loop invariant the compiler hoists
// out of the tracer's loop and keeps in two VGPRs for the kernel's life: the batched fp32
// k_trace spilled it to scratch.)
__device__ __forceinline__ uint32_t rank_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Position of the d-th (0-based) set bit of m (m must have more than d bits set).
__device__ __forceinline__ int select_bit(uint64_t m, int d) {
    int lo = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        uint64_t below = m & ((1ull << (lo + step)) - 1ull);
        if (__popcll(below) <= d) lo += step;
    }
    return lo;
}

// n / d (d >= 1) from a precomputed f64 reciprocal: n * (1/d) = (n/d)(1 + e), |e| <= 2^-52,
// is within n/d * 2^-52 < 1/d of n/d -- closer than any non-integer n/d is to an
// integer -- so the truncation is the quotient or, for an exact multiple, one less,
// which the remainder test repairs.
__device__ __forceinline__ uint32_t udiv_r(uint32_t n, uint32_t d, double inv_d) {
    uint32_t q = (uint32_t)((double)n * inv_d);
    if (n - q * d >= d) ++q;
    return q;
}

// Exclusive position of this lane among the set lanes of `pred`, and one atomic per wave.
__device__ __forceinline__ uint32_t wave_append(bool pred, uint32_t *counter) {
    uint64_t m = __ballot(pred);
    uint32_t cnt = (uint32_t)__popcll(m);
    if (cnt == 0) return 0;
    int lane = lane_id();
    int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, cnt);
    base = __shfl(base, leader);
    return base + rank_below(m);
}

// Block-aggregated append to two queues: one atomic per queue per block.  Same-address
// atomics serialise at ~10 ns each in L2, so per-wave appends of a 1M-ray queue cost
// more than the step itself.  Every thread of the block (<= 16 waves) must call it.
struct Slots {
    uint32_t a, b;    // this lane's slot in queue a / b (valid where its predicate holds)
    uint32_t na, nb;  // the block's totals
};
__device__ __forceinline__ Slots block_append2(bool pa, uint32_t *ca, bool pb, uint32_t *cb) {
    __shared__ uint32_t s_app[2][17];  // per-wave counts -> exclusive offsets; [16] = base, then total
    __shared__ uint32_t s_tot[2];
    const int wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6, lane = lane_id();
    const uint64_t ma = __ballot(pa), mb = __ballot(pb);
    if (lane == 0) {
        s_app[0][wv] = (uint32_t)__popcll(ma);
        s_app[1][wv] = (uint32_t)__popcll(mb);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const int q = threadIdx.x;
        uint32_t tot = 0;
        for (int w = 0; w < nw; ++w) {
            const uint32_t c = s_app[q][w];
            s_app[q][w] = tot;
            tot += c;
        }
        s_app[q][16] = tot ? atomicAdd(q ? cb : ca, tot) : 0u;
        s_tot[q] = tot;
    }
    __syncthreads();
    Slots r;
    r.a = s_app[0][16] + s_app[0][wv] + rank_below(ma);
    r.b = s_app[1][16] + s_app[1][wv] + rank_below(mb);
    r.na = s_tot[0];
    r.nb = s_tot[1];
    __syncthreads();  // the arrays are reused by the next call
    return r;
}

}  // namespace nr
