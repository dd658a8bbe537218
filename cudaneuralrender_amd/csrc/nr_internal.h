// nr_internal.h -- declarations shared by the host side of libnr.so.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/neural_render.h"

#if defined(__HIPCC__)
#define NR_HD __host__ __device__
#else
#define NR_HD
#endif

namespace nr {

// ---- host-side file formats (h5_keras.cpp, png_codec.cpp) ----
int h5_read_keras(const char *path, std::vector<int> &dims, std::vector<std::vector<float>> &kernels,
                  std::vector<std::vector<float>> &biases, std::string &err);
int png_decode(const char *path, std::vector<uint32_t> &rgba, int &w, int &h, std::string &err);
int png_encode(const char *path, const uint32_t *rgba, int w, int h, int flip, std::string &err);
int ppm_encode(const char *path, const uint32_t *rgba, int w, int h, std::string &err);
// Records the calling thread's last error (nr_last_error(NULL)) and returns code.
int report_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// ---- packed network layouts (nr_pack.cpp) ----
// fp32 16-point-tile layout (nr_mlp16.h), in floats.  Lane (j, g) of a wave = row /
// point j, unit group g; hidden unit u lives in register k of group g with u = 4k + g
// (u = 8g + k for the layer that feeds the final VALU layer), so every f32 MFMA chain
// runs over k ascending:
//   [0,128)    layer-0 A operand   [row tile 2][lane 64]      (k = x, y, z, frame)
//   [128,160)  layer-0 bias        [group 4][register 8]
//   per hidden layer j (0..nh-1), base 160 + j*1056:
//              A operand           [m >> 2][lane 64][m & 3]   (m = 2 * k-step + row tile)
//              bias                [group 4][register 8]
//   final:     weights [group 4][register 8], bias [1], layer-0 output scale 2^-e0 [1] (+2 pad)
constexpr int PK_L0W = 0;
constexpr int PK_L0B = 128;
constexpr int PK_HID = 160;
constexpr int PK_HID_STRIDE = 1024 + 32;
constexpr int MAX_HIDDEN = 16;
NR_HD constexpr inline int pk_final(int nh) { return PK_HID + nh * PK_HID_STRIDE; }
NR_HD constexpr inline int pk_floats(int nh) { return pk_final(nh) + 36; }

// Low-precision (bf16/fp16) pack for the 32-point-tile MLP (nr_mlp16.h, mlp32_lowp):
// v_mfma_f32_32x32x16_{bf16,f16}, lane l = (row / point r = l & 31, half h = l >> 5).
// 16-bit elements (a_ops):
//   [0, 512)                    layer-0 A operand [lane 64][8]: K = 16 slots holding the
//                               hi/lo split of weights and inputs (w*x ~ wh*xh + wh*xl + wl*xh)
//   LP32_HID + j*LP32_HSTRIDE   hidden layer j: A operand [k-step 2][lane 64][8]; element e of
//                               lane half h in k-step s multiplies unit 16s + 8(e>>2) + 4h + (e&3)
//                               (the accumulator-as-B-operand order of the previous layer)
//   lp32_final(nh)              final layer: row 0 of the A operand only, [k-step 2][h 2][8]
// floats (fl): biases as accumulator inits, [h 2][register 16] per layer (register i of half
// h = unit (i&3) + 8(i>>2) + 4h): layer 0 at 0, hidden j at 32 + 32j, final bias at 32 + 32nh.
constexpr int LP32_HID = 512;
constexpr int LP32_HSTRIDE = 1024;
NR_HD constexpr inline int lp32_final(int nh) { return LP32_HID + nh * LP32_HSTRIDE; }
NR_HD constexpr inline int lp32_elems(int nh) { return lp32_final(nh) + 32; }
NR_HD constexpr inline int lp32_floats(int nh) { return 32 + 32 * nh + 4; }
// bf16 clamped-ReLU pack: every network input within +-LP_INPUT_BOUND keeps every scaled
// activation at or below 1/4 (interval bounds, nr_pack.cpp pack_lowp_32)
constexpr float LP_INPUT_BOUND = 1048576.0f;
// fp32 clamped-ReLU pack (pack_fp32_16): inputs within +-F32_INPUT_BOUND keep every scaled
// activation at or below 1/2 (nr_mlp16.h inputs_in_bound_f32; beyond it the add + max form)
constexpr float F32_INPUT_BOUND = 1024.0f;

// fp32x3 pack (pack_x3_32): fp32-class hidden layers on the fp16 matrix core by a three-term
// split, a.w ~ ah.wh + al.wh + ah.wl (nr_mlp16.h mlp32_x3_nt).  16-bit elements (fp16):
//   [0, 512)                    layer-0 A operand, as LP32 (hi/lo split of scaled weights)
//   X3_HID + j*X3_HSTRIDE       hidden layer j: hi A operand [k-step 2][lane 64][8], then the
//                               residual (lo) A operand in the same order (+1024)
// floats (fl): layer-0 bias [h 2][register 16] at 0, hidden j's bias at 32 + 32j (all scaled,
// accumulator inits), the final layer's f32 weights in the accumulator's register order
// [h 2][register 16] at x3_final(nh), its bias at +32, then -1 (the residual's multiplier, read
// at run time so that the compiler emits v_fma_mix), the xyz input scale and the 4th input's
// scale.  Activations of ReLU layer l are scaled by 2^-e[l] so that their interval bound over
// inputs within X3_INPUT_BOUND (xyz) / X3_FRAME_BOUND (4th input) is at most 2^10: the split's
// residual (x - rtz(x)) is then below 1 and the clamp of v_fma_mixlo_f16 is its ReLU.
constexpr int X3_HID = 512;
constexpr int X3_HSTRIDE = 2048;
NR_HD constexpr inline int x3_elems(int nh) { return X3_HID + nh * X3_HSTRIDE; }
NR_HD constexpr inline int x3_final(int nh) { return 32 + 32 * nh; }
NR_HD constexpr inline int x3_floats(int nh) { return x3_final(nh) + 36; }
constexpr float X3_INPUT_BOUND = 4.0f;
constexpr float X3_FRAME_BOUND = 1024.0f;
constexpr int X3_XYZ_SHIFT = 6;  // xyz inputs enter layer 0 times 2^6

bool fused_shape_ok(const std::vector<int> &dims);
// Keras kernels (in x out, row-major) -> packs.  Return false if the shape is not
// [3|4, 32, ..., 32, 1] (those networks render on the layered schedule).
// pack_fp32_16: clamp (if not null) = 1 when the pack is scaled for the clamped ReLU
bool pack_fp32_16(const std::vector<int> &dims, const std::vector<std::vector<float>> &kernels,
                  const std::vector<std::vector<float>> &biases, std::vector<float> &pack, int *clamp = nullptr);
bool pack_lowp_32(const std::vector<int> &dims, const std::vector<std::vector<float>> &kernels,
                  const std::vector<std::vector<float>> &biases, int precision,
                  std::vector<uint16_t> &a_ops, std::vector<float> &bias, int *clamp = nullptr);
// The 16x16x32 form of pack_lowp_32's output for k_mlp16 (round 6; nr_mlp16_asm.h NR_S16_*,
// tools/gen_mlp_asm.py build_s16): the same elements re-ordered -- the input layer's rows permuted,
// each hidden layer's A operand as [half 2][lane 64][8] (lane (row j, group g): output unit
// U(half, j), k-slot 8g + e: input unit V(g, e)) and its bias as [group 4][half 2][4]; the final
// layer unchanged.  Same sizes as the 32x32x16 pack.
void pack_lowp_s16(const std::vector<uint16_t> &a32, const std::vector<float> &f32, int nh,
                   std::vector<uint16_t> &a16, std::vector<float> &f16);
// ok (if not null) = 1 when the scales exist (every scaled weight and bound inside fp16's range);
// otherwise the kernels run the fp32 MLP for every point
bool pack_x3_32(const std::vector<int> &dims, const std::vector<std::vector<float>> &kernels,
                const std::vector<std::vector<float>> &biases, std::vector<uint16_t> &a_ops, std::vector<float> &fl,
                int *ok = nullptr);

// ---- context internals for nr_group.hip (nr_api.hip) ----
int ctx_device(const nr_ctx *c);
void *ctx_stream(nr_ctx *c);  // the hipStream_t the context's work runs on (creates its own stream if selected)

// ---- camera (nr_pack.cpp; the C ABI's nr_camera) ----
void camera_matrices(float rx, float ry, float zoom, float tx, float ty, float inv_view[12], float normal[16]);
void camera_matrices_eigen(float rx, float ry, float zoom, float tx, float ty, float inv_view[12], float normal[16]);

}  // namespace nr
