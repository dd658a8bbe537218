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
//   final:     weights [group 4][register 8], bias [1] (+3 pad)
constexpr int PK_L0W = 0;
constexpr int PK_L0B = 128;
constexpr int PK_HID = 160;
constexpr int PK_HID_STRIDE = 1024 + 32;
constexpr int MAX_HIDDEN = 16;
NR_HD constexpr inline int pk_final(int nh) { return PK_HID + nh * PK_HID_STRIDE; }
NR_HD constexpr inline int pk_floats(int nh) { return pk_final(nh) + 36; }

// Low-precision (bf16/fp16) hidden-layer A operands, 16-bit elements per layer:
// [row tile 2][lane 64][8] for v_mfma_f32_16x16x32_{bf16,f16}; a separate float array
// holds layer 0 (f32 MFMA), the hidden biases and the final layer.
constexpr int LP_A_ELEMS = 2 * 64 * 8;

bool fused_shape_ok(const std::vector<int> &dims);
// Keras kernels (in x out, row-major) -> packs.  Return false if the shape is not
// [3|4, 32, ..., 32, 1] (those networks render on the layered schedule).
bool pack_fp32_16(const std::vector<int> &dims, const std::vector<std::vector<float>> &kernels,
                  const std::vector<std::vector<float>> &biases, std::vector<float> &pack);
bool pack_lowp_16(const std::vector<int> &dims, const std::vector<std::vector<float>> &kernels,
                  const std::vector<std::vector<float>> &biases, int precision,
                  std::vector<uint16_t> &a_ops, std::vector<float> &bias);

// ---- camera (nr_camera.cpp) ----
void camera_matrices(float rx, float ry, float zoom, float tx, float ty, float inv_view[12], float normal[16]);

}  // namespace nr
