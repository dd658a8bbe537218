// volumeRender.hh -- the reference's render entry points over libnr
// (src/volumeRender_kernel.cu:608-706, declared in src/main.cpp:97-109).
//
// render_kernel keeps the reference signature (grid/block are accepted and ignored:
// the gfx950 renderer picks its own persistent launch geometry) but takes the network
// by reference (the reference declared it by value, quirk Q11).  View matrices and
// static settings set by copyViewMatrices / copyStaticSettings are process-wide, as
// the reference's __constant__ state is.
#pragma once
#include <cstddef>

#include "image.hh"
#include "neuralNetwork.hh"

extern int NR_MAX_STEPS;      // host-loop cap, reference MAX_STEPS = 6000 (:61)
extern int NR_SCENE_MODE;     // NR_SCENE_V1 (manySphere union, :222) or NR_SCENE_TANH (:229)
extern int NR_PRECISION_MODE; // NR_PRECISION_FP32 (bit-exact contract) / _BF16 / _FP16

void render_kernel_nr(unsigned *d_output, unsigned imageW, unsigned imageH, unsigned numInputs, NeuralNetwork &nn,
                      const Image &matcap);

template <class D3>
inline void render_kernel(D3 gridSize, D3 blockSize, unsigned *d_output, unsigned imageW, unsigned imageH,
                          unsigned numInputs, NeuralNetwork &nn, const Image &matcap) {
    (void)gridSize;
    (void)blockSize;
    render_kernel_nr(d_output, imageW, imageH, numInputs, nn, matcap);
}

extern "C" void copyViewMatrices(float *invViewMatrix, size_t sizeofViewMatrix, float *normalMatrix,
                                 size_t sizeofNormalMatrix, int frameNumber);
extern "C" void copyStaticSettings(int colorType, int numInputs);
