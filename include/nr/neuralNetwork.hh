// neuralNetwork.hh -- MLP container + Keras .h5 loader (reference src/neuralNetwork.hh:9-30).
// Same methods.  Differences: the object is non-copyable
// (the reference's by-value pass to render_kernel deleted its layers twice), and it
// owns a libnr context whose fused gfx950 kernel evaluates the whole network in one
// launch when the layers have the bundled shape [3|4, 32, ..., 32, 1].
#pragma once
#include <string>
#include <vector>

#include "layer.hh"

struct nr_ctx;

class NeuralNetwork {
  private:
    std::vector<Layer *> layers;
    Matrix Y;
    nr_ctx *ctx = nullptr;   // created on first use (device 0, like the reference)
    bool dirty = true;       // layers changed since the context was loaded
    int device = 0;

  public:
    NeuralNetwork();
    NeuralNetwork(std::string geomPath);
    ~NeuralNetwork();
    NeuralNetwork(const NeuralNetwork &) = delete;
    NeuralNetwork &operator=(const NeuralNetwork &) = delete;

    Matrix forward(Matrix X, int maxBatchSize = -1);
    void addLayer(Layer *layer);
    std::vector<Layer *> getLayers() const;

    int getNumWeightParams() const;
    int getNumBiasParams() const;

    bool load(std::string fp, bool hostOnly = false);

    // libnr context with this network loaded (fused path); nullptr on error
    nr_ctx *context();
};
