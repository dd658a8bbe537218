// denseLayer.hh -- fully connected layer on the MI355X (reference src/layers/denseLayer.hh).
// Same constructor and accessors; forward runs the gfx950 dense kernel of libnr
// (fmaf chain over the inputs + bias, ReLU unless the layer is tagged Tanh -- the
// reference computes the Tanh-tagged last layer as LINEAR, denseLayer.cu:150-166).
#pragma once
#include <string>
#include <vector>

#include "layer.hh"

enum Activation { ReLU, Tanh };

class DenseLayer : public Layer {
  private:
    Matrix W;  // out-major: W[y * in + x] = weights[x][y]  (denseLayer.cu:217-227)
    Matrix b;
    Matrix A;
    Matrix Z;

    int activation;
    bool hostOnly = false;

    void initializeWeights(std::vector<std::vector<float>> weights);
    void initializeBias(std::vector<float> biases);

  public:
    DenseLayer(std::string name, std::vector<std::vector<float>> weights, std::vector<float> biases, int activation,
               bool hostOnly = false);
    ~DenseLayer();

    Matrix &forward(Matrix &A, int maxBatchSize = -1);

    int getXDim() const;
    int getYDim() const;
    int getActivation() const { return activation; }
    Matrix getWeightsMatrix() const;
    Matrix getBiasVector() const;
};
