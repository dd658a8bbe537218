// layer.hh -- abstract layer (reference src/layers/layer.hh:11-27).
#pragma once
#include <string>

#include "matrix.hh"

enum LayerType { eDense };

class Layer {
  protected:
    std::string name;
    int type = -1;
    int numBiasParams = 0;
    int numWeightParams = 0;

  public:
    virtual ~Layer() = 0;
    virtual Matrix &forward(Matrix &A, int maxBatchSize = -1) = 0;

    std::string getName() { return this->name; }
    int getType() { return this->type; }
    int getNumWeightParams() { return this->numWeightParams; }
    int getNumBiasParams() { return this->numBiasParams; }
};

inline Layer::~Layer() {}
