// matrix.hh -- host + device float buffer pair, HIP-backed.
// Same members and methods as the reference's Matrix (src/neuralUtils/matrix.hh:9-37,
// matrix.cu:12-72): shape.x = features, shape.y = batch; hostOnly skips the device copy.
#pragma once
#include <memory>

#include "shape.hh"

class Matrix {
  private:
    bool deviceAllocated;
    bool hostAllocated;
    bool hostOnly = false;

    void allocateDeviceMemory();
    void allocateHostMemory();

  public:
    Shape shape;

    std::shared_ptr<float> deviceData;
    std::shared_ptr<float> hostData;

    Matrix(size_t x_dim = 1, size_t y_dim = 1, bool hostOnly = false);
    Matrix(Shape shape, bool hostOnly = false);

    void allocateMemory();
    void maybeAllocateMemory(Shape shape);

    void copyHostToDevice();
    void copyDeviceToHost();

    int size() { return (int)(shape.x * shape.y); }

    float &operator[](const int index);
    const float &operator[](const int index) const;
};
