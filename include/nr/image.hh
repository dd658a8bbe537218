// image.hh -- packed RGBA (a<<24|b<<16|g<<8|r) host + device image, HIP-backed.
// Same API as the reference's Image (src/neuralUtils/image.hh:12-43, image.cu:36-110).
#pragma once
#include <memory>
#include <string>

#include "shape.hh"

typedef unsigned int uint;

class Image {
  private:
    bool deviceAllocated;
    bool hostAllocated;
    bool hostOnly = false;

    void allocateDeviceMemory();
    void allocateHostMemory();

  public:
    Shape shape;

    std::shared_ptr<uint> deviceData;
    std::shared_ptr<uint> hostData;

    Image(size_t x_dim = 1, size_t y_dim = 1, bool hostOnly = false);
    Image(Shape shape, bool hostOnly = false);

    void allocateMemory();
    void maybeAllocateMemory(Shape shape);

    // decode to packed RGBA and upload (image.cu:36-65); false + message on error
    bool loadPNG(std::string filename);
    // doFlip reproduces the reference's 180-degree rotation (image.cu:84-98, quirk Q9)
    bool savePNG(std::string filename, bool doFlip = true, bool doMirror = true);
    // sdkSavePPM4ub-style P6, buffer row 0 first (format of neuralGeometries/*.h5.ppm)
    bool savePPM(std::string filename);

    void copyHostToDevice();
    void copyDeviceToHost();

    int size() { return (int)(shape.x * shape.y); }

    uint &operator[](const int index);
    const uint &operator[](const int index) const;
};
