// shape.hh -- Shape (reference src/neuralUtils/shape.hh:3-7).
#pragma once
#include <cstddef>

struct Shape {
    size_t x, y;
    Shape(size_t x = 1, size_t y = 1) : x(x), y(y) {}
};
