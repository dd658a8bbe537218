// simpleInfer -- restatement of the reference's src/simpleInfer.cpp on libnr:
// batchTest(1e6) (:112-147) pushes 1,000,000 identical zero inputs through
// NeuralNetwork::forward and checks every output equals the first; singleTest (:81-110)
// prints the network output for (0.1, 0.2, 0.3).  Timing is wall clock (the reference
// used std::clock, i.e. CPU time).  usage: simpleInfer [model.h5] [batch]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>

#include "nr/neuralNetwork.hh"

static bool singleTest(const std::string &path) {
    NeuralNetwork nn;
    if (!nn.load(path, false)) return false;
    printf("Testing single inference\n");
    Matrix X = Matrix(Shape(3, 1));
    X.allocateMemory();
    X[0] = 0.1f; X[1] = 0.2f; X[2] = 0.3f;
    X.copyHostToDevice();
    Matrix Y = nn.forward(X);
    Y.copyDeviceToHost();
    printf("(%f %f %f): %f \n", X[0], X[1], X[2], tanh(Y[0]));
    return true;
}

static bool batchTest(const std::string &path, int batchSize, bool doVerify) {
    NeuralNetwork nn;
    if (!nn.load(path, false)) return false;
    printf("\n\nTesting Batched inference (Batchsize: %d)\n\n", batchSize);
    Matrix X = Matrix(Shape(3, batchSize));
    X.allocateMemory();
    for (int i = 0; i < batchSize * 3; ++i) X[i] = 0.0f;
    X.copyHostToDevice();
    Matrix Y = nn.forward(X);  // first call builds the packed weights
    auto t0 = std::chrono::steady_clock::now();
    Y = nn.forward(X);
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::cout << "Took: " << ms << " ms for " << batchSize << " inferences\n";
    if (doVerify) {
        printf("Checking for errors...\n");
        Y.copyDeviceToHost();
        float first = Y[0];
        for (int i = 1; i < (int)Y.shape.y; ++i)
            if (Y[i] != first) {
                printf("ERROR: %f\n", Y[i]);
                return false;
            }
        printf("Woah there aren't any!! All evaluated (%f,%f,%f):%f\n", X[0], X[1], X[2], Y[0]);
    }
    return true;
}

int main(int argc, char **argv) {
    std::string path = argc > 1 ? argv[1] : "model.h5";
    int batch = argc > 2 ? atoi(argv[2]) : 1000000;
    if (!singleTest(path)) return 1;
    return batchTest(path, batch, true) ? 0 : 1;
}
