// highfive_load.cpp -- the reference's HighFive weight loader, restated for this repo's test
// suite, compiled against include/highfive (the read-only HighFive subset over libnr).
//
// loadModelFromH5 below walks the file with exactly the HighFive calls of the reference's
// simpleInfer.cpp:13-79 / NeuralNetwork::load (neuralNetwork.cpp:86-129): File(fp,
// File::ReadOnly), listObjectNames, getObjectType, getGroup, getNumberObjects, the inner
// getGroup(same name), getDataSet, getDimensions, read(biases) / read(weights), and builds
// host-only DenseLayers (ReLU, the last one Tanh).  main() then prints every layer as
// "name in out" followed by its kernel (Keras in x out order) and bias as hex floats, which
// tests/test_highfive.py compares with h5py's reading (tests/golden/weights_h5py.npz).
// usage: highfive_load model.h5
#include <highfive/H5DataSet.hpp>
#include <highfive/H5DataSpace.hpp>
#include <highfive/H5File.hpp>

#include <cstdio>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "nr/denseLayer.hh"
#include "nr/neuralNetwork.hh"

static bool loadModelFromH5(const std::string &fp, NeuralNetwork &nn, bool hostOnly) {
    HighFive::File file(fp, HighFive::File::ReadOnly);
    const std::vector<std::string> layerNames = file.listObjectNames();
    int index = 0;
    for (auto it = layerNames.begin(); it != layerNames.end(); ++it) {
        if (file.getObjectType(*it) != HighFive::ObjectType::Group) {
            std::cout << "Unsupported Layer\n";
            return false;
        }
        HighFive::Group outer = file.getGroup(*it);
        if (outer.getNumberObjects() != 1) {
            std::cout << "Unsupported Layer\n";
            return false;
        }
        HighFive::Group group = outer;
        group = group.getGroup(*it);  // Keras nests <name>/<name>/{bias:0, kernel:0}
        std::vector<std::vector<float>> weights;
        std::vector<float> biases;
        for (const std::string &m : group.listObjectNames()) {
            if (group.getObjectType(m) != HighFive::ObjectType::Dataset) {
                std::cout << "Unsupported Layer\n";
                return false;
            }
            HighFive::DataSet ds = group.getDataSet(m);
            const std::vector<size_t> dim = ds.getDimensions();
            if (dim.size() == 1) ds.read(biases);
            else if (dim.size() == 2) ds.read(weights);
            else {
                std::cout << "Unsupported layer, to many dims!\n";
                return false;
            }
        }
        const int act = std::next(it) == layerNames.end() ? Tanh : ReLU;
        nn.addLayer(new DenseLayer("Dense_" + std::to_string(index), weights, biases, act, hostOnly));
        ++index;
    }
    return true;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s model.h5\n", argv[0]);
        return 2;
    }
    NeuralNetwork nn;
    try {
        if (!loadModelFromH5(argv[1], nn, true)) return 1;
    } catch (const HighFive::Exception &e) {
        printf("HighFive error: %s\n", e.what());
        return 3;
    }
    const std::vector<Layer *> layers = nn.getLayers();
    printf("layers %zu weights %d biases %d\n", layers.size(), nn.getNumWeightParams(), nn.getNumBiasParams());
    for (Layer *l : layers) {
        DenseLayer *d = static_cast<DenseLayer *>(l);
        const int in = d->getXDim(), out = d->getYDim();
        Matrix W = d->getWeightsMatrix(), b = d->getBiasVector();
        printf("%s %d %d %s\n", l->getName().c_str(), in, out, d->getActivation() == Tanh ? "tanh" : "relu");
        for (int x = 0; x < in; ++x)  // Keras order: kernel[x][y] = W[y * in + x] (out-major)
            for (int y = 0; y < out; ++y) printf("%a%c", W[y * in + x], y + 1 == out ? '\n' : ' ');
        for (int y = 0; y < out; ++y) printf("%a%c", b[y], y + 1 == out ? '\n' : ' ');
    }
    return 0;
}
