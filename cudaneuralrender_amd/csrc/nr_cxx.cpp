// nr_cxx.cpp -- the reference's C++ host API (Matrix, Image, DenseLayer, NeuralNetwork,
// render_kernel, copyViewMatrices, copyStaticSettings) implemented over libnr's C ABI and
// the HIP runtime, so main.cpp / simpleInfer.cpp-style drivers build against
// include/nr/*.hh with include-path changes only.
//
// Reference: src/neuralUtils/{matrix,image}.cu, src/layers/denseLayer.cu:180-278,
// src/neuralNetwork.cpp:36-151, src/volumeRender_kernel.cu:608-706.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstring>
#include <iostream>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/nr/denseLayer.hh"
#include "../../include/nr/image.hh"
#include "../../include/nr/matrix.hh"
#include "../../include/nr/neuralNetwork.hh"
#include "../../include/nr/volumeRender.hh"
#include "nr_internal.h"

// ------------------------------------------------------------------ helpers
namespace {
bool hipok(hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    fprintf(stderr, "[nr] %s: %s\n", what, hipGetErrorString(e));
    return false;
}

// Context for layer-level work that does not belong to a loaded network.
nr_ctx *default_ctx() {
    static std::once_flag once;
    static nr_ctx *ctx = nullptr;
    std::call_once(once, [] {
        if (nr_create(0, &ctx) != NR_OK) {
            fprintf(stderr, "[nr] %s\n", nr_last_error(nullptr));
            ctx = nullptr;
        }
    });
    return ctx;
}

struct ViewState {
    float inv_view[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 2};
    float normal[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -2, 0, 0, 0, 1};
    int frame = 0, color_type = 0, num_inputs = 3;
} g_view;
}  // namespace

int NR_MAX_STEPS = 6000;
int NR_SCENE_MODE = NR_SCENE_V1;
int NR_PRECISION_MODE = NR_PRECISION_FP32;

// ------------------------------------------------------------------ Matrix
Matrix::Matrix(size_t x_dim, size_t y_dim, bool hostOnly)
    : deviceAllocated(false), hostAllocated(false), hostOnly(hostOnly), shape(x_dim, y_dim) {}
Matrix::Matrix(Shape shape, bool hostOnly) : Matrix(shape.x, shape.y, hostOnly) {}

void Matrix::allocateDeviceMemory() {
    if (deviceAllocated) return;
    float *p = nullptr;
    if (!hipok(hipMalloc(&p, shape.x * shape.y * sizeof(float)), "Matrix hipMalloc")) return;
    deviceData = std::shared_ptr<float>(p, [](float *q) { (void)hipFree(q); });
    deviceAllocated = true;
}
void Matrix::allocateHostMemory() {
    if (hostAllocated) return;
    hostData = std::shared_ptr<float>(new float[shape.x * shape.y], [](float *q) { delete[] q; });
    hostAllocated = true;
}
void Matrix::allocateMemory() {
    allocateHostMemory();
    if (!hostOnly) allocateDeviceMemory();
}
void Matrix::maybeAllocateMemory(Shape s) {
    if (!deviceAllocated && !hostAllocated) {
        shape = s;
        allocateMemory();
    }
}
void Matrix::copyHostToDevice() {
    if (deviceAllocated && hostAllocated)
        hipok(hipMemcpy(deviceData.get(), hostData.get(), shape.x * shape.y * sizeof(float), hipMemcpyHostToDevice),
              "Matrix H2D");
    else
        printf("Failed to copy from host to device... nothing initialized\n");
}
void Matrix::copyDeviceToHost() {
    if (deviceAllocated && hostAllocated)
        hipok(hipMemcpy(hostData.get(), deviceData.get(), shape.x * shape.y * sizeof(float), hipMemcpyDeviceToHost),
              "Matrix D2H");
    else
        printf("Failed to copy from device to host... nothing initialized\n");
}
float &Matrix::operator[](const int i) { return hostData.get()[i]; }
const float &Matrix::operator[](const int i) const { return hostData.get()[i]; }

// ------------------------------------------------------------------ Image
Image::Image(size_t x_dim, size_t y_dim, bool hostOnly)
    : deviceAllocated(false), hostAllocated(false), hostOnly(hostOnly), shape(x_dim, y_dim) {}
Image::Image(Shape shape, bool hostOnly) : Image(shape.x, shape.y, hostOnly) {}

void Image::allocateDeviceMemory() {
    if (deviceAllocated) return;
    uint *p = nullptr;
    if (!hipok(hipMalloc(&p, shape.x * shape.y * sizeof(uint)), "Image hipMalloc")) return;
    deviceData = std::shared_ptr<uint>(p, [](uint *q) { (void)hipFree(q); });
    deviceAllocated = true;
}
void Image::allocateHostMemory() {
    if (hostAllocated) return;
    hostData = std::shared_ptr<uint>(new uint[shape.x * shape.y], [](uint *q) { delete[] q; });
    hostAllocated = true;
}
void Image::allocateMemory() {
    allocateHostMemory();
    if (!hostOnly) allocateDeviceMemory();
}
void Image::maybeAllocateMemory(Shape s) {
    if (!deviceAllocated && !hostAllocated) {
        shape = s;
        allocateMemory();
    }
}
bool Image::loadPNG(std::string filename) {
    std::vector<uint32_t> px;
    int w = 0, h = 0;
    std::string err;
    if (nr::png_decode(filename.c_str(), px, w, h, err) != NR_OK) {
        std::cout << "Error reading png: " << err << std::endl;
        return false;
    }
    maybeAllocateMemory(Shape((size_t)w, (size_t)h));
    if (shape.x * shape.y != px.size()) {
        std::cout << "Error reading png: image size does not match the allocated Image" << std::endl;
        return false;
    }
    memcpy(hostData.get(), px.data(), px.size() * 4);
    if (!hostOnly) copyHostToDevice();
    return true;
}
bool Image::savePNG(std::string filename, bool doFlip, bool) {
    if (!hostAllocated) {
        std::cout << "[ERROR] no data to save...\n";
        return false;
    }
    std::string err;
    if (nr::png_encode(filename.c_str(), hostData.get(), (int)shape.x, (int)shape.y, doFlip ? 1 : 0, err) != NR_OK) {
        std::cout << "[ERROR] Unable to save png: " << err << std::endl;
        return false;
    }
    return true;
}
bool Image::savePPM(std::string filename) {
    if (!hostAllocated) return false;
    std::string err;
    return nr::ppm_encode(filename.c_str(), hostData.get(), (int)shape.x, (int)shape.y, err) == NR_OK;
}
void Image::copyHostToDevice() {
    if (deviceAllocated && hostAllocated)
        hipok(hipMemcpy(deviceData.get(), hostData.get(), shape.x * shape.y * sizeof(uint), hipMemcpyHostToDevice),
              "Image H2D");
    else
        printf("Failed to copy from host to device... nothing initialized\n");
}
void Image::copyDeviceToHost() {
    if (deviceAllocated && hostAllocated)
        hipok(hipMemcpy(hostData.get(), deviceData.get(), shape.x * shape.y * sizeof(uint), hipMemcpyDeviceToHost),
              "Image D2H");
    else
        printf("Failed to copy from device to host... nothing initialized\n");
}
uint &Image::operator[](const int i) { return hostData.get()[i]; }
const uint &Image::operator[](const int i) const { return hostData.get()[i]; }

// ------------------------------------------------------------------ DenseLayer
DenseLayer::DenseLayer(std::string name, std::vector<std::vector<float>> weights, std::vector<float> biases,
                       int activation, bool hostOnly) {
    this->W = Matrix(Shape(weights.size(), weights.empty() ? 0 : weights[0].size()), hostOnly);
    this->numWeightParams = (int)(W.shape.x * W.shape.y);
    this->b = Matrix(Shape(biases.size(), 1), hostOnly);
    this->numBiasParams = (int)biases.size();
    this->name = name;
    this->type = eDense;
    this->hostOnly = hostOnly;
    b.allocateMemory();
    W.allocateMemory();
    initializeBias(biases);
    initializeWeights(weights);
    this->activation = activation;
}
DenseLayer::~DenseLayer() {}

void DenseLayer::initializeBias(std::vector<float> biases) {
    for (size_t x = 0; x < biases.size(); ++x) b[(int)x] = biases[x];
    if (!hostOnly) b.copyHostToDevice();
}
void DenseLayer::initializeWeights(std::vector<std::vector<float>> weights) {
    for (size_t x = 0; x < weights.size(); ++x)
        for (size_t y = 0; y < weights[0].size(); ++y) W[(int)(y * W.shape.x + x)] = weights[x][y];  // out-major
    if (!hostOnly) W.copyHostToDevice();
}

Matrix &DenseLayer::forward(Matrix &Ain, int maxBatchSize) {
    this->A = Ain;
    size_t need = maxBatchSize == -1 ? Ain.shape.y : (size_t)maxBatchSize;
    if (need < Ain.shape.y) need = Ain.shape.y;
    // the reference keeps the first capacity forever (quirk Q12); grow when needed
    if (Z.deviceData && Z.shape.x == W.shape.y && Z.shape.y >= need) {
    } else {
        Z = Matrix(Shape(W.shape.y, need), false);
        Z.allocateMemory();
    }
    nr_ctx *c = default_ctx();
    if (!c || nr_dense_forward(c, W.deviceData.get(), b.deviceData.get(), (int)W.shape.x, (int)W.shape.y,
                               activation == ReLU ? 1 : 0, Ain.deviceData.get(), Z.deviceData.get(),
                               (long)Ain.shape.y, NR_DEVICE) != NR_OK ||
        nr_synchronize(c) != NR_OK)
        fprintf(stderr, "[nr] DenseLayer::forward failed: %s\n", nr_last_error(c));
    Z.shape.y = Ain.shape.y;
    return Z;
}

int DenseLayer::getXDim() const { return (int)W.shape.x; }
int DenseLayer::getYDim() const { return (int)W.shape.y; }
Matrix DenseLayer::getWeightsMatrix() const { return W; }
Matrix DenseLayer::getBiasVector() const { return b; }

// ------------------------------------------------------------------ NeuralNetwork
NeuralNetwork::NeuralNetwork() {}
NeuralNetwork::NeuralNetwork(std::string geomPath) {
    if (!load(geomPath, false)) std::cerr << "[ERROR]: failed to load model: " << geomPath;
}
NeuralNetwork::~NeuralNetwork() {
    for (auto layer : layers) delete layer;
    if (ctx) nr_destroy(ctx);
}
void NeuralNetwork::addLayer(Layer *layer) {
    layers.push_back(layer);
    dirty = true;
}
std::vector<Layer *> NeuralNetwork::getLayers() const { return layers; }
int NeuralNetwork::getNumWeightParams() const {
    int n = 0;
    for (auto l : layers) n += l->getNumWeightParams();
    return n;
}
int NeuralNetwork::getNumBiasParams() const {
    int n = 0;
    for (auto l : layers) n += l->getNumBiasParams();
    return n;
}

bool NeuralNetwork::load(std::string fp, bool hostOnly) {
    std::vector<int> dims;
    std::vector<std::vector<float>> K, B;
    std::string err;
    if (nr::h5_read_keras(fp.c_str(), dims, K, B, err) != NR_OK) {
        std::cout << err << "\n";
        return false;
    }
    int nl = (int)K.size();
    for (int l = 0; l < nl; ++l) {
        int in = dims[l], out = dims[l + 1];
        std::vector<std::vector<float>> w(in, std::vector<float>(out));
        for (int x = 0; x < in; ++x)
            for (int y = 0; y < out; ++y) w[x][y] = K[l][(size_t)x * out + y];
        addLayer(new DenseLayer(std::string("Dense_") + std::to_string(l), w, B[l], l == nl - 1 ? Tanh : ReLU,
                                hostOnly));
    }
    return true;
}

nr_ctx *NeuralNetwork::context() {
    if (!ctx && nr_create(device, &ctx) != NR_OK) {
        fprintf(stderr, "[nr] %s\n", nr_last_error(nullptr));
        ctx = nullptr;
        return nullptr;
    }
    if (dirty) {
        std::vector<int> dims;
        std::vector<std::vector<float>> K, B;
        for (auto l : layers) {
            auto *d = dynamic_cast<DenseLayer *>(l);
            if (!d) {
                fprintf(stderr, "[nr] only DenseLayer networks are supported\n");
                return nullptr;
            }
            Matrix W = d->getWeightsMatrix(), b = d->getBiasVector();
            int in = d->getXDim(), out = d->getYDim();
            if (dims.empty()) dims.push_back(in);
            dims.push_back(out);
            std::vector<float> k((size_t)in * out);
            for (int x = 0; x < in; ++x)
                for (int y = 0; y < out; ++y) k[(size_t)x * out + y] = W[y * in + x];  // back to Keras (in, out)
            K.push_back(k);
            B.push_back(std::vector<float>(b.hostData.get(), b.hostData.get() + out));
        }
        std::vector<const float *> kp, bp;
        for (size_t i = 0; i < K.size(); ++i) { kp.push_back(K[i].data()); bp.push_back(B[i].data()); }
        if (nr_load_mlp(ctx, (int)K.size(), dims.data(), kp.data(), bp.data()) != NR_OK) {
            fprintf(stderr, "[nr] %s\n", nr_last_error(ctx));
            return nullptr;
        }
        dirty = false;
    }
    return ctx;
}

Matrix NeuralNetwork::forward(Matrix X, int maxBatchSize) {
    (void)maxBatchSize;
    nr_ctx *c = context();
    int nl = 0, dims[64];
    if (c) nr_mlp_info(c, &nl, nullptr, nullptr, nullptr);
    if (c && nl > 0 && nl < 63) {
        nr_mlp_info(c, &nl, dims, nullptr, nullptr);
        Y = Matrix(Shape(dims[nl], X.shape.y));
        Y.allocateMemory();
        if (nr_mlp_forward(c, X.deviceData.get(), Y.deviceData.get(), (long)X.shape.y, NR_DEVICE) != NR_OK ||
            nr_synchronize(c) != NR_OK)
            fprintf(stderr, "[nr] NeuralNetwork::forward failed: %s\n", nr_last_error(c));
        return Y;
    }
    Matrix Z = X;  // layer by layer (neuralNetwork.cpp:54-63)
    for (auto layer : layers) Z = layer->forward(Z, maxBatchSize);
    Y = Z;
    return Y;
}

// ------------------------------------------------------------------ render entry points
extern "C" void copyViewMatrices(float *invViewMatrix, size_t sizeofViewMatrix, float *normalMatrix,
                                 size_t sizeofNormalMatrix, int frameNumber) {
    memcpy(g_view.inv_view, invViewMatrix, std::min(sizeofViewMatrix, sizeof g_view.inv_view));
    memcpy(g_view.normal, normalMatrix, std::min(sizeofNormalMatrix, sizeof g_view.normal));
    g_view.frame = frameNumber;
}

extern "C" void copyStaticSettings(int colorType, int numInputs) {
    g_view.color_type = colorType;
    g_view.num_inputs = numInputs;
}

void render_kernel_nr(unsigned *d_output, unsigned imageW, unsigned imageH, unsigned numInputs, NeuralNetwork &nn,
                      const Image &matcap) {
    nr_ctx *c = nn.context();
    if (!c) return;
    (void)numInputs;  // copyStaticSettings carries it, as c_numInputs does in the reference
    int rc = nr_set_view(c, g_view.inv_view, g_view.normal, g_view.frame);
    if (rc == NR_OK) rc = nr_set_static(c, g_view.color_type, g_view.num_inputs);
    if (rc == NR_OK) rc = nr_set_scene(c, NR_SCENE_MODE);
    if (rc == NR_OK) rc = nr_set_precision(c, NR_PRECISION_MODE);
    if (rc == NR_OK && g_view.color_type == NR_COLOR_MATCAP) {
        static const void *last = nullptr;
        static const nr_ctx *last_ctx = nullptr;
        static size_t last_n = 0;
        const uint *host = matcap.hostData.get();
        size_t n = matcap.shape.x * matcap.shape.y;
        if (host && (host != last || n != last_n || c != last_ctx)) {
            rc = nr_set_matcap(c, host, (int)matcap.shape.x, (int)matcap.shape.y);
            last = host;
            last_n = n;
            last_ctx = c;
        }
    }
    if (rc == NR_OK) rc = nr_render(c, d_output, (int)imageW, (int)imageH, NR_MAX_STEPS, NR_DEVICE, nullptr);
    if (rc == NR_OK) rc = nr_synchronize(c);
    if (rc != NR_OK) fprintf(stderr, "[nr] render_kernel failed: %s\n", nr_last_error(c));
}
