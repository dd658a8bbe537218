// neuralSDFRenderer -- headless restatement of the reference's src/main.cpp on libnr.
//
// Same flags (main.cpp:536-631), camera (updateViewMatrices :207-222), single-image
// and spin modes (:404-478), output naming (:445-461), PNG with the reference's
// 180-degree rotation, and the throughput printf (:436-437).  The GLUT interactive
// viewer (:480-519) needs a display and is not built; extra flags: --max-steps,
// --precision {fp32,bf16,fp16,fp32x3}, --scene {v1,tanh}, --ppm (also write a .ppm),
// --camera {eigen,f64}, --gpus N (each frame's row-band shards on N GPUs, one RCCL gather:
// nr_group_render_batch).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "neural_render.h"
#include "nr/image.hh"
#include "nr/neuralNetwork.hh"
#include "nr/volumeRender.hh"

static std::string neuralGeometryPath, renderSavePath, matcapPath;
static bool singleImage = false, doSpin = false, writePPM = false;
static unsigned width = 512, height = 512;
static int colorType = 0, numInputs = 3, frameNumber = 0;
static float rotX = 0, rotY = 0, zoom = 2.0f;
static unsigned saveCount = 0;

static NeuralNetwork nn;
static Image matcap;

struct dim3_ { unsigned x, y, z; };

// updateViewMatrices' arithmetic (--camera): f64 by default -- the reference's x86-64 build takes
// Eigen's SSE 4x4 inverse, whose last bits the scalar restatement (eigen) is not pinned to
static int cameraMode = NR_CAMERA_F64;
// --gpus N: every frame split into row-band shards over GPUs 0..N-1 of this process (one context
// per GPU, nr_group: one RCCL gather per frame); 0 = the reference's single-GPU render_kernel path
static int numGpus = 0;
static std::vector<nr_ctx *> groupCtx;
static nr_group *group = nullptr;

static char *getCmdOption(char **begin, char **end, const std::string &option) {
    char **itr = std::find(begin, end, option);
    if (itr != end && ++itr != end) return *itr;
    return nullptr;
}
static bool cmdOptionExists(char **begin, char **end, const std::string &option) {
    return std::find(begin, end, option) != end;
}

static void usage() {
    std::cout << "Usage: neuralSDFRenderer [OPTION]... -i SOURCE.h5 --single\n"
                 "Options\n"
                 "\t-i input neuralGeometry path (string) REQUIRED\n"
                 "\t-o output image prefix (string) default: {inputPath}\n"
                 "\t-H imageH (int)  -W imageW (int)\n"
                 "\t-M matcap file path (string)\n"
                 "\t-rx / -ry rotation in degree about x / y\n"
                 "\t-z zoom (default 2)\n"
                 "\t--single render one frame and save it\n"
                 "\t--spin render 360 frames rotating about y\n"
                 "\t--animation 4-input networks (frame number as 4th input)\n"
                 "\t--max-steps N (default 6000)  --precision fp32|bf16|fp16|fp32x3  --scene v1|tanh  --ppm\n"
                 "\t--camera f64|eigen (default f64: exact matrices rounded once; eigen: a restatement of Eigen's scalar float path, unpinned)\n"
                 "\t--gpus N split every frame into row-band shards over N GPUs (one RCCL gather per frame)\n";
}

static void parseCmdOptions(int argc, char **argv) {
    char **b = argv, **e = argv + argc;
    if (cmdOptionExists(b, e, "-h") || cmdOptionExists(b, e, "--help")) { usage(); exit(0); }
    if (!cmdOptionExists(b, e, "-i") || !getCmdOption(b, e, "-i")) { std::cerr << "You must give path to neuralGeometry\n"; exit(2); }
    neuralGeometryPath = getCmdOption(b, e, "-i");
    renderSavePath = getCmdOption(b, e, "-o") ? getCmdOption(b, e, "-o") : neuralGeometryPath;
    if (getCmdOption(b, e, "-H")) height = atoi(getCmdOption(b, e, "-H"));
    if (getCmdOption(b, e, "-W")) width = atoi(getCmdOption(b, e, "-W"));
    if (getCmdOption(b, e, "-M")) matcapPath = getCmdOption(b, e, "-M");
    if (getCmdOption(b, e, "-rx")) rotX = (float)atof(getCmdOption(b, e, "-rx"));
    if (getCmdOption(b, e, "-ry")) rotY = (float)atof(getCmdOption(b, e, "-ry"));
    if (getCmdOption(b, e, "-z")) zoom = (float)atof(getCmdOption(b, e, "-z"));
    doSpin = cmdOptionExists(b, e, "--spin");
    singleImage = cmdOptionExists(b, e, "--single");
    writePPM = cmdOptionExists(b, e, "--ppm");
    if (getCmdOption(b, e, "--camera")) cameraMode = std::string(getCmdOption(b, e, "--camera")) == "eigen" ? NR_CAMERA_EIGEN : NR_CAMERA_F64;
    if (cmdOptionExists(b, e, "--animation")) numInputs = 4;
    if (getCmdOption(b, e, "--gpus")) numGpus = std::max(0, atoi(getCmdOption(b, e, "--gpus")));
    if (getCmdOption(b, e, "--max-steps")) NR_MAX_STEPS = atoi(getCmdOption(b, e, "--max-steps"));
    if (getCmdOption(b, e, "--scene")) NR_SCENE_MODE = std::string(getCmdOption(b, e, "--scene")) == "tanh" ? NR_SCENE_TANH : NR_SCENE_V1;
    if (getCmdOption(b, e, "--precision")) {
        std::string p = getCmdOption(b, e, "--precision");
        NR_PRECISION_MODE = p == "bf16" ? NR_PRECISION_BF16
                            : p == "fp16" ? NR_PRECISION_FP16
                            : p == "fp32x3" ? NR_PRECISION_FP32X3 : NR_PRECISION_FP32;
    }
}

static int countDigit(unsigned n) {
    int c = 0;
    while (n != 0) { n /= 10; ++c; }
    return c;
}

static bool saveFrame(Image &out);

// One context per GPU with the same network and settings, joined into an nr_group.
static bool groupInit() {
    for (int d = 0; d < numGpus; ++d) {
        nr_ctx *c = nullptr;
        if (nr_create(d, &c) != NR_OK || nr_load_h5(c, neuralGeometryPath.c_str()) != NR_OK ||
            nr_set_precision(c, NR_PRECISION_MODE) != NR_OK || nr_set_scene(c, NR_SCENE_MODE) != NR_OK ||
            nr_set_static(c, colorType, numInputs) != NR_OK ||
            (colorType == NR_COLOR_MATCAP &&
             nr_set_matcap(c, matcap.hostData.get(), (int)matcap.shape.x, (int)matcap.shape.y) != NR_OK)) {
            printf("GPU %d: %s\n", d, nr_last_error(c));
            return false;
        }
        groupCtx.push_back(c);
    }
    if (nr_group_create(groupCtx.data(), numGpus, &group) != NR_OK) {
        printf("nr_group_create: %s\n", nr_last_error(nullptr));
        return false;
    }
    return true;
}

static bool generateSingleImage() {
    if (numGpus > 0) {  // the frame across numGpus GPUs
        if (!group && !groupInit()) return false;
        nr_frame f{};
        nr_camera_ex(rotX, rotY, zoom, 0.0f, 0.0f, cameraMode, f.inv_view, f.normal);
        f.frame = frameNumber;
        Image out(width, height, true);
        out.allocateMemory();
        f.out = out.hostData.get();
        auto t0 = std::chrono::steady_clock::now();
        if (nr_group_render_batch(group, &f, 1, (int)width, (int)height, 1, NR_MAX_STEPS, NR_HOST, nullptr) != NR_OK) {
            printf("nr_group_render_batch: %s\n", nr_last_error(nullptr));
            return false;
        }
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (saveCount == 0)
            printf("volumeRender, Throughput = %.4f MTexels/s, Time = %.5f s, Size = %u Texels, NumDevsUsed = %d, "
                   "Workgroup = %u\n",
                   (1.0e-6 * width * height) / dt, dt, width * height, numGpus, 256u);
        return saveFrame(out);
    }
    unsigned *d_output = nullptr;
    if (hipMalloc(&d_output, (size_t)width * height * sizeof(unsigned)) != hipSuccess) return false;
    (void)hipMemset(d_output, 0, (size_t)width * height * sizeof(unsigned));
    float invView[12], normal[16];
    nr_camera_ex(rotX, rotY, zoom, 0.0f, 0.0f, cameraMode, invView, normal);  // updateViewMatrices
    copyViewMatrices(invView, sizeof invView, normal, sizeof normal, frameNumber);
    (void)hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    dim3_ block{8, 8, 1}, grid{(width + 7) / 8, (height + 7) / 8, 1};
    render_kernel(grid, block, d_output, width, height, (unsigned)numInputs, nn, matcap);
    (void)hipDeviceSynchronize();
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (saveCount == 0)
        printf("volumeRender, Throughput = %.4f MTexels/s, Time = %.5f s, Size = %u Texels, NumDevsUsed = %u, "
               "Workgroup = %u\n",
               (1.0e-6 * width * height) / dt, dt, width * height, 1u, 256u);
    Image out(width, height, true);
    out.allocateMemory();
    (void)hipMemcpy(out.hostData.get(), d_output, (size_t)width * height * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_output);
    return saveFrame(out);
}

// main.cpp:445-461: the frame's file name and PNG (+ PPM)
static bool saveFrame(Image &out) {
    std::string ext;
    if (!singleImage) {
        if (countDigit(saveCount) < 2) ext += "00";
        else if (countDigit(saveCount) == 2) ext += "0";
        ext += std::to_string(saveCount) + ".png";
    } else {
        std::string base = neuralGeometryPath.substr(neuralGeometryPath.find_last_of("/\\") + 1);
        ext = base + ".png";
    }
    std::cout << "saving frame: " << renderSavePath + ext << std::endl;
    bool ok = out.savePNG(renderSavePath + ext);
    if (writePPM) ok = out.savePPM(renderSavePath + ext + ".ppm") && ok;
    ++saveCount;
    return ok;
}

int main(int argc, char **argv) {
    parseCmdOptions(argc, argv);
    if (!nn.load(neuralGeometryPath)) {
        printf("Failed to initialize model (%s)... exiting \n", neuralGeometryPath.c_str());
        return 1;
    }
    printf("Model initialized...\n\n");
    if (!matcapPath.empty()) {
        if (!matcap.loadPNG(matcapPath)) {
            printf("Failed to load matcap file (%s)... exiting \n", matcapPath.c_str());
            return 1;
        }
        colorType = 1;
    }
    copyStaticSettings(colorType, numInputs);
    if (singleImage) return generateSingleImage() ? 0 : 1;
    if (doSpin) {
        for (int i = 0; i < 360; ++i) {  // doABarrelRoll (main.cpp:470-478)
            rotY = (float)i;
            frameNumber = i;
            if (!generateSingleImage()) return 1;
        }
        return 0;
    }
    std::cerr << "interactive GLUT viewer is not part of the headless MI355X build; use --single or --spin\n";
    return 2;
}
