// parser_sanitize.cpp -- host-side driver for the AddressSanitizer / UndefinedBehaviorSanitizer build
// of the untrusted-input parsers (csrc/h5_keras.cpp: the Keras HDF5 reader; csrc/png_codec.cpp: the
// PNG decoder) and of the CPU oracle (oracle/nr_oracle.c), built and run by
// tests/test_sanitizers_cpu.py with g++/gcc -fsanitize=address,undefined.
//
//   parser_sanitize h5 FILE...    read every file as a Keras .h5 (nr::h5_read_keras); a malformed
//                                 file must fail with an error message, never touch memory it
//                                 does not own
//   parser_sanitize png FILE...   the same for nr::png_decode
//   parser_sanitize oracle H5     the oracle's MLP (every precision) on ordinary and non-finite
//                                 inputs and a small render of every scene, with that network
// Prints "ok N failed M" per mode; the sanitizers abort on the first finding (exit status != 0).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "nr_internal.h"

// nr_api.hip is not part of this build: its error recorder, as a plain formatter
int nr::report_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return code;
}

extern "C" {
int or_mlp_forward(int nlayers, const int *dims, const float *params, const float *X, long n, int in_stride, float *Y,
                   int precision, int nthreads);
int or_render_ex(int nlayers, const int *dims, const float *params, const float *inv_view, const float *normal,
                 int frame, int color_type, int num_inputs, int scene, const uint32_t *matcap, int mw, int mh, int W,
                 int H, int max_steps, uint32_t *out, long long *stats, int nthreads, int precision, int y0, int y1);
}

static int run_oracle(const char *path) {
    std::vector<int> dims;
    std::vector<std::vector<float>> K, B;
    std::string err;
    if (nr::h5_read_keras(path, dims, K, B, err) != NR_OK) {
        fprintf(stderr, "%s: %s\n", path, err.c_str());
        return 1;
    }
    const int nl = (int)dims.size() - 1;
    std::vector<float> params;
    for (int l = 0; l < nl; ++l) {
        params.insert(params.end(), K[l].begin(), K[l].end());
        params.insert(params.end(), B[l].begin(), B[l].end());
    }
    const float inf = INFINITY, nan = NAN;
    std::vector<float> X = {0, 0, 0, 0.1f, 0.2f, 0.3f, 1e30f, -1e30f, 0, inf, 0, 0, nan, 1, 1, -0.0f, 1e-40f, 2};
    std::vector<float> Y(X.size() / 3);
    for (int prec = 0; prec <= 3; ++prec)
        if (or_mlp_forward(nl, dims.data(), params.data(), X.data(), (long)Y.size(), 3, Y.data(), prec, 2) != 0) {
            fprintf(stderr, "or_mlp_forward precision %d failed\n", prec);
            return 1;
        }
    const float iv[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 2};
    const float nm[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -2, 0, 0, 0, 1};
    std::vector<uint32_t> matcap(16 * 16, 0xff804020u), out(24 * 20);
    long long stats[5];
    for (int scene = 0; scene < 6; ++scene)
        for (int color = 0; color < 2; ++color)
            if (or_render_ex(nl, dims.data(), params.data(), iv, nm, 7, color, 3, scene, matcap.data(), 16, 16, 24, 20, 64,
                             out.data(), stats, 2, scene == 0 ? 3 : 0, 0, 20) != 0) {
                fprintf(stderr, "or_render_ex scene %d failed\n", scene);
                return 1;
            }
    printf("oracle ok\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s h5|png|oracle FILE...\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "oracle") return run_oracle(argv[2]);
    int ok = 0, failed = 0;
    for (int i = 2; i < argc; ++i) {
        std::string err;
        int rc;
        if (mode == "h5") {
            std::vector<int> dims;
            std::vector<std::vector<float>> K, B;
            rc = nr::h5_read_keras(argv[i], dims, K, B, err);
        } else {
            std::vector<uint32_t> rgba;
            int w = 0, h = 0;
            rc = nr::png_decode(argv[i], rgba, w, h, err);
            if (rc == NR_OK && rgba.size() != (size_t)w * h) {
                fprintf(stderr, "%s: %zu pixels for %dx%d\n", argv[i], rgba.size(), w, h);
                return 1;
            }
        }
        if (rc == NR_OK) ++ok;
        else if (err.empty()) {
            fprintf(stderr, "%s: failed without a message\n", argv[i]);
            return 1;
        } else ++failed;
    }
    printf("%s ok %d failed %d\n", mode.c_str(), ok, failed);
    return 0;
}
