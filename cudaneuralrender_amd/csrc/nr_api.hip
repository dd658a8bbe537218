// nr_api.hip -- the C ABI of libnr.so (include/neural_render.h): contexts, buffers,
// the render loop driver and the host helpers.
//
// Replaces, on the reference side (daviesthomas/cudaNeuralRender @ v1):
//   render_kernel / copyViewMatrices / copyStaticSettings  src/volumeRender_kernel.cu:608-706
//   allocateBuffers + the static scratch globals           :578-606
//   NeuralNetwork::load / forward                          src/neuralNetwork.cpp:54-151
//   DenseLayer ctor / forward                              src/layers/denseLayer.cu:180-278
//   Image::loadPNG / savePNG                               src/neuralUtils/image.cu:36-110
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "nr_internal.h"

constexpr int NR_MAX_QUEUES = 64;
#include "nr_kernels.h"

using namespace nr;

struct nr_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr, stream = nullptr;
    bool use_own = true;  // stream = own_stream, created lazily: a context driven on a
                          // caller's stream never takes a hardware queue of its own
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;

    // network
    std::vector<int> dims;
    std::vector<std::vector<float>> kernels, biases;  // Keras (in x out), bias
    std::vector<float *> d_W, d_b;                     // out-major per layer (generic kernel)
    bool fused = false;
    int precision = NR_PRECISION_FP32;
    float *d_pack16 = nullptr;
    uint16_t *d_lp16 = nullptr;
    uint16_t *d_x3lp = nullptr;  // bf16/fp16: the fp32x3 pack for the normals (MlpArgs::x3n)
    float *d_x3fl = nullptr;
    int x3lp_bytes = 0, x3fl_bytes = 0;  // its sizes (TraceArgs: the EG instances stage it in LDS)
    bool fp32_normals = false;   // nr_set_debug bit 15: the bf16/fp16 tracers' normals in fp32 (A/B)
    float eg_tau = NR_ENDGAME_DEFAULT;  // nr_set_endgame: bf16/fp16 persistent renders' fp32x3 endgame
    float *d_lpf16 = nullptr;
    uint16_t *d_lps16 = nullptr;  // the 16x16x32 layout of d_lp16 / d_lpf16 (k_mlp16, 7 hidden layers)
    float *d_lpfs16 = nullptr;
    bool no_s16 = true;           // nr_set_debug bit 12 clear: k_mlp16 on the 32x32x16 stream (the
                                  // default; the 16x16x32 one measured 3-5 % slower, round 6)
    MlpArgs mlp16{};  // 16-point-tile packs: k_trace, k_mlp16, k_march16, k_shade16
    bool clamp_ok = false;  // the bf16 pack is scaled for the clamped ReLU (pack_lowp_32)
    bool no_stream = false;  // nr_set_debug bit 11: the 16-bit MLP's builtin form (MlpArgs::lp_stream)
    bool no_clamp = false;  // nr_set_debug bit 9: bf16 ReLU by v_pk_max_i16, fp32 by add + max,
                            // on the same packs
    bool f32_clamp_ok = false;  // the fp32 pack is scaled for the clamped ReLU (pack_fp32_16)
    int schedule = 0; // NR_SCHED_PERSISTENT
    uint32_t *d_tr = nullptr;  // persistent-schedule counters + stats
    int debug = 0;
    int blocks_per_cu = 0;     // persistent grid: blocks (4 waves) per CU; 0 = auto
    // temporal block ordering (nr_set_temporal_order)
    int temporal = 0;
    int spread = -1;  // nr_set_pixel_spread; -1 = auto (spread_for)
    int probe_steps = 0, probe_take = 16, probe_dilate = 1;  // nr_set_cost_probe
    int wave_rays = 0;  // nr_set_wave_rays (0: automatic, wave_rays_for)
    int nq_shift = 3;    // nr_set_queue_shards: 8
    // nr_render_batch: per-frame arguments (pinned staging + device copy), host-output scratch
    FrameArgs *h_frames = nullptr, *d_frames = nullptr;
    size_t cap_frames = 0;
    hipEvent_t ev_frames = nullptr;
    uint32_t *d_bout = nullptr;
    size_t cap_bout = 0;
    uint32_t *d_bcost = nullptr, *d_order[2] = {nullptr, nullptr};
    size_t cap_blocks = 0;
    int order_valid = 0, order_cur = 0;
    long long order_key = -1;  // image configuration the stored order belongs to
    unsigned long long *d_stamps = nullptr;
    size_t n_stamps = 0;       // waves of the last traced launch

    // settings
    float inv_view[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 2};
    float normal[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -2, 0, 0, 0, 1};
    int frame = 0, color_type = NR_COLOR_FACING, num_inputs = 3, scene = NR_SCENE_V1;
    uint32_t *d_matcap = nullptr;
    int mw = 0, mh = 0;

    // scratch (owned per context; the reference keeps static globals)
    size_t cap_rays = 0;
    float4 *d_P[2] = {nullptr, nullptr}, *d_D[2] = {nullptr, nullptr};
    float4 *d_SP = nullptr, *d_SD = nullptr;
    float4 *d_FP[2] = {nullptr, nullptr}, *d_FD[2] = {nullptr, nullptr};  // wavefront endgame: fine queues
    size_t cap_fine = 0;
    size_t cap_ctr = 0;
    uint32_t *d_ctr = nullptr;       // [cap_ctr]: live counts per iteration, then shade count, then shade_it
    uint32_t *h_ctr = nullptr;       // pinned mirror
    size_t cap_out = 0;
    uint32_t *d_out = nullptr;
    size_t cap_io = 0;
    float *d_io = nullptr;           // mlp_forward staging
    int check_every = 32;            // host polls the live count every N iterations
    // layered schedule (any dense network): per-frame args in device memory, the frame's
    // launch sequence captured once per image configuration and replayed as a hipGraph
    RenderArgs *d_rargs = nullptr;
    float *d_lsdf = nullptr, *d_lz = nullptr;  // SDFs (4 per converged ray), layer scratch
    size_t cap_lsdf = 0, cap_lz = 0;
    hipGraphExec_t lgraph = nullptr;
    std::vector<long long> lkey;               // configuration lgraph was captured for
    long long net_ver = 0;                     // bumped by every network upload
    long layer_chunk = 0;                      // nr_set_layer_chunk (0: auto)

    // per-launch profiling (nr_set_profiling)
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    struct Rec { int kind; int e0, e1; };   // kind 0 init, 1 march, 2 shade
    std::vector<Rec> recs;
    uint64_t prof_renders = 0;
};

namespace {
thread_local std::string g_err;

int set_err(nr_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    g_err = buf;
    return code;
}

// Pixel spread of a launch of `nframes` frames of `npix` pixels each (nr_set_pixel_spread;
// -1 = auto).  One frame deals groups of 16 blocks pixel-major, so one slow block's rays
// spread over many waves and the frame's tail is shorter (fp32 2.649 -> 2.517 ms).  A batch
// hides the tails behind the next frame's bulk, and block-major dealing (coherent waves: one
// 8x8 block per refill) is faster there: bf16 at every batch size (1024^2 x 32: 0.568 ->
// 0.519 ms/frame, one 8-way shard: 0.087 -> 0.081), fp32 once a launch holds >= 8 M pixels
// (1024^2 x 32: 1.961 -> 1.908; one 8-way shard x 32 frames, 4 M: 0.290 vs 0.293).
// Measurements: profiles/r1_ab_experiments.txt.
int spread_for(const nr_ctx *c, int nframes, size_t npix) {
    if (c->spread >= 0) return c->spread;
    if (nframes < 4) return 16;
    if (c->precision != NR_PRECISION_FP32) return 0;
    return (size_t)nframes * npix >= ((size_t)8 << 20) ? 0 : 16;
}

}  // namespace

int nr::report_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

namespace {

#define HIPCHK(ctx, expr)                                                                            \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) return set_err(ctx, NR_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

template <class T>
void dfree(T *&p) {
    if (p) { (void)hipFree(p); p = nullptr; }
}

int free_network(nr_ctx *c) {
    for (auto *p : c->d_W) (void)hipFree(p);
    for (auto *p : c->d_b) (void)hipFree(p);
    c->d_W.clear(); c->d_b.clear();
    dfree(c->d_pack16); dfree(c->d_lp16); dfree(c->d_lpf16); dfree(c->d_x3lp); dfree(c->d_x3fl);
    dfree(c->d_lps16); dfree(c->d_lpfs16);
    c->fused = false;
    if (c->lgraph) { (void)hipGraphExecDestroy(c->lgraph); c->lgraph = nullptr; }
    c->lkey.clear();
    ++c->net_ver;
    return NR_OK;
}

int upload_pack(nr_ctx *c, const std::vector<uint16_t> &a, const std::vector<float> &f, uint16_t *&d_a, float *&d_f,
                MlpArgs &M) {
    std::vector<uint16_t> aa(a);
    std::vector<float> ff(f);
    size_t ab = (aa.size() * 2 + 15) / 16 * 16, fb = (ff.size() * 4 + 15) / 16 * 16;
    aa.resize(ab / 2, 0); ff.resize(fb / 4, 0.0f);
    HIPCHK(c, hipMalloc(&d_a, ab));
    HIPCHK(c, hipMalloc(&d_f, fb));
    HIPCHK(c, hipMemcpy(d_a, aa.data(), ab, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(d_f, ff.data(), fb, hipMemcpyHostToDevice));
    M.lp = d_a; M.lpf = d_f;
    M.lp_bytes = (int)ab; M.lpf_bytes = (int)fb;
    return NR_OK;
}

int upload_lowp(nr_ctx *c) {
    dfree(c->d_lp16); dfree(c->d_lpf16);
    c->mlp16.lp = nullptr; c->mlp16.lpf = nullptr; c->mlp16.lp_bytes = 0; c->mlp16.lpf_bytes = 0;
    c->mlp16.lp_clamp = 0;
    dfree(c->d_x3lp); dfree(c->d_x3fl);
    c->mlp16.x3lp = nullptr; c->mlp16.x3fl = nullptr; c->mlp16.x3n = 0;
    c->x3lp_bytes = 0; c->x3fl_bytes = 0;
    dfree(c->d_lps16); dfree(c->d_lpfs16);
    c->mlp16.lps = nullptr; c->mlp16.lpfs = nullptr;
    if (!c->fused || c->precision == NR_PRECISION_FP32) return NR_OK;
    std::vector<uint16_t> a;
    std::vector<float> f;
    int clamp = 0;
    if (c->precision == NR_PRECISION_FP32X3) {
        // lp_clamp = the fp32x3 pack is valid (its scales exist); without it (or with
        // nr_set_debug bit 9) every wave runs the fp32 MLP
        if (!pack_x3_32(c->dims, c->kernels, c->biases, a, f, &clamp))
            return set_err(c, NR_E_INVALID, "fp32x3 pack failed");
        c->clamp_ok = clamp != 0;
        c->mlp16.lp_clamp = c->clamp_ok && !c->no_clamp;
        return upload_pack(c, a, f, c->d_lp16, c->d_lpf16, c->mlp16);
    }
    if (!pack_lowp_32(c->dims, c->kernels, c->biases, c->precision, a, f, &clamp))
        return set_err(c, NR_E_INVALID, "low-precision pack failed");
    c->clamp_ok = clamp != 0;
    c->mlp16.lp_clamp = c->clamp_ok && !c->no_clamp;
    int rc = upload_pack(c, a, f, c->d_lp16, c->d_lpf16, c->mlp16);
    if (rc != NR_OK) return rc;
    // k_mlp16's 16x16x32 layout of the same pack (the networks its streams take: 7 hidden layers)
    if (c->mlp16.nh == 7) {
        std::vector<uint16_t> sa;
        std::vector<float> sf;
        pack_lowp_s16(a, f, c->mlp16.nh, sa, sf);
        MlpArgs S{};
        if ((rc = upload_pack(c, sa, sf, c->d_lps16, c->d_lpfs16, S)) != NR_OK) return rc;
        if (S.lp_bytes != c->mlp16.lp_bytes || S.lpf_bytes != c->mlp16.lpf_bytes)
            return set_err(c, NR_E_INVALID, "16x16x32 pack size mismatch");
        c->mlp16.lps = c->no_s16 ? nullptr : c->d_lps16;
        c->mlp16.lpfs = c->no_s16 ? nullptr : c->d_lpfs16;
    }
    // the fp32x3 pack beside it, for the normals (read from global memory); a network whose
    // pack is not valid keeps the fp32 normals
    std::vector<uint16_t> xa;
    std::vector<float> xf;
    int xok = 0;
    if (pack_x3_32(c->dims, c->kernels, c->biases, xa, xf, &xok) && xok) {
        MlpArgs X{};
        if ((rc = upload_pack(c, xa, xf, c->d_x3lp, c->d_x3fl, X)) != NR_OK) return rc;
        c->mlp16.x3lp = X.lp; c->mlp16.x3fl = X.lpf;
        c->x3lp_bytes = X.lp_bytes; c->x3fl_bytes = X.lpf_bytes;
        c->mlp16.x3n = c->fp32_normals ? 0 : 1;
    }
    return NR_OK;
}

int set_network(nr_ctx *c, std::vector<int> dims, std::vector<std::vector<float>> K, std::vector<std::vector<float>> B) {
    HIPCHK(c, hipSetDevice(c->device));
    free_network(c);
    c->dims = std::move(dims); c->kernels = std::move(K); c->biases = std::move(B);
    int nl = (int)c->dims.size() - 1;
    for (int l = 0; l < nl; ++l) {
        int in = c->dims[l], out = c->dims[l + 1];
        // DenseLayer::initializeWeights (denseLayer.cu:217-227): W[y*in + x] = kernel[x][y]
        std::vector<float> W((size_t)in * out);
        for (int x = 0; x < in; ++x)
            for (int y = 0; y < out; ++y) W[(size_t)y * in + x] = c->kernels[l][(size_t)x * out + y];
        float *dw = nullptr, *db = nullptr;
        HIPCHK(c, hipMalloc(&dw, W.size() * 4));
        HIPCHK(c, hipMalloc(&db, (size_t)out * 4));
        c->d_W.push_back(dw); c->d_b.push_back(db);
        HIPCHK(c, hipMemcpy(dw, W.data(), W.size() * 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(db, c->biases[l].data(), (size_t)out * 4, hipMemcpyHostToDevice));
    }
    std::vector<float> pack16;
    int f32_clamp = 0;
    c->fused = pack_fp32_16(c->dims, c->kernels, c->biases, pack16, &f32_clamp);
    c->mlp16 = MlpArgs{};
    c->mlp16.lp_stream = !c->no_stream;
    c->f32_clamp_ok = c->fused && f32_clamp != 0;
    c->mlp16.f32_clamp = c->f32_clamp_ok && !c->no_clamp;
    if (c->fused) {
        size_t pb = (pack16.size() * 4 + 15) / 16 * 16;
        pack16.resize(pb / 4, 0.0f);
        HIPCHK(c, hipMalloc(&c->d_pack16, pb));
        HIPCHK(c, hipMemcpy(c->d_pack16, pack16.data(), pb, hipMemcpyHostToDevice));
        c->mlp16.pk = c->d_pack16;
        c->mlp16.pk_bytes = (int)pb;
        c->mlp16.in0 = c->dims[0];
        c->mlp16.nh = nl - 2;
    }
    return upload_lowp(c);
}

int ensure_rays(nr_ctx *c, size_t n) {
    if (n <= c->cap_rays) return NR_OK;
    for (int i = 0; i < 2; ++i) { dfree(c->d_P[i]); dfree(c->d_D[i]); }
    dfree(c->d_SP); dfree(c->d_SD);
    c->cap_rays = 0;
    size_t b = std::max<size_t>(n, 64) * sizeof(float4);
    for (int i = 0; i < 2; ++i) {
        HIPCHK(c, hipMalloc(&c->d_P[i], b));
        HIPCHK(c, hipMalloc(&c->d_D[i], b));
    }
    HIPCHK(c, hipMalloc(&c->d_SP, b));
    HIPCHK(c, hipMalloc(&c->d_SD, b));
    c->cap_rays = std::max<size_t>(n, 64);
    return NR_OK;
}

// the wavefront schedule's fine queues (the endgame: rays marching in fp32x3), ping-pong
int ensure_fine(nr_ctx *c, size_t n) {
    if (n <= c->cap_fine) return NR_OK;
    for (int i = 0; i < 2; ++i) { dfree(c->d_FP[i]); dfree(c->d_FD[i]); }
    c->cap_fine = 0;
    const size_t b = std::max<size_t>(n, 64) * sizeof(float4);
    for (int i = 0; i < 2; ++i) {
        HIPCHK(c, hipMalloc(&c->d_FP[i], b));
        HIPCHK(c, hipMalloc(&c->d_FD[i], b));
    }
    c->cap_fine = std::max<size_t>(n, 64);
    return NR_OK;
}

int ensure_ctr(nr_ctx *c, size_t n) {
    if (n <= c->cap_ctr) return NR_OK;
    dfree(c->d_ctr);
    if (c->h_ctr) { (void)hipHostFree(c->h_ctr); c->h_ctr = nullptr; }
    c->cap_ctr = 0;
    HIPCHK(c, hipMalloc(&c->d_ctr, n * 4));
    HIPCHK(c, hipHostMalloc(&c->h_ctr, n * 4, hipHostMallocDefault));
    c->cap_ctr = n;
    return NR_OK;
}

template <class T>
int ensure_buf(nr_ctx *c, T *&p, size_t &cap, size_t n) {
    if (n <= cap) return NR_OK;
    dfree(p);
    cap = 0;
    HIPCHK(c, hipMalloc(&p, std::max<size_t>(n, 64) * sizeof(T)));
    cap = std::max<size_t>(n, 64);
    return NR_OK;
}

// event pair for one launch when profiling; returns indices into ev_pool
int prof_begin(nr_ctx *c, int kind, hipStream_t s) {
    if (!c->profiling) return 0;
    size_t need = c->recs.size() * 2 + 2;
    while (c->ev_pool.size() < need) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreate(&e));
        c->ev_pool.push_back(e);
    }
    int e0 = (int)c->recs.size() * 2;
    c->recs.push_back({kind, e0, e0 + 1});
    HIPCHK(c, hipEventRecord(c->ev_pool[e0], s));
    return NR_OK;
}
int prof_end(nr_ctx *c, hipStream_t s) {
    if (!c->profiling) return NR_OK;
    HIPCHK(c, hipEventRecord(c->ev_pool[c->recs.back().e1], s));
    return NR_OK;
}

int num_cus(int dev) {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    return cus;
}


int read_queue_counters(nr_ctx *c, int max_steps, nr_stats &st, hipStream_t s);

// The endgame's threshold for a persistent render (TraceArgs::eg_tau): nr_set_endgame's, for the
// bf16/fp16 tracers with fp32x3 normals (the fine passes use their fp32x3 pack) and iteration
// counts that fit the fine queue's 24 bits; 0 otherwise (the pure 16-bit march)
static float endgame_tau(const nr_ctx *c, int max_steps) {
    const bool lowp = c->precision == NR_PRECISION_BF16 || c->precision == NR_PRECISION_FP16;
    return lowp && c->mlp16.x3n && max_steps < (1 << 24) ? c->eg_tau : 0.0f;
}

// Persistent-tracer workgroups per CU for a launch of `total` pixels over `nframes` frames
// (profiles/r2_occupancy.txt, r2_single_bpc.txt, r2_lowp_occ.txt):
//   fp32: 2 for one frame or fewer than 4 frames or under 1 M pixels (the tail outweighs the
//         bulk), 4 from 8 M pixels (the 38 KB, <= 128-VGPR batched instance), else 3;
//   bf16/fp16 (<= 128 VGPRs, 31 KB): 2 under 1 M pixels, 3 under 2 M (a 1024^2 frame: 0.885 /
//         0.843 / 0.856 ms at 2 / 3 / 4), else 4 (1024^2 x 20: 0.424 -> 0.404 ms/frame at 3 -> 4,
//         2048^2 x 8: 1.661 -> 1.569, one 2048^2 frame 2.503 -> 2.481).
int default_bpc(const nr_ctx *c, size_t total, int nframes) {
    const size_t M = (size_t)1 << 20;
    // fp32x3: its k_trace instance is built for 3 waves per SIMD (168 VGPRs)
    if (c->precision == NR_PRECISION_FP32X3) return total < M ? 2 : 3;
    if (c->precision == NR_PRECISION_FP32) {
        if (nframes < 4 || total < M) return 2;
        return total >= 8 * M ? 4 : 3;
    }
    if (total < M) return 2;
    return total < 2 * M ? 3 : 4;
}

// Workgroups per CU of a persistent launch: nr_set_occupancy's value or default_bpc's; for the
// endgame's instances (eg: a bf16/fp16 launch with T.eg_tau > 0; the diagnostic stamps and probe
// instances march without the endgame, launch_trace_k) NR_TRACE_BPC_EG 4-wave workgroups' worth:
// with NR_EG_WAVES > 4 exactly that -- launch_trace_k runs them as one NR_EG_WAVES-wave workgroup
// per CU, and fewer would leave CUs idle -- else at most that
int trace_bpc(const nr_ctx *c, size_t total, int nframes, bool eg) {
    const int bpc = c->blocks_per_cu > 0 ? c->blocks_per_cu : default_bpc(c, total, nframes);
    if (eg) return NR_EG_WAVES > 4 ? NR_TRACE_BPC_EG : std::min(bpc, NR_TRACE_BPC_EG);
    return bpc;
}

// Rays per wave of a persistent launch (nr_set_wave_rays; 0 = automatic): an fp32 launch whose
// pixels fill at most 2x its waves' 64-ray slots marches 32 per wave -- at 64 nearly every ray
// is dealt in the first refills and every wave runs 4 tiles per iteration (one 1024^2 frame on
// 8 row-band shards: 1.015 -> 0.854 ms, on 4 shards 1.139 -> 1.124; on 2 shards or whole frames
// 32 is slower, and bf16, whose tiles are cheap, gains nothing; profiles/r3_ab_experiments.txt
// (24), (25)).
int wave_rays_for(const nr_ctx *c, size_t pixels, int grid) {
    if (c->wave_rays > 0) return c->wave_rays;
    if (c->precision == NR_PRECISION_FP32 && pixels <= 2 * (size_t)grid * 4 * 64) return 32;
    return 64;
}

// Block-cost buffers of the temporal order / cost probe for a frame-shard shape: a new shape
// (key) invalidates the recorded order; the buffers grow with the block count.
int order_buffers(nr_ctx *c, int W, int H, int band, int nshards, int shard, int nblocks) {
    const long long key = ((((long long)W * 65536 + H) * 4096 + band) * 64 + nshards) * 64 + shard;
    if (key != c->order_key) { c->order_valid = 0; c->order_key = key; }
    if ((size_t)nblocks > c->cap_blocks) {
        dfree(c->d_bcost); dfree(c->d_order[0]); dfree(c->d_order[1]);
        HIPCHK(c, hipMalloc(&c->d_bcost, (size_t)nblocks * 4));
        HIPCHK(c, hipMalloc(&c->d_order[0], (size_t)nblocks * 4));
        HIPCHK(c, hipMalloc(&c->d_order[1], (size_t)nblocks * 4));
        c->cap_blocks = nblocks;
        c->order_valid = 0;
    }
    return NR_OK;
}

// Per-frame arguments of a batch: pinned staging (reused only once the previous upload
// has been consumed) + device copy.  With host outputs the frames of one launch go
// through d_bout (`chunk` frames).
// The MLP arguments of a launch over these frame numbers: the bf16 clamped-ReLU form
// (nr_mlp16.h) needs every network input within LP_INPUT_BOUND.  Ray positions stay inside
// the bounding sphere; the 4th input of an animation network is the frame number, checked here.
MlpArgs mlp_for_frames(const nr_ctx *c, const nr_frame *frames, int nframes, int frame) {
    MlpArgs M = c->mlp16;
    if (M.in0 == 4) {
        bool ok = std::fabs((float)frame) <= LP_INPUT_BOUND;
        for (int i = 0; i < nframes && ok; ++i) ok = std::fabs((float)frames[i].frame) <= LP_INPUT_BOUND;
        if (!ok) M.lp_clamp = 0;
    }
    return M;
}

int upload_frames(nr_ctx *c, const nr_frame *frames, int nframes, size_t npix, int loc, int chunk, hipStream_t s) {
    if (!c->ev_frames) HIPCHK(c, hipEventCreateWithFlags(&c->ev_frames, hipEventDisableTiming));
    HIPCHK(c, hipEventSynchronize(c->ev_frames));
    if ((size_t)nframes > c->cap_frames) {
        if (c->h_frames) HIPCHK(c, hipHostFree(c->h_frames));
        dfree(c->d_frames);
        c->h_frames = nullptr;
        c->cap_frames = 0;
        HIPCHK(c, hipHostMalloc(&c->h_frames, (size_t)nframes * sizeof(FrameArgs)));
        HIPCHK(c, hipMalloc(&c->d_frames, (size_t)nframes * sizeof(FrameArgs)));
        c->cap_frames = nframes;
    }
    int rc;
    if (loc != NR_DEVICE && (rc = ensure_buf(c, c->d_bout, c->cap_bout, npix * chunk)) != NR_OK) return rc;
    for (int i = 0; i < nframes; ++i) {
        FrameArgs &f = c->h_frames[i];
        memcpy(f.inv_view, frames[i].inv_view, sizeof f.inv_view);
        memcpy(f.normal, frames[i].normal, sizeof f.normal);
        f.zoff = -0.7 + ((double)(frames[i].frame * 2) * 0.7 / 360.0);  // sphere_zoff, same f64 ops
        f.frame = frames[i].frame;
        f.frame_f = (float)frames[i].frame;
        f.out = loc == NR_DEVICE ? frames[i].out : c->d_bout + (size_t)(i % chunk) * npix;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_frames, c->h_frames, (size_t)nframes * sizeof(FrameArgs), hipMemcpyHostToDevice, s));
    HIPCHK(c, hipEventRecord(c->ev_frames, s));
    return NR_OK;
}

// Wavefront schedule over the frames of a batch (one frame for nr_render_shard): the
// rays of up to 32 frames share one queue; per iteration ONE k_march16 launch (mlp16 +
// step + compaction) over it, at the end k_shade16.  The host polls the live count every
// check_every iterations and stops early once it is 0.
// bf16 / fp16 with the endgame (round 6, the persistent tracer's rule; endgame_tau): per
// iteration the coarse pass (k_march16 mode 1) hands the rays whose 16-bit SDF is below tau to
// the iteration's fine queue, then the fine pass (mode 2) marches that queue in fp32x3 -- so the
// frames equal the persistent schedule's, bit for bit (tests/test_gpu_endgame.py).
int render_wavefront(nr_ctx *c, const nr_frame *frames, int nframes, int W, int H, int band, int nshards, int shard,
                     int max_steps, int loc, nr_stats *stats, hipStream_t s) {
    const int rows = nr_shard_rows(H, band, nshards, shard);
    const size_t npix = (size_t)W * rows;
    nr_stats tot{};
    if (npix == 0) { if (stats) *stats = tot; return NR_OK; }
    if (npix > (1u << 27))
        return set_err(c, NR_E_INVALID, "nr_render: the wavefront schedule takes at most 2^27 pixels per shard");
    const int chunk = std::min(nframes, NR_MAX_BATCH);
    // WF_SEGS queue segments of seg_cap entries (a multiple of the 256-thread block)
    const size_t seg_cap = ((npix * chunk + WF_SEGS - 1) / WF_SEGS + 255) / 256 * 256;
    // counters: (max_steps + 1) x [WF_SEGS live counts], [WF_SEGS shade counts], then
    // max_steps shade flags; each count on its own 128-byte line
    const size_t line = (size_t)WF_SEGS * 32;
    const float tau = endgame_tau(c, max_steps);
    const bool eg = tau > 0.0f;
    // the endgame's counters after them: (max_steps + 1) x [WF_SEGS fine counts], then one switch
    // count per iteration
    const size_t f_base = ((size_t)(max_steps + 2) * line + max_steps + line - 1) / line * line;
    const size_t sw_base = f_base + (size_t)(max_steps + 1) * line;
    const size_t nctr = eg ? sw_base + max_steps : (size_t)(max_steps + 2) * line + max_steps;
    int rc;
    if ((rc = ensure_rays(c, seg_cap * WF_SEGS)) != NR_OK) return rc;
    if (eg && (rc = ensure_fine(c, seg_cap * WF_SEGS)) != NR_OK) return rc;
    if ((rc = ensure_ctr(c, nctr + 8)) != NR_OK) return rc;
    if ((rc = upload_frames(c, frames, nframes, npix, loc, chunk, s)) != NR_OK) return rc;
    RenderArgs A{};
    A.out = nullptr; A.W = W; A.H = H; A.rows = rows; A.band = band; A.nshards = nshards; A.shard = shard;
    A.max_steps = max_steps; A.scene = c->scene; A.frame = 0; A.color_type = c->color_type;
    A.matcap = c->d_matcap; A.mw = c->mw; A.mh = c->mh;
    set_recips(A);
    const int cus = num_cus(c->device);
    const int bpc = c->blocks_per_cu > 0 ? c->blocks_per_cu : 16;  // measured: 4 -> 2.10, 8 -> 2.06, 16 -> 2.02 ms/frame (32-frame batch)
    uint32_t *cnt = c->d_ctr, *shade_cnt = c->d_ctr + (size_t)(max_steps + 1) * line,
             *shade_it = c->d_ctr + (size_t)(max_steps + 2) * line;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    for (int f0 = 0; f0 < nframes; f0 += chunk) {
        const int n = std::min(chunk, nframes - f0);
        const FrameArgs *F = c->d_frames + f0;
        const size_t total = npix * n;
        HIPCHK(c, hipMemsetAsync(c->d_ctr, 0, nctr * 4, s));
        QueueArgs Q{};
        Q.seg_cap = (long)seg_cap;
        Q.cnt_out = cnt; Q.p_out = c->d_P[0]; Q.d_out = c->d_D[0];
        Q.shade_cnt = shade_cnt; Q.shade_p = c->d_SP; Q.shade_d = c->d_SD; Q.shade_it = shade_it;
        Q.eg_tau = tau;
        uint32_t *fcnt = c->d_ctr + f_base, *fsw = c->d_ctr + sw_base;
        if ((rc = prof_begin(c, 0, s)) != NR_OK) return rc;
        HIPCHK(c, launch_init_f(A, F, Q, (long)npix, (long)total, cus * 8, s));
        if ((rc = prof_end(c, s)) != NR_OK) return rc;
        tot.launches += 2;
        const int grid = (int)std::max<size_t>(1, std::min<size_t>((total + 255) / 256, (size_t)cus * bpc));
        for (int it = 0; it < max_steps; ++it) {
            Q.cnt_in = cnt + (size_t)it * line; Q.cnt_out = cnt + (size_t)(it + 1) * line;
            Q.p_in = c->d_P[it & 1]; Q.d_in = c->d_D[it & 1];
            Q.p_out = c->d_P[(it + 1) & 1]; Q.d_out = c->d_D[(it + 1) & 1];
            // the endgame: the coarse pass appends this iteration's switched rays to fine queue `it`
            // (where the previous fine pass left its survivors), the fine pass then marches it
            Q.fcnt = fcnt + (size_t)it * line; Q.fp = c->d_FP[it & 1]; Q.fd = c->d_FD[it & 1]; Q.fsw = fsw + it;
            if ((rc = prof_begin(c, 1, s)) != NR_OK) return rc;
            HIPCHK(c, launch_march16(A, mlp_for_frames(c, frames, nframes, 0), Q, F, c->precision, it, grid, s, eg ? 1 : 0));
            if ((rc = prof_end(c, s)) != NR_OK) return rc;
            ++tot.launches;
            if (eg) {
                QueueArgs G = Q;
                G.cnt_in = fcnt + (size_t)it * line; G.cnt_out = fcnt + (size_t)(it + 1) * line;
                G.p_in = c->d_FP[it & 1]; G.d_in = c->d_FD[it & 1];
                G.p_out = c->d_FP[(it + 1) & 1]; G.d_out = c->d_FD[(it + 1) & 1];
                if ((rc = prof_begin(c, 1, s)) != NR_OK) return rc;
                HIPCHK(c, launch_march16(A, mlp_for_frames(c, frames, nframes, 0), G, F, c->precision, it, grid, s, 2));
                if ((rc = prof_end(c, s)) != NR_OK) return rc;
                ++tot.launches;
            }
            if (c->check_every > 0 && (it + 1) % c->check_every == 0 && it + 1 < max_steps) {
                HIPCHK(c, hipMemcpyAsync(c->h_ctr, Q.cnt_out, line * 4, hipMemcpyDeviceToHost, s));
                if (eg) HIPCHK(c, hipMemcpyAsync(c->h_ctr + line, fcnt + (size_t)(it + 1) * line, line * 4,
                                                 hipMemcpyDeviceToHost, s));
                HIPCHK(c, hipStreamSynchronize(s));
                uint64_t live = 0;
                for (int q = 0; q < WF_SEGS; ++q) live += c->h_ctr[q * 32] + (eg ? c->h_ctr[line + q * 32] : 0u);
                if (live == 0) break;
            }
        }
        const int shade_grid = (int)std::max<size_t>(1, std::min<size_t>((total + 1023) / 1024, (size_t)cus * 4));
        if ((rc = prof_begin(c, 2, s)) != NR_OK) return rc;
        HIPCHK(c, launch_shade16(A, c->mlp16, Q, F, shade_grid, s));
        if ((rc = prof_end(c, s)) != NR_OK) return rc;
        if (loc != NR_DEVICE)
            for (int i = f0; i < f0 + n; ++i)
                HIPCHK(c, hipMemcpyAsync(frames[i].out, c->d_bout + (size_t)(i % chunk) * npix, npix * 4,
                                         hipMemcpyDeviceToHost, s));
        if (stats) {
            HIPCHK(c, hipMemcpyAsync(c->h_ctr, c->d_ctr, nctr * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            const uint32_t *h = c->h_ctr;
            int iters = 0;
            for (int it = 0; it < max_steps; ++it) {
                uint64_t live = 0, fine = 0;
                for (int q = 0; q < WF_SEGS; ++q) live += h[(size_t)it * line + q * 32];
                if (it == 0) tot.rays_hit += live;
                if (eg) {
                    // the fine queue of iteration it: its switched rays (counted in `live` too: their
                    // 16-bit evaluation) and the survivors of the previous fine pass
                    for (int q = 0; q < WF_SEGS; ++q) fine += h[f_base + (size_t)it * line + q * 32];
                    tot.endgame_evals += fine;
                    tot.endgame_switches += h[sw_base + it];
                    live += fine;
                }
                tot.ray_steps += live;
                if (live) iters = std::max(iters, it + 1);
                if (h[(size_t)(max_steps + 2) * line + it]) iters = std::max(iters, std::min(it + 2, max_steps));
            }
            uint64_t shaded = 0;
            for (int q = 0; q < WF_SEGS; ++q) shaded += h[(size_t)(max_steps + 1) * line + q * 32];
            tot.rays_shaded += shaded;
            tot.shade_evals += 4 * shaded;
            tot.iterations = std::max(tot.iterations, iters);
        }
    }
    if (c->profiling) c->prof_renders += nframes;
    HIPCHK(c, hipEventRecord(c->ev1, s));
    if (stats) {
        HIPCHK(c, hipStreamSynchronize(s));
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        tot.ms_total = ms;
        *stats = tot;
    } else if (loc != NR_DEVICE) {
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return NR_OK;
}

// one dense layer over n rows (k_dense<0>)
hipError_t dense_rows(const float *W, const float *b, const float *A, float *Z, long n, int in, int out, int relu,
                      int cus, hipStream_t s) {
    DenseArgs D{};
    D.W = W; D.b = b; D.A = A; D.Z = Z;
    D.n = n; D.chunk0 = 0; D.chunk_n = n;
    D.in = in; D.out = out; D.relu = relu;
    const int grid = (int)std::max<long>(1, std::min<long>((n * out + 255) / 256, (long)cus * 8));
    return launch_dense(D, 0, grid, s);
}

// counts of the queue schedules (wavefront, layered) from their per-iteration counters
int read_queue_counters(nr_ctx *c, int max_steps, nr_stats &st, hipStream_t s) {
    const size_t nctr = (size_t)2 * max_steps + 2;
    HIPCHK(c, hipMemcpyAsync(c->h_ctr, c->d_ctr, nctr * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    uint64_t steps = 0;
    int iters = 0;
    for (int it = 0; it < max_steps; ++it) {
        steps += c->h_ctr[it];
        if (c->h_ctr[it]) iters = std::max(iters, it + 1);
        if (c->h_ctr[max_steps + 2 + it]) iters = std::max(iters, std::min(it + 2, max_steps));
    }
    st.ray_steps = steps;
    st.rays_hit = c->h_ctr[0];
    st.rays_shaded = c->h_ctr[max_steps + 1];
    st.shade_evals = 4ull * st.rays_shaded;
    st.iterations = iters;
    return NR_OK;
}
int queue_stats(nr_ctx *c, int max_steps, int launches, nr_stats *stats, hipStream_t s) {
    if (!stats) return NR_OK;
    nr_stats st{};
    int rc = read_queue_counters(c, max_steps, st, s);
    if (rc != NR_OK) return rc;
    st.launches = launches;
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    st.ms_total = ms;
    *stats = st;
    return NR_OK;
}

// Layered schedule: the reference's structure (render_kernel :608-692, one
// NeuralNetwork::forward over the live points per iteration, denseLayer.cu:229-278) for
// any dense [3|4, ..., 1] network.  Per iteration: the dense layers over the live-ray
// queue in chunks of lchunk points (bounded scratch, the kernel.cu:659-660 TODO), then
// k_march_l; at the end the layers over 4 points per converged ray and k_shade_l.  All
// counts stay on the device; the whole frame is captured once per configuration and
// replayed as a hipGraph (the per-frame RenderArgs are rewritten in device memory by
// k_set_args before each replay).  fp32 throughout (nr_set_precision applies to the
// fused kernels).
int render_layered(nr_ctx *c, const RenderArgs &A0, uint32_t *out, size_t npix, int max_steps, int loc, nr_stats *stats,
                   hipStream_t s) {
    const int nl = (int)c->dims.size() - 1;
    if (c->dims[0] > 4) return set_err(c, NR_E_FORMAT, "nr_render: at most 4 network inputs (has %d)", c->dims[0]);
    int maxw = 1;
    for (int l = 1; l < nl; ++l) maxw = std::max(maxw, c->dims[l]);
    // chunk: 128 MiB per scratch buffer, at least 64K points, at most what a frame needs
    const long lchunk = c->layer_chunk > 0 ? c->layer_chunk
                                           : std::min<long>(4l * (long)npix, std::max<long>(65536, (128l << 20) / (4l * maxw)));
    int rc;
    if ((rc = ensure_rays(c, npix)) != NR_OK) return rc;
    if ((rc = ensure_ctr(c, (size_t)2 * max_steps + 8)) != NR_OK) return rc;
    if ((rc = ensure_buf(c, c->d_lsdf, c->cap_lsdf, 4 * npix)) != NR_OK) return rc;
    if ((rc = ensure_buf(c, c->d_lz, c->cap_lz, (size_t)2 * lchunk * maxw)) != NR_OK) return rc;
    if (!c->d_rargs) HIPCHK(c, hipMalloc(&c->d_rargs, sizeof(RenderArgs)));
    RenderArgs A = A0;
    if (loc != NR_DEVICE) {
        if ((rc = ensure_buf(c, c->d_out, c->cap_out, npix)) != NR_OK) return rc;
        A.out = c->d_out;
    }
    const int cus = num_cus(c->device);
    const int step_grid = (int)std::max<size_t>(1, std::min<size_t>((npix + 255) / 256, (size_t)cus * 4));
    const int shade_grid = (int)std::max<size_t>(1, std::min<size_t>((npix + 1023) / 1024, (size_t)cus * 4));
    const long nch_march = ((long)npix + lchunk - 1) / lchunk, nch_shade = (4l * (long)npix + lchunk - 1) / lchunk;
    uint32_t *cnt = c->d_ctr, *shade_cnt = c->d_ctr + max_steps + 1, *shade_it = c->d_ctr + max_steps + 2;
    const size_t nctr = (size_t)2 * max_steps + 2;
    float *zb[2] = {c->d_lz, c->d_lz + (size_t)lchunk * maxw};
    QueueArgs Q{};
    Q.shade_cnt = shade_cnt; Q.shade_p = c->d_SP; Q.shade_d = c->d_SD; Q.shade_it = shade_it;
    // the dense chain over one chunk of a queue (src 1: live rays, 2: tetrahedron points)
    auto chain = [&](int src, const float4 *pts, const uint32_t *count, int mul, long chunk0) -> hipError_t {
        for (int l = 0; l < nl; ++l) {
            DenseArgs D{};
            D.W = c->d_W[l]; D.b = c->d_b[l];
            D.in = c->dims[l]; D.out = c->dims[l + 1]; D.relu = l != nl - 1;
            D.A = l == 0 ? nullptr : zb[(l - 1) & 1];
            D.Z = l == nl - 1 ? c->d_lsdf + chunk0 : zb[l & 1];
            D.pts = pts; D.count = count; D.count_mul = mul; D.args = c->d_rargs;
            D.chunk0 = chunk0; D.chunk_n = lchunk;
            const int grid = (int)std::max<long>(1, std::min<long>((lchunk * D.out + 255) / 256, (long)cus * 8));
            hipError_t e = launch_dense(D, l == 0 ? src : 0, grid, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    };
    // one frame's launches (captured into the graph, or issued directly for long caps)
    auto frame = [&]() -> hipError_t {
        hipError_t e = hipMemsetAsync(c->d_ctr, 0, nctr * 4, s);
        if (e != hipSuccess) return e;
        Q.cnt_out = cnt; Q.p_out = c->d_P[0]; Q.d_out = c->d_D[0];
        if ((e = launch_init_l(c->d_rargs, Q, (long)npix, s)) != hipSuccess) return e;
        for (int it = 0; it < max_steps; ++it) {
            Q.cnt_in = cnt + it; Q.cnt_out = cnt + it + 1;
            Q.p_in = c->d_P[it & 1]; Q.d_in = c->d_D[it & 1];
            Q.p_out = c->d_P[(it + 1) & 1]; Q.d_out = c->d_D[(it + 1) & 1];
            for (long ch = 0; ch < nch_march; ++ch)
                if ((e = chain(1, Q.p_in, Q.cnt_in, 1, ch * lchunk)) != hipSuccess) return e;
            if ((e = launch_march_l(c->d_rargs, Q, c->d_lsdf, it, step_grid, s)) != hipSuccess) return e;
        }
        for (long ch = 0; ch < nch_shade; ++ch)
            if ((e = chain(2, c->d_SP, shade_cnt, 4, ch * lchunk)) != hipSuccess) return e;
        return launch_shade_l(c->d_rargs, Q, c->d_lsdf, shade_grid, s);
    };
    const int launches = 2 + max_steps * (int)(1 + nch_march * nl) + (int)(nch_shade * nl) + 1;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    HIPCHK(c, launch_set_args(A, c->d_rargs, s));
    if ((rc = prof_begin(c, 1, s)) != NR_OK) return rc;
    // graph unless: long caps, the legacy null stream (not capturable), or debug bit 256
    // (direct launches, for profilers that do not follow graph launches)
    if (max_steps <= 1024 && s != nullptr && !(c->debug & 256)) {
        const std::vector<long long> key = {A.W, A.rows, A.band, A.nshards, A.shard, max_steps, c->net_ver, lchunk,
                                            (long long)(uintptr_t)c->d_P[0], (long long)(uintptr_t)c->d_ctr,
                                            (long long)(uintptr_t)c->d_lsdf, (long long)(uintptr_t)c->d_lz,
                                            (long long)(uintptr_t)c->d_SP, (long long)(uintptr_t)s};
        if (!c->lgraph || key != c->lkey) {
            if (c->lgraph) { HIPCHK(c, hipGraphExecDestroy(c->lgraph)); c->lgraph = nullptr; }
            hipGraph_t g = nullptr;
            HIPCHK(c, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            hipError_t e = frame();
            hipError_t e2 = hipStreamEndCapture(s, &g);
            if (e != hipSuccess || e2 != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                return set_err(c, NR_E_HIP, "nr_render: layered graph capture failed: %s",
                               hipGetErrorString(e != hipSuccess ? e : e2));
            }
            e = hipGraphInstantiate(&c->lgraph, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (e != hipSuccess) { c->lgraph = nullptr; return set_err(c, NR_E_HIP, "hipGraphInstantiate: %s", hipGetErrorString(e)); }
            c->lkey = key;
        }
        HIPCHK(c, hipGraphLaunch(c->lgraph, s));
    } else {
        HIPCHK(c, frame());
    }
    if ((rc = prof_end(c, s)) != NR_OK) return rc;
    if (c->profiling) c->prof_renders++;
    HIPCHK(c, hipEventRecord(c->ev1, s));
    if (loc != NR_DEVICE) HIPCHK(c, hipMemcpyAsync(out, A.out, npix * 4, hipMemcpyDeviceToHost, s));
    if (!stats && loc != NR_DEVICE) HIPCHK(c, hipStreamSynchronize(s));
    return queue_stats(c, max_steps, launches, stats, s);
}

}  // namespace

extern "C" {

int nr_abi_version(void) { return NR_ABI_VERSION; }

const char *nr_last_error(const nr_ctx *ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

// The context's stream: the caller's (nr_set_stream) or the private one, created here on
// first use.  Returns NULL only if that creation failed (error recorded).
#define GET_STREAM(c, s)                                           \
    hipStream_t s = cur_stream(c);                                 \
    if ((c)->use_own && !(c)->own_stream) return NR_E_HIP;

static hipStream_t cur_stream(nr_ctx *c) {
    if (c->use_own && !c->own_stream) {
        if (hipSetDevice(c->device) != hipSuccess ||
            hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
            c->own_stream = nullptr;
            set_err(c, NR_E_HIP, "stream creation failed");
            return nullptr;
        }
        c->stream = c->own_stream;
    }
    return c->stream;
}

int nr_create(int device, nr_ctx **out) {
    if (!out) return set_err(nullptr, NR_E_INVALID, "nr_create: out is NULL");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) return set_err(nullptr, NR_E_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    if (device < 0 || device >= ndev) return set_err(nullptr, NR_E_INVALID, "device %d out of range (%d devices)", device, ndev);
    nr_ctx *c = new (std::nothrow) nr_ctx();
    if (!c) return set_err(nullptr, NR_E_NOMEM, "out of host memory");
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipEventCreate(&c->ev0) != hipSuccess ||
        hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return set_err(nullptr, NR_E_HIP, "stream/event creation failed");
    }
    c->use_own = true;  // the private stream is created on first use (cur_stream)
    *out = c;
    return NR_OK;
}

int nr_destroy(nr_ctx *c) {
    if (!c) return NR_OK;
    (void)hipSetDevice(c->device);
    if (!(c->use_own && !c->own_stream)) (void)hipStreamSynchronize(c->stream);
    free_network(c);
    for (int i = 0; i < 2; ++i) { dfree(c->d_P[i]); dfree(c->d_D[i]); dfree(c->d_FP[i]); dfree(c->d_FD[i]); }
    dfree(c->d_SP); dfree(c->d_SD); dfree(c->d_ctr); dfree(c->d_out); dfree(c->d_tr); dfree(c->d_stamps); dfree(c->d_bcost); dfree(c->d_order[0]); dfree(c->d_order[1]); dfree(c->d_io); dfree(c->d_matcap);
    dfree(c->d_rargs); dfree(c->d_lsdf); dfree(c->d_lz);
    dfree(c->d_frames); dfree(c->d_bout);
    if (c->h_frames) (void)hipHostFree(c->h_frames);
    if (c->ev_frames) (void)hipEventDestroy(c->ev_frames);
    if (c->h_ctr) (void)hipHostFree(c->h_ctr);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return NR_OK;
}

int nr_set_stream(nr_ctx *c, void *s, int own) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    c->use_own = own != 0;
    c->stream = own ? c->own_stream : (hipStream_t)s;
    return NR_OK;
}

int nr_synchronize(nr_ctx *c) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    {
        GET_STREAM(c, s_);
        HIPCHK(c, hipStreamSynchronize(s_));
    }
    return NR_OK;
}

int nr_load_h5(nr_ctx *c, const char *path) {
    if (!c || !path) return set_err(c, NR_E_INVALID, "nr_load_h5: NULL argument");
    std::vector<int> dims;
    std::vector<std::vector<float>> K, B;
    std::string err;
    int rc = h5_read_keras(path, dims, K, B, err);
    if (rc != NR_OK) return set_err(c, rc, "Failed to initialize model (%s): %s", path, err.c_str());
    return set_network(c, std::move(dims), std::move(K), std::move(B));
}

int nr_load_mlp(nr_ctx *c, int nlayers, const int *dims, const float *const *kernels, const float *const *biases) {
    if (!c || nlayers < 1 || !dims || !kernels || !biases) return set_err(c, NR_E_INVALID, "nr_load_mlp: bad arguments");
    std::vector<int> d(dims, dims + nlayers + 1);
    for (int v : d)
        if (v < 1 || v > 4096) return set_err(c, NR_E_INVALID, "nr_load_mlp: layer size %d out of range", v);
    std::vector<std::vector<float>> K(nlayers), B(nlayers);
    for (int l = 0; l < nlayers; ++l) {
        if (!kernels[l] || !biases[l]) return set_err(c, NR_E_INVALID, "nr_load_mlp: NULL layer %d", l);
        K[l].assign(kernels[l], kernels[l] + (size_t)d[l] * d[l + 1]);
        B[l].assign(biases[l], biases[l] + d[l + 1]);
    }
    return set_network(c, std::move(d), std::move(K), std::move(B));
}

int nr_mlp_info(const nr_ctx *c, int *nlayers, int *dims, int *nw, int *nb) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    int nl = c->dims.empty() ? 0 : (int)c->dims.size() - 1;
    if (nlayers) *nlayers = nl;
    int w = 0, b = 0;
    for (int l = 0; l < nl; ++l) {
        if (dims) dims[l] = c->dims[l];
        w += c->dims[l] * c->dims[l + 1];
        b += c->dims[l + 1];
    }
    if (dims && nl) dims[nl] = c->dims[nl];
    if (nw) *nw = w;
    if (nb) *nb = b;
    return NR_OK;
}

int nr_set_precision(nr_ctx *c, int precision) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    if (precision < NR_PRECISION_FP32 || precision > NR_PRECISION_FP32X3)
        return set_err(c, NR_E_INVALID, "unknown precision %d", precision);
    c->precision = precision;
    HIPCHK(c, hipSetDevice(c->device));
    return upload_lowp(c);
}

int nr_set_view(nr_ctx *c, const float inv_view[12], const float normal[16], int frame) {
    if (!c || !inv_view || !normal) return set_err(c, NR_E_INVALID, "nr_set_view: NULL argument");
    memcpy(c->inv_view, inv_view, sizeof c->inv_view);
    memcpy(c->normal, normal, sizeof c->normal);
    c->frame = frame;
    return NR_OK;
}

int nr_set_static(nr_ctx *c, int color_type, int num_inputs) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    if (color_type != NR_COLOR_FACING && color_type != NR_COLOR_MATCAP)
        return set_err(c, NR_E_INVALID, "unknown color type %d", color_type);
    if (num_inputs != 3 && num_inputs != 4) return set_err(c, NR_E_INVALID, "numInputs must be 3 or 4");
    c->color_type = color_type;
    c->num_inputs = num_inputs;
    return NR_OK;
}

int nr_set_scene(nr_ctx *c, int scene) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    if (scene < NR_SCENE_V1 || scene > NR_SCENE_ROUND) return set_err(c, NR_E_INVALID, "unknown scene %d", scene);
    c->scene = scene;
    return NR_OK;
}

int nr_set_matcap(nr_ctx *c, const uint32_t *rgba, int w, int h) {
    if (!c || !rgba || w < 1 || h < 1) return set_err(c, NR_E_INVALID, "nr_set_matcap: bad arguments");
    HIPCHK(c, hipSetDevice(c->device));
    dfree(c->d_matcap);
    HIPCHK(c, hipMalloc(&c->d_matcap, (size_t)w * h * 4));
    HIPCHK(c, hipMemcpy(c->d_matcap, rgba, (size_t)w * h * 4, hipMemcpyHostToDevice));
    c->mw = w; c->mh = h;
    return NR_OK;
}

int nr_render_batch(nr_ctx *c, const nr_frame *frames, int nframes, int W, int H, int band, int nshards, int shard,
                    int max_steps, int loc, nr_stats *stats) {
    if (!c || !frames || nframes < 1) return set_err(c, NR_E_INVALID, "nr_render_batch: bad arguments");
    for (int i = 0; i < nframes; ++i)
        if (!frames[i].out) return set_err(c, NR_E_INVALID, "nr_render_batch: frame %d has no output", i);
    if (W < 1 || H < 1 || (long)W * H > (1l << 31)) return set_err(c, NR_E_INVALID, "nr_render: bad size %dx%d", W, H);
    if (band < 1 || nshards < 1 || shard < 0 || shard >= nshards) return set_err(c, NR_E_INVALID, "nr_render: bad shard");
    if (max_steps < 0) return set_err(c, NR_E_INVALID, "nr_render: max_steps < 0");
    if (c->schedule == NR_SCHED_WAVEFRONT && c->fused) {
        if (c->dims[0] != c->num_inputs)
            return set_err(c, NR_E_STATE, "nr_render: network takes %d inputs but numInputs = %d", c->dims[0], c->num_inputs);
        if (c->color_type == NR_COLOR_MATCAP && !c->d_matcap) return set_err(c, NR_E_STATE, "nr_render: matcap colouring without a matcap");
        HIPCHK(c, hipSetDevice(c->device));
        GET_STREAM(c, s);
        return render_wavefront(c, frames, nframes, W, H, band, nshards, shard, max_steps, loc, stats, s);
    }
    if (c->schedule != NR_SCHED_PERSISTENT || !c->fused || (c->debug & (1 | 8))) {
        // frame by frame (the wavefront and layered schedules and the diagnostics are
        // single-frame)
        float iv[12], nm[16];
        memcpy(iv, c->inv_view, sizeof iv);
        memcpy(nm, c->normal, sizeof nm);
        const int fr0 = c->frame;
        nr_stats tot{};
        int rc = NR_OK;
        for (int i = 0; i < nframes && rc == NR_OK; ++i) {
            memcpy(c->inv_view, frames[i].inv_view, sizeof iv);
            memcpy(c->normal, frames[i].normal, sizeof nm);
            c->frame = frames[i].frame;
            nr_stats st{};
            rc = nr_render_shard(c, frames[i].out, W, H, band, nshards, shard, max_steps, loc, stats ? &st : nullptr);
            tot.ray_steps += st.ray_steps; tot.shade_evals += st.shade_evals; tot.rays_hit += st.rays_hit;
            tot.rays_shaded += st.rays_shaded; tot.iterations = std::max(tot.iterations, st.iterations);
            tot.launches += st.launches; tot.ms_total += st.ms_total; tot.endgame_evals += st.endgame_evals;
            tot.endgame_switches += st.endgame_switches;
        }
        memcpy(c->inv_view, iv, sizeof iv);
        memcpy(c->normal, nm, sizeof nm);
        c->frame = fr0;
        if (rc == NR_OK && stats) *stats = tot;
        return rc;
    }
    if (c->dims.empty()) return set_err(c, NR_E_STATE, "nr_render: no network loaded");
    if (!c->fused)
        return set_err(c, NR_E_FORMAT, "nr_render: network shape unsupported by the fused march kernel "
                                       "(needs [3|4, 32, ..., 32, 1])");
    if (c->dims[0] != c->num_inputs)
        return set_err(c, NR_E_STATE, "nr_render: network takes %d inputs but numInputs = %d", c->dims[0], c->num_inputs);
    if (c->color_type == NR_COLOR_MATCAP && !c->d_matcap) return set_err(c, NR_E_STATE, "nr_render: matcap colouring without a matcap");
    HIPCHK(c, hipSetDevice(c->device));
    const int rows = nr_shard_rows(H, band, nshards, shard);
    const size_t npix = (size_t)W * rows;
    nr_stats st{};
    if (npix == 0) { if (stats) *stats = st; return NR_OK; }
    GET_STREAM(c, s);
    int rc;
    const int chunk = nr_batch_frames_per_launch(W, H, band, nshards, shard, nframes, 1 << c->nq_shift);
    if (chunk < 1)
        return set_err(c, NR_E_INVALID, "nr_render_batch: %dx%d shard overflows the 32-bit pixel queue", W, H);
    if ((rc = upload_frames(c, frames, nframes, npix, loc, chunk, s)) != NR_OK) return rc;

    RenderArgs A{};
    A.out = nullptr; A.W = W; A.H = H; A.rows = rows; A.band = band; A.nshards = nshards; A.shard = shard;
    A.max_steps = max_steps; A.scene = c->scene; A.frame = 0; A.color_type = c->color_type;
    A.matcap = c->d_matcap; A.mw = c->mw; A.mh = c->mh;
    set_recips(A);
    const size_t tr_bytes = NR_MAX_QUEUES * 128 + 8 * 8;
    if (!c->d_tr) HIPCHK(c, hipMalloc(&c->d_tr, 2 * tr_bytes));
    TraceArgs T{};
    T.pix_ctr = c->d_tr;
    T.stats = reinterpret_cast<unsigned long long *>(c->d_tr + NR_MAX_QUEUES * 32);
    T.nq_shift = c->nq_shift;
    T.bw = (W + 7) / 8;
    T.nblocks = T.bw * ((rows + 7) / 8);
    {
        const int sp = spread_for(c, nframes, npix);
        T.spread_shift = sp > 1 ? 31 - __builtin_clz((unsigned)sp) : 0;
    }
    T.inv_bw = 1.0 / (double)T.bw;
    T.inv_band = 1.0 / (double)band;
    const int cus = num_cus(c->device);
    // temporal block order (nr_set_temporal_order): every launch dispenses the blocks of its
    // frames longest-first by the costs the previous launch of this frame-shard shape recorded
    // (the block layout is the same for every frame of a batch; the costs are the max over them)
    if (c->temporal) {
        int rc3;
        if ((rc3 = order_buffers(c, W, H, band, nshards, shard, T.nblocks)) != NR_OK) return rc3;
    }
    HIPCHK(c, hipEventRecord(c->ev0, s));
    int launches = 0;
    for (int f0 = 0; f0 < nframes; f0 += chunk) {
        const int n = std::min(chunk, nframes - f0);
        T.frames = c->d_frames + f0;
        T.nframes = n;
        T.inv_nframes = 1.0 / (double)n;
        // frames interleaved in 64-position chunks: every frame of the launch progresses
        // together, so the launch does not end on one frame's silhouette rays started last
        // (1024^2 x 32 frames 1.866 -> 1.825 ms/frame, one 8-way shard x 8 frames 0.367 ->
        // 0.334; profiles/r2_ab_experiments.txt (10)).  Debug bit 10: frame-major (A/B).
        T.interleave = !((c->debug >> 10) & 1);
        T.eg_tau = endgame_tau(c, max_steps);
        T.x3lp_bytes = c->x3lp_bytes;
        T.x3fl_bytes = c->x3fl_bytes;
        // the counters restart for every launch; the statistics accumulate
        HIPCHK(c, hipMemsetAsync(c->d_tr, 0, f0 == 0 ? tr_bytes : (size_t)NR_MAX_QUEUES * 128, s));
        // workgroups per CU: default_bpc (with several frames in a launch their tails overlap,
        // so the extra waves per SIMD lift the bulk rate instead of lengthening the tail)
        const int bpc = trace_bpc(c, npix * n, n, T.eg_tau > 0.0f && c->mlp16.x3n);
        int grid = (int)std::min<size_t>((npix * n + 255) / 256, (size_t)cus * bpc);
        if (grid < 1) grid = 1;
        T.take = wave_rays_for(c, npix * n, grid);
        T.lane_cap = T.take >= 64 ? ~0ull : (1ull << T.take) - 1ull;
        if (c->temporal) {
            T.order = c->order_valid ? c->d_order[c->order_cur] : nullptr;
            T.bcost = c->d_bcost;
            HIPCHK(c, hipMemsetAsync(c->d_bcost, 0, (size_t)T.nblocks * 4, s));
        }
        int rc2;
        if ((rc2 = prof_begin(c, 1, s)) != NR_OK) return rc2;
        HIPCHK(c, launch_trace(A, mlp_for_frames(c, frames, nframes, 0), T, c->precision, grid, s));
        if ((rc2 = prof_end(c, s)) != NR_OK) return rc2;
        if (c->temporal) {  // the order for the next launch of this shape
            HIPCHK(c, launch_order(c->d_bcost, c->d_order[c->order_cur ^ 1], T.nblocks, T.bw, c->temporal > 1, s));
            c->order_cur ^= 1;
            c->order_valid = 1;
        }
        ++launches;
        if (loc != NR_DEVICE)
            for (int i = f0; i < f0 + n; ++i)
                HIPCHK(c, hipMemcpyAsync(frames[i].out, c->d_bout + (size_t)(i % chunk) * npix, npix * 4,
                                         hipMemcpyDeviceToHost, s));
    }
    if (c->profiling) c->prof_renders += nframes;
    HIPCHK(c, hipEventRecord(c->ev1, s));
    if (stats) {
        unsigned long long hs[6];
        HIPCHK(c, hipMemcpyAsync(hs, T.stats, sizeof hs, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        st.ray_steps = hs[0];
        st.endgame_evals = hs[4];
        st.endgame_switches = hs[5];
        st.rays_hit = hs[1];
        st.iterations = (int32_t)hs[2];
        st.rays_shaded = hs[3];
        st.shade_evals = 4ull * hs[3];
        st.launches = launches;
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        st.ms_total = ms;
        *stats = st;
    } else if (loc != NR_DEVICE) {
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return NR_OK;
}

// Queue positions are uint32 (pix_ctr atomics in k_trace): one launch hands out
// shard_total = blocks of the busiest queue shard x 64 x frames positions.  Past a shard's end
// a wave of the low-precision tracers can take two pending reservations of up to 64 positions
// (NR_QUEUE_CHUNK_DENSE: one absorbed and found past the end while the wave still had positions
// of its pool, the next requested right after) and one blocking reservation of up to 64 before
// it moves on: with the grid nr_set_occupancy allows (16 workgroups x 4 waves per CU) on up to
// 512 CUs the over-reservation stays below 512 x 16 x 4 x 192 = 6,291,456 (the old
// 2^19 assumed 8 workgroups and no pending reservation).
int nr_batch_frames_per_launch(int W, int H, int band, int nshards, int shard, int nframes, int queue_shards) {
    if (W < 1 || H < 1 || nframes < 1 || queue_shards < 1) return 0;
    const int rows = nr_shard_rows(H, band, nshards, shard);
    if (rows < 1) return std::min(nframes, NR_MAX_BATCH);
    const long long nblocks = (long long)((W + 7) / 8) * ((rows + 7) / 8);
    const long long per_frame = ((nblocks + queue_shards - 1) / queue_shards) * 64;  // busiest shard
    const long long slop = 512ll * 16 * 4 * (64 + 2 * 64);
    const long long cap = ((1ll << 32) - 1 - slop) / per_frame;
    return (int)std::min<long long>(std::min(nframes, NR_MAX_BATCH), cap);
}

int nr_shard_rows(int H, int band, int nshards, int shard) {
    if (H < 0 || band < 1 || nshards < 1 || shard < 0 || shard >= nshards) return 0;
    int full = H / band, rem = H % band;
    int rows = (full / nshards) * band;
    int extra = full % nshards;               // bands beyond the complete rounds
    if (shard < extra) rows += band;
    if (shard == extra && rem) rows += rem;   // the partial last band
    return rows;
}

int nr_render_shard(nr_ctx *c, uint32_t *out, int W, int H, int band, int nshards, int shard, int max_steps, int loc,
                    nr_stats *stats) {
    if (!c || !out) return set_err(c, NR_E_INVALID, "nr_render: NULL argument");
    if (W < 1 || H < 1 || (long)W * H > (1l << 31)) return set_err(c, NR_E_INVALID, "nr_render: bad size %dx%d", W, H);
    if (band < 1 || nshards < 1 || shard < 0 || shard >= nshards) return set_err(c, NR_E_INVALID, "nr_render: bad shard");
    if (max_steps < 0) return set_err(c, NR_E_INVALID, "nr_render: max_steps < 0");
    if (c->dims.empty()) return set_err(c, NR_E_STATE, "nr_render: no network loaded");
    if (c->dims.back() != 1)
        return set_err(c, NR_E_FORMAT, "nr_render: the SDF network must have one output (has %d)", c->dims.back());
    if (c->dims[0] != c->num_inputs)
        return set_err(c, NR_E_STATE, "nr_render: network takes %d inputs but numInputs = %d", c->dims[0], c->num_inputs);
    if (c->color_type == NR_COLOR_MATCAP && !c->d_matcap) return set_err(c, NR_E_STATE, "nr_render: matcap colouring without a matcap");
    HIPCHK(c, hipSetDevice(c->device));
    int rows = nr_shard_rows(H, band, nshards, shard);
    size_t npix = (size_t)W * rows;
    nr_stats st{};
    if (npix == 0) { if (stats) *stats = st; return NR_OK; }
    int rc;
    if ((rc = ensure_rays(c, npix)) != NR_OK) return rc;
    if ((rc = ensure_ctr(c, (size_t)2 * max_steps + 8)) != NR_OK) return rc;
    uint32_t *dout = out;
    if (loc != NR_DEVICE) {
        if ((rc = ensure_buf(c, c->d_out, c->cap_out, npix)) != NR_OK) return rc;
        dout = c->d_out;
    }
    RenderArgs A{};
    A.out = dout; A.W = W; A.H = H; A.rows = rows; A.band = band; A.nshards = nshards; A.shard = shard;
    A.max_steps = max_steps; A.scene = c->scene; A.frame = c->frame; A.color_type = c->color_type;
    A.matcap = c->d_matcap; A.mw = c->mw; A.mh = c->mh;
    set_recips(A);
    memcpy(A.inv_view, c->inv_view, sizeof A.inv_view);
    memcpy(A.normal, c->normal, sizeof A.normal);
    GET_STREAM(c, s);
    int cus = num_cus(c->device);
    int rc2;
    if (!c->fused || c->schedule == NR_SCHED_LAYERED) return render_layered(c, A, out, npix, max_steps, loc, stats, s);
    if (c->schedule == NR_SCHED_PERSISTENT) {
        // 8 shard counters on their own 128-byte lines, then 4 x u64 stats
        // (a second set for the cost probe)
        const size_t tr_bytes = NR_MAX_QUEUES * 128 + 8 * 8;
        if (!c->d_tr) HIPCHK(c, hipMalloc(&c->d_tr, 2 * tr_bytes));
        TraceArgs T{};
        T.pix_ctr = c->d_tr;
        T.stats = reinterpret_cast<unsigned long long *>(c->d_tr + NR_MAX_QUEUES * 32);
        T.nq_shift = c->nq_shift;
        const int bw = (W + 7) / 8, bh = (rows + 7) / 8;
        T.bw = bw;
        T.nblocks = bw * bh;
        T.itmap = (c->debug & 8) != 0;
        // the stamps instance (nr_set_debug bit 0) marches without the endgame
        T.eg_tau = (c->debug & 1) ? 0.0f : endgame_tau(c, max_steps);
        T.x3lp_bytes = c->x3lp_bytes;
        T.x3fl_bytes = c->x3fl_bytes;
        {
            const int sp = spread_for(c, 1, npix);
            T.spread_shift = sp > 1 ? 31 - __builtin_clz((unsigned)sp) : 0;
        }
        T.inv_bw = 1.0 / (double)T.bw;
        T.inv_band = 1.0 / (double)band;
        if (c->temporal || c->probe_steps > 0)
            if ((rc2 = order_buffers(c, W, H, band, nshards, shard, T.nblocks)) != NR_OK) return rc2;
        const bool probe = c->probe_steps > 0 && max_steps > 0 && !(c->temporal && c->order_valid);
        if (c->temporal) {
            T.order = c->order_valid ? c->d_order[c->order_cur] : nullptr;
            T.bcost = c->d_bcost;
        }
        const int bpc = trace_bpc(c, npix, 1, T.eg_tau > 0.0f && c->mlp16.x3n);
        int grid = (int)std::min<size_t>((npix + 255) / 256, (size_t)cus * bpc);
        if (grid < 1) grid = 1;
        T.take = wave_rays_for(c, npix, grid);
        T.lane_cap = T.take >= 64 ? ~0ull : (1ull << T.take) - 1ull;
        if (c->debug & 1) {
            if (!c->d_stamps) HIPCHK(c, hipMalloc(&c->d_stamps, (size_t)cus * 16 * 4 * 16 * 8));
            T.stamps = c->d_stamps;
            c->n_stamps = (size_t)grid * 4;
        }
        HIPCHK(c, hipEventRecord(c->ev0, s));
        HIPCHK(c, hipMemsetAsync(c->d_tr, 0, (probe ? 2 : 1) * tr_bytes, s));
        if (probe) {
            // cost probe: march each block's centre ray for at most probe_steps iterations,
            // then hand the blocks out longest-first
            if ((rc2 = prof_begin(c, 0, s)) != NR_OK) return rc2;
            HIPCHK(c, hipMemsetAsync(c->d_bcost, 0, (size_t)T.nblocks * 4, s));
            TraceArgs P = T;
            P.probe = 1;
            P.take = c->probe_take;
            P.lane_cap = P.take >= 64 ? ~0ull : (1ull << P.take) - 1ull;
            P.pix_ctr = c->d_tr + tr_bytes / 4;
            P.stats = reinterpret_cast<unsigned long long *>(c->d_tr + tr_bytes / 4 + NR_MAX_QUEUES * 32);
            P.stamps = nullptr;
            P.order = nullptr;
            P.bcost = c->d_bcost;
            P.spread_shift = 0;
            RenderArgs Ap = A;
            Ap.max_steps = std::min(max_steps, c->probe_steps);
            const long pwaves = ((long)T.nblocks + P.take - 1) / P.take;
            const int pgrid = (int)std::max<long>(1, std::min<long>((pwaves + 3) / 4, grid));
            HIPCHK(c, launch_trace(Ap, mlp_for_frames(c, nullptr, 0, A.frame), P, c->precision, pgrid, s));
            HIPCHK(c, launch_order(c->d_bcost, c->d_order[c->order_cur], T.nblocks, T.bw, c->probe_dilate, s));
            if ((rc2 = prof_end(c, s)) != NR_OK) return rc2;
            T.order = c->d_order[c->order_cur];
        }
        if (T.bcost) HIPCHK(c, hipMemsetAsync(c->d_bcost, 0, (size_t)T.nblocks * 4, s));
        if ((rc2 = prof_begin(c, 1, s)) != NR_OK) return rc2;
        HIPCHK(c, launch_trace(A, mlp_for_frames(c, nullptr, 0, A.frame), T, c->precision, grid, s));
        if ((rc2 = prof_end(c, s)) != NR_OK) return rc2;
        if (c->temporal) {  // order for the next frame of the same configuration
            HIPCHK(c, launch_order(c->d_bcost, c->d_order[c->order_cur ^ 1], T.nblocks, T.bw, c->temporal > 1, s));
            c->order_cur ^= 1;
            c->order_valid = 1;
        }
        if (c->profiling) c->prof_renders++;
        HIPCHK(c, hipEventRecord(c->ev1, s));
        if (loc != NR_DEVICE) HIPCHK(c, hipMemcpyAsync(out, dout, npix * 4, hipMemcpyDeviceToHost, s));
        if (stats) {
            unsigned long long hs[6];
            HIPCHK(c, hipMemcpyAsync(hs, T.stats, sizeof hs, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            st.ray_steps = hs[0];
            st.endgame_evals = hs[4];
            st.endgame_switches = hs[5];
            st.rays_hit = hs[1];
            st.iterations = (int32_t)hs[2];
            st.rays_shaded = hs[3];
            st.shade_evals = 4ull * hs[3];
            st.launches = 2;
            float ms = 0;
            HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
            st.ms_total = ms;
            *stats = st;
        } else if (loc != NR_DEVICE) {
            HIPCHK(c, hipStreamSynchronize(s));
        }
        return NR_OK;
    }
    // ---- wavefront schedule (render_wavefront) on this one frame
    nr_frame fr{};
    memcpy(fr.inv_view, c->inv_view, sizeof fr.inv_view);
    memcpy(fr.normal, c->normal, sizeof fr.normal);
    fr.frame = c->frame;
    fr.out = dout;
    if ((rc2 = render_wavefront(c, &fr, 1, W, H, band, nshards, shard, max_steps, NR_DEVICE, stats, s)) != NR_OK)
        return rc2;
    if (loc != NR_DEVICE) {
        HIPCHK(c, hipMemcpyAsync(out, dout, npix * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return NR_OK;
}

int nr_render(nr_ctx *c, uint32_t *out, int W, int H, int max_steps, int loc, nr_stats *stats) {
    return nr_render_shard(c, out, W, H, H > 0 ? H : 1, 1, 0, max_steps, loc, stats);
}

int nr_assemble_shards(nr_ctx *c, const uint32_t *src, size_t stride, uint32_t *dst, int W, int H, int band,
                       int nshards, int loc) {
    if (!src || !dst || W < 1 || H < 1 || band < 1 || nshards < 1) return set_err(c, NR_E_INVALID, "nr_assemble_shards: bad arguments");
    if (loc == NR_DEVICE) {
        if (!c) return set_err(nullptr, NR_E_INVALID, "device assembly needs a context");
        HIPCHK(c, hipSetDevice(c->device));
        GET_STREAM(c, s);
        HIPCHK(c, launch_assemble(src, stride, dst, W, H, band, nshards, s));
        return NR_OK;
    }
    for (int y = 0; y < H; ++y) {
        int b = y / band, s = b % nshards, lr = (b / nshards) * band + y % band;
        memcpy(dst + (size_t)y * W, src + (size_t)s * stride + (size_t)lr * W, (size_t)W * 4);
    }
    return NR_OK;
}

int nr_pack_x3(int nlayers, const int *dims, const float *const *kernels, const float *const *biases, uint16_t *a,
               long a_cap, float *f, long f_cap, long *a_len, long *f_len, int *ok) {
    if (nlayers < 1 || !dims || !kernels || !biases || !a_len || !f_len || !ok)
        return nr::report_error(NR_E_INVALID, "nr_pack_x3: bad arguments");
    std::vector<int> d(dims, dims + nlayers + 1);
    std::vector<std::vector<float>> K(nlayers), B(nlayers);
    for (int l = 0; l < nlayers; ++l) {
        if (!kernels[l] || !biases[l] || d[l] < 1 || d[l + 1] < 1)
            return nr::report_error(NR_E_INVALID, "nr_pack_x3: layer %d", l);
        K[l].assign(kernels[l], kernels[l] + (size_t)d[l] * d[l + 1]);
        B[l].assign(biases[l], biases[l] + d[l + 1]);
    }
    std::vector<uint16_t> av;
    std::vector<float> fv;
    int k = 0;
    if (!pack_x3_32(d, K, B, av, fv, &k)) return nr::report_error(NR_E_INVALID, "nr_pack_x3: not a fused shape");
    *a_len = (long)av.size();
    *f_len = (long)fv.size();
    *ok = k;
    if (a && a_cap >= (long)av.size()) std::memcpy(a, av.data(), av.size() * 2);
    if (f && f_cap >= (long)fv.size()) std::memcpy(f, fv.data(), fv.size() * 4);
    return NR_OK;
}

int nr_mlp_forward(nr_ctx *c, const float *X, float *Y, long n, int loc) {
    if (!c || (n > 0 && (!X || !Y)) || n < 0) return set_err(c, NR_E_INVALID, "nr_mlp_forward: bad arguments");
    if (c->dims.empty()) return set_err(c, NR_E_STATE, "nr_mlp_forward: no network loaded");
    if (n == 0) return NR_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int nl = (int)c->dims.size() - 1, in0 = c->dims[0], outn = c->dims[nl];
    GET_STREAM(c, s);
    const float *dX = X;
    float *dY = Y;
    int rc;
    int maxw = *std::max_element(c->dims.begin(), c->dims.end());
    // the generic chain runs in chunks of at most 64 MiB of activations per buffer
    const long chunk = std::min<long>(n, std::max<long>(16384, (64l << 20) / (4l * maxw)));
    size_t need = (loc == NR_DEVICE ? 0 : (size_t)n * (in0 + outn)) + (c->fused ? 0 : (size_t)2 * chunk * maxw);
    if ((rc = ensure_buf(c, c->d_io, c->cap_io, need)) != NR_OK) return rc;
    float *scratch = c->d_io;
    if (loc != NR_DEVICE) {
        float *hx = scratch; scratch += (size_t)n * in0;
        dY = scratch; scratch += (size_t)n * outn;
        HIPCHK(c, hipMemcpyAsync(hx, X, (size_t)n * in0 * 4, hipMemcpyHostToDevice, s));
        dX = hx;
    }
    if (c->fused) {
        // workgroups per CU: 8 (queued beyond the resident ones, they keep every SIMD fed
        // to the end of the batch): 2^24 points fp32 0.796 -> 0.825 of peak, bf16 (102 VGPRs,
        // 5 waves per SIMD resident) 0.352 -> 0.410 against 4 (profiles/r2_mlp_microbench.txt)
        // 12 workgroups per CU by default: more than fit at once (3-5), so that workgroups start
        // staggered as earlier ones retire -- a grid of exactly the resident workgroups runs the
        // bf16 MLP 17 % slower (its waves stay in step: profiles/r3_mlp_bpc.txt)
        // (a per-CU LDS chunk queue balanced the SIMD's waves but left the kernel time unchanged,
        // round 4: profiles/r4_mlp_ab.txt)
        const MlpArgs M = c->mlp16;
        const int bpc = c->blocks_per_cu > 0 ? c->blocks_per_cu : 12;
        const int grid = num_cus(c->device) * bpc;
        if (c->debug & 64)  // diagnostic: n = repetitions, X >= 64 points, Y >= 65 floats
            HIPCHK(c, launch_mlp_latency(c->mlp16, c->precision, dX, dY, (int)n,
                                         ((c->wave_rays > 0 ? c->wave_rays : 64) + 15) / 16,
                                         ((c->debug >> 7) & 1) | (((c->debug >> 13) & 3) << 1), s));
            // (bf16/fp16: wave_rays 16 / 32 time the tracer's 64-point form on 1 / 2 32-point tiles,
            // otherwise the 128-point form)
        else
            HIPCHK(c, launch_mlp16(M, c->precision, dX, dY, n, grid, s));
    } else {
        float *bufs[2] = {scratch, scratch + (size_t)chunk * maxw};
        const int cus = num_cus(c->device);
        for (long p0 = 0; p0 < n; p0 += chunk) {
            const long m = std::min(chunk, n - p0);
            const float *a = dX + (size_t)p0 * in0;
            for (int l = 0; l < nl; ++l) {
                float *z = (l == nl - 1) ? dY + (size_t)p0 * outn : bufs[l & 1];
                HIPCHK(c, dense_rows(c->d_W[l], c->d_b[l], a, z, m, c->dims[l], c->dims[l + 1], l != nl - 1, cus, s));
                a = z;
            }
        }
    }
    if (loc != NR_DEVICE) {
        HIPCHK(c, hipMemcpyAsync(Y, dY, (size_t)n * outn * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return NR_OK;
}

int nr_layer_forward(nr_ctx *c, int layer, const float *A, float *Z, long n, int loc) {
    if (!c || n < 0 || (n > 0 && (!A || !Z))) return set_err(c, NR_E_INVALID, "nr_layer_forward: bad arguments");
    int nl = c->dims.empty() ? 0 : (int)c->dims.size() - 1;
    if (layer < 0 || layer >= nl) return set_err(c, NR_E_INVALID, "nr_layer_forward: layer %d out of range", layer);
    if (n == 0) return NR_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int in = c->dims[layer], out = c->dims[layer + 1];
    GET_STREAM(c, s);
    const float *dA = A;
    float *dZ = Z;
    if (loc != NR_DEVICE) {
        int rc = ensure_buf(c, c->d_io, c->cap_io, (size_t)n * (in + out));
        if (rc != NR_OK) return rc;
        float *ha = c->d_io;
        dZ = c->d_io + (size_t)n * in;
        HIPCHK(c, hipMemcpyAsync(ha, A, (size_t)n * in * 4, hipMemcpyHostToDevice, s));
        dA = ha;
    }
    HIPCHK(c, dense_rows(c->d_W[layer], c->d_b[layer], dA, dZ, n, in, out, layer != nl - 1, num_cus(c->device), s));
    if (loc != NR_DEVICE) {
        HIPCHK(c, hipMemcpyAsync(Z, dZ, (size_t)n * out * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return NR_OK;
}

int nr_set_profiling(nr_ctx *c, int on) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    c->profiling = on != 0;
    return NR_OK;
}

int nr_prof_collect(nr_ctx *c, nr_kernel_prof *out) {
    if (!c || !out) return set_err(c, NR_E_INVALID, "nr_prof_collect: NULL argument");
    HIPCHK(c, hipSetDevice(c->device));
    {
        GET_STREAM(c, s_);
        HIPCHK(c, hipStreamSynchronize(s_));
    }
    nr_kernel_prof p{};
    for (auto &r : c->recs) {
        float ms = 0;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev_pool[r.e0], c->ev_pool[r.e1]));
        if (r.kind == 0) { p.init_ms += ms; p.init_launches++; }
        else if (r.kind == 1) { p.march_ms += ms; p.march_launches++; }
        else { p.shade_ms += ms; p.shade_launches++; }
    }
    p.renders = c->prof_renders;
    c->recs.clear();
    c->prof_renders = 0;
    *out = p;
    return NR_OK;
}

int nr_set_schedule(nr_ctx *c, int schedule) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    if (schedule != NR_SCHED_PERSISTENT && schedule != NR_SCHED_WAVEFRONT && schedule != NR_SCHED_LAYERED)
        return set_err(c, NR_E_INVALID, "unknown schedule %d", schedule);
    c->schedule = schedule;
    return NR_OK;
}

int nr_set_temporal_order(nr_ctx *c, int on) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    c->temporal = on < 0 ? 0 : (on > 2 ? 2 : on);
    c->order_valid = 0;
    return NR_OK;
}

int nr_set_pixel_spread(nr_ctx *c, int group_blocks) {
    if (!c || group_blocks < -1 || group_blocks > 65536 || (group_blocks > 0 && (group_blocks & (group_blocks - 1))))
        return set_err(c, NR_E_INVALID,
                       "nr_set_pixel_spread: group_blocks must be -1 (auto), 0 or a power of two <= 65536");
    c->spread = group_blocks;
    return NR_OK;
}

int nr_set_cost_probe(nr_ctx *c, int max_steps, int rays_per_wave) {
    if (!c || max_steps < 0 || max_steps > 1023 || rays_per_wave < 1 || rays_per_wave > 64)
        return set_err(c, NR_E_INVALID, "nr_set_cost_probe: bad arguments");
    c->probe_steps = max_steps;
    c->probe_take = rays_per_wave;
    c->probe_dilate = (c->debug & 16) ? 0 : 1;
    return NR_OK;
}

int nr_set_layer_chunk(nr_ctx *c, long points) {
    if (!c || points < 0 || (points > 0 && points < 64))
        return set_err(c, NR_E_INVALID, "nr_set_layer_chunk: points must be 0 (auto) or >= 64");
    c->layer_chunk = points;
    return NR_OK;
}

int nr_set_queue_shards(nr_ctx *c, int n) {
    if (!c || n < 1 || n > NR_MAX_QUEUES || (n & (n - 1)))
        return set_err(c, NR_E_INVALID, "nr_set_queue_shards: n must be a power of two in [1, %d]", NR_MAX_QUEUES);
    c->nq_shift = 31 - __builtin_clz((unsigned)n);
    return NR_OK;
}

int nr_set_wave_rays(nr_ctx *c, int rays) {
    if (!c || rays < 0 || rays > 64) return set_err(c, NR_E_INVALID, "nr_set_wave_rays: rays must be in [0, 64]");
    c->wave_rays = rays;
    return NR_OK;
}

int nr_set_occupancy(nr_ctx *c, int blocks_per_cu) {
    if (!c || blocks_per_cu < 0 || blocks_per_cu > 16) return set_err(c, NR_E_INVALID, "nr_set_occupancy: bad arguments");
    c->blocks_per_cu = blocks_per_cu;
    return NR_OK;
}

int nr_set_endgame(nr_ctx *c, float tau) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    if (!(tau >= 0.0f) || tau > 1e30f) return set_err(c, NR_E_INVALID, "nr_set_endgame: tau must be finite and >= 0");
    c->eg_tau = tau;
    return NR_OK;
}

int nr_set_debug(nr_ctx *c, int flags) {
    if (!c) return set_err(nullptr, NR_E_INVALID, "ctx is NULL");
    c->debug = flags;
    c->no_clamp = (flags >> 9) & 1;
    c->no_stream = (flags >> 11) & 1;
    c->no_s16 = !((flags >> 12) & 1);
    c->mlp16.lps = c->no_s16 ? nullptr : c->d_lps16;
    c->mlp16.lpfs = c->no_s16 ? nullptr : c->d_lpfs16;
    c->fp32_normals = (flags >> 15) & 1;
    c->mlp16.x3n = !c->fp32_normals && c->mlp16.x3lp != nullptr;
    c->mlp16.lp_stream = !c->no_stream;
    c->mlp16.lp_clamp = c->clamp_ok && !c->no_clamp && c->mlp16.lp != nullptr;
    c->mlp16.f32_clamp = c->f32_clamp_ok && !c->no_clamp;
    return NR_OK;
}

int nr_debug_stamps(nr_ctx *c, unsigned long long *out, size_t cap, size_t *n) {
    if (!c || !n) return set_err(c, NR_E_INVALID, "nr_debug_stamps: NULL argument");
    *n = c->n_stamps;
    if (!out || !c->d_stamps) return NR_OK;
    {
        GET_STREAM(c, s_);
        HIPCHK(c, hipStreamSynchronize(s_));
    }
    size_t m = std::min(cap / 16, c->n_stamps);
    HIPCHK(c, hipMemcpy(out, c->d_stamps, m * 16 * 8, hipMemcpyDeviceToHost));
    return NR_OK;
}

int nr_set_poll_interval(nr_ctx *c, int every) {
    if (!c || every < 0) return set_err(c, NR_E_INVALID, "nr_set_poll_interval: bad arguments");
    c->check_every = every;
    return NR_OK;
}

int nr_dense_forward(nr_ctx *c, const float *W, const float *b, int in, int out, int relu, const float *A, float *Z,
                     long n, int loc) {
    if (!c || !W || !b || in < 1 || out < 1 || n < 0 || (n > 0 && (!A || !Z)))
        return set_err(c, NR_E_INVALID, "nr_dense_forward: bad arguments");
    if (n == 0) return NR_OK;
    HIPCHK(c, hipSetDevice(c->device));
    GET_STREAM(c, s);
    if (loc == NR_DEVICE) {
        HIPCHK(c, dense_rows(W, b, A, Z, n, in, out, relu, num_cus(c->device), s));
        return NR_OK;
    }
    // host buffers: stage everything
    size_t need = (size_t)in * out + out + (size_t)n * (in + out);
    int rc = ensure_buf(c, c->d_io, c->cap_io, need);
    if (rc != NR_OK) return rc;
    float *dW = c->d_io, *db = dW + (size_t)in * out, *dA = db + out, *dZ = dA + (size_t)n * in;
    HIPCHK(c, hipMemcpyAsync(dW, W, (size_t)in * out * 4, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(db, b, (size_t)out * 4, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(dA, A, (size_t)n * in * 4, hipMemcpyHostToDevice, s));
    HIPCHK(c, dense_rows(dW, db, dA, dZ, n, in, out, relu, num_cus(c->device), s));
    HIPCHK(c, hipMemcpyAsync(Z, dZ, (size_t)n * out * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return NR_OK;
}

int nr_camera(float rx, float ry, float zoom, float tx, float ty, float inv_view[12], float normal[16]) {
    return nr_camera_ex(rx, ry, zoom, tx, ty, NR_CAMERA_F64, inv_view, normal);
}

int nr_camera_ex(float rx, float ry, float zoom, float tx, float ty, int mode, float inv_view[12], float normal[16]) {
    if (!inv_view || !normal) return set_err(nullptr, NR_E_INVALID, "nr_camera: NULL output");
    if (mode == NR_CAMERA_F64) camera_matrices(rx, ry, zoom, tx, ty, inv_view, normal);
    else if (mode == NR_CAMERA_EIGEN) camera_matrices_eigen(rx, ry, zoom, tx, ty, inv_view, normal);
    else return set_err(nullptr, NR_E_INVALID, "nr_camera_ex: unknown mode %d", mode);
    return NR_OK;
}

int nr_h5_read_keras(const char *path, int max_layers, int *nlayers, int *dims, float *params, size_t cap) {
    if (!path || !nlayers) return set_err(nullptr, NR_E_INVALID, "nr_h5_read_keras: NULL argument");
    std::vector<int> d;
    std::vector<std::vector<float>> K, B;
    std::string err;
    int rc = h5_read_keras(path, d, K, B, err);
    if (rc != NR_OK) return set_err(nullptr, rc, "%s", err.c_str());
    int nl = (int)d.size() - 1;
    *nlayers = nl;
    if (dims) {
        if (max_layers < nl) return set_err(nullptr, NR_E_INVALID, "nr_h5_read_keras: %d layers > max_layers", nl);
        for (int i = 0; i <= nl; ++i) dims[i] = d[i];
    }
    if (params) {
        size_t need = 0;
        for (int l = 0; l < nl; ++l) need += K[l].size() + B[l].size();
        if (cap < need) return set_err(nullptr, NR_E_INVALID, "nr_h5_read_keras: params buffer too small (%zu < %zu)", cap, need);
        float *p = params;
        for (int l = 0; l < nl; ++l) {
            memcpy(p, K[l].data(), K[l].size() * 4); p += K[l].size();
            memcpy(p, B[l].data(), B[l].size() * 4); p += B[l].size();
        }
    }
    return NR_OK;
}

int nr_png_load(const char *path, uint32_t **rgba, int *w, int *h) {
    if (!path || !rgba || !w || !h) return set_err(nullptr, NR_E_INVALID, "nr_png_load: NULL argument");
    std::vector<uint32_t> px;
    std::string err;
    int rc = png_decode(path, px, *w, *h, err);
    if (rc != NR_OK) return set_err(nullptr, rc, "Error reading png: %s", err.c_str());
    *rgba = (uint32_t *)malloc(px.size() * 4);
    if (!*rgba) return set_err(nullptr, NR_E_NOMEM, "out of memory");
    memcpy(*rgba, px.data(), px.size() * 4);
    return NR_OK;
}

int nr_png_save(const char *path, const uint32_t *rgba, int w, int h, int flip) {
    if (!path || !rgba) return set_err(nullptr, NR_E_INVALID, "nr_png_save: NULL argument");
    std::string err;
    int rc = png_encode(path, rgba, w, h, flip, err);
    if (rc != NR_OK) return set_err(nullptr, rc, "[ERROR] Unable to save png: %s", err.c_str());
    return NR_OK;
}

int nr_ppm_save(const char *path, const uint32_t *rgba, int w, int h) {
    if (!path || !rgba || w < 1 || h < 1) return set_err(nullptr, NR_E_INVALID, "nr_ppm_save: bad arguments");
    std::string err;
    int rc = ppm_encode(path, rgba, w, h, err);
    if (rc != NR_OK) return set_err(nullptr, rc, "%s", err.c_str());
    return NR_OK;
}

void nr_free(void *p) { free(p); }

}  // extern "C"

// context internals for nr_group.hip (nr_internal.h)
namespace nr {
int ctx_device(const nr_ctx *c) { return c->device; }
void *ctx_stream(nr_ctx *c) { return (void *)cur_stream(c); }
}  // namespace nr
