// nr_group.hip -- multi-GPU rendering from one process: the reference's render loop
// (main.cpp:404-468 driving render_kernel, volumeRender_kernel.cu:608-692) with every frame
// split across the GPUs of a node.
//
//   * one context per GPU (nr_create on its device, the same network and settings loaded into
//     each), joined by one RCCL communicator (ncclCommInitAll: one process, N devices);
//   * context r renders row-band shard r of every frame of the call (nr_render_batch with
//     nshards = N, shard = r: bands of `band` rows dealt round-robin), the contexts in parallel
//     (one host thread each; a context is used by one thread at a time);
//   * the shards' render status is checked on the host before any transfer: a failed shard
//     ends the call with its error and no collective is started (a status
//     exchange before the gather, so no GPU waits in a collective for a rank that failed);
//   * ONE gather per call over xGMI (ncclGroupStart, every rank's ncclSend to rank 0 and rank 0's
//     ncclRecv from every rank, ncclGroupEnd) brings all frames' shards to the first GPU;
//   * one re-interleave launch per frame (nr_assemble_shards) writes the frames there.
// Rays are independent, so nothing is exchanged while the frames march.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "nr_internal.h"

struct nr_group {
    int n = 0;
    std::vector<nr_ctx *> ctx;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    std::vector<uint32_t *> shard;      // per context, on its device: its shards of the call's frames
    std::vector<size_t> shard_cap;      // pixels
    uint32_t *gather = nullptr;         // first device: N x frames x shard pixels
    size_t gather_cap = 0;
    uint32_t *staging = nullptr;        // first device: frames for a host destination
    size_t staging_cap = 0;
};

namespace {

int ensure(int device, uint32_t *&p, size_t &cap, size_t pixels) {
    if (pixels <= cap) return NR_OK;
    if (hipSetDevice(device) != hipSuccess) return NR_E_HIP;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, std::max<size_t>(pixels, 1) * 4) != hipSuccess) return NR_E_HIP;
    cap = pixels;
    return NR_OK;
}

}  // namespace

extern "C" {

int nr_group_create(nr_ctx *const *ctxs, int n, nr_group **out) {
    if (!ctxs || n < 1 || !out) return nr::report_error(NR_E_INVALID, "nr_group_create: bad arguments");
    nr_group *g = new nr_group();
    g->n = n;
    for (int r = 0; r < n; ++r) {
        if (!ctxs[r]) {
            delete g;
            return nr::report_error(NR_E_INVALID, "nr_group_create: context %d is NULL", r);
        }
        const int d = nr::ctx_device(ctxs[r]);
        if (std::find(g->dev.begin(), g->dev.end(), d) != g->dev.end()) {
            delete g;
            return nr::report_error(NR_E_INVALID, "nr_group_create: two contexts on device %d (one GPU per rank)", d);
        }
        g->ctx.push_back(ctxs[r]);
        g->dev.push_back(d);
    }
    g->comm.resize(n);
    const ncclResult_t rc = ncclCommInitAll(g->comm.data(), n, g->dev.data());
    if (rc != ncclSuccess) {
        delete g;
        return nr::report_error(NR_E_HIP, "nr_group_create: ncclCommInitAll: %s", ncclGetErrorString(rc));
    }
    g->shard.assign(n, nullptr);
    g->shard_cap.assign(n, 0);
    *out = g;
    return NR_OK;
}

int nr_group_destroy(nr_group *g) {
    if (!g) return NR_OK;
    for (int r = 0; r < g->n; ++r) {
        (void)hipSetDevice(g->dev[r]);
        if (g->shard[r]) (void)hipFree(g->shard[r]);
        if (g->comm[r]) ncclCommDestroy(g->comm[r]);
    }
    (void)hipSetDevice(g->dev[0]);
    if (g->gather) (void)hipFree(g->gather);
    if (g->staging) (void)hipFree(g->staging);
    delete g;
    return NR_OK;
}

int nr_group_size(const nr_group *g) { return g ? g->n : 0; }

int nr_group_render_batch(nr_group *g, const nr_frame *frames, int nframes, int W, int H, int band, int max_steps,
                          int loc, nr_stats *stats) {
    if (!g || !frames || nframes < 1 || W < 1 || H < 1 || band < 1 || max_steps < 0)
        return nr::report_error(NR_E_INVALID, "nr_group_render_batch: bad arguments");
    for (int i = 0; i < nframes; ++i)
        if (!frames[i].out) return nr::report_error(NR_E_INVALID, "nr_group_render_batch: frame %d has no output", i);
    const int n = g->n;
    const int max_rows = nr_shard_rows(H, band, n, 0);  // shard 0 holds the most rows
    const size_t shard_px = (size_t)max_rows * W, per_rank = shard_px * (size_t)nframes;
    for (int r = 0; r < n; ++r)
        if (ensure(g->dev[r], g->shard[r], g->shard_cap[r], per_rank) != NR_OK)
            return nr::report_error(NR_E_HIP, "nr_group_render_batch: shard buffer on device %d", g->dev[r]);
    if (ensure(g->dev[0], g->gather, g->gather_cap, per_rank * n) != NR_OK ||
        (loc != NR_DEVICE && ensure(g->dev[0], g->staging, g->staging_cap, (size_t)W * H * nframes) != NR_OK))
        return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "gather buffer");
    // ---- every context renders its shard of every frame, in parallel
    std::vector<int> rc(n, NR_OK);
    std::vector<nr_stats> st(n);
    std::vector<std::string> msg(n);
    auto work = [&](int r) {
        if (hipSetDevice(g->dev[r]) != hipSuccess) {
            rc[r] = NR_E_HIP;
            msg[r] = "hipSetDevice failed";
            return;
        }
        std::vector<nr_frame> fr(frames, frames + nframes);
        for (int i = 0; i < nframes; ++i) fr[i].out = g->shard[r] + (size_t)i * shard_px;
        rc[r] = nr_render_batch(g->ctx[r], fr.data(), nframes, W, H, band, n, r, max_steps, NR_DEVICE, &st[r]);
        if (rc[r] == NR_OK) rc[r] = nr_synchronize(g->ctx[r]);  // a fault surfaces here, before the gather
        if (rc[r] != NR_OK) msg[r] = nr_last_error(g->ctx[r]);
    };
    if (n == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int r = 0; r < n; ++r) th.emplace_back(work, r);
        for (auto &t : th) t.join();
    }
    // ---- status of every shard before any transfer
    for (int r = 0; r < n; ++r)
        if (rc[r] != NR_OK) {
            const std::string m = "shard " + std::to_string(r) + " (device " + std::to_string(g->dev[r]) + "): " + msg[r];
            return nr::report_error(rc[r], "nr_group_render_batch: %s", m.c_str());
        }
    // ---- one gather of every frame's shards to the first device
    ncclResult_t e = ncclGroupStart();
    for (int r = 0; r < n && e == ncclSuccess; ++r) {
        e = ncclSend(g->shard[r], per_rank, ncclUint32, 0, g->comm[r], (hipStream_t)nr::ctx_stream(g->ctx[r]));
    }
    for (int r = 0; r < n && e == ncclSuccess; ++r)
        e = ncclRecv(g->gather + (size_t)r * per_rank, per_rank, ncclUint32, r, g->comm[0],
                     (hipStream_t)nr::ctx_stream(g->ctx[0]));
    const ncclResult_t e2 = ncclGroupEnd();
    if (e != ncclSuccess || e2 != ncclSuccess)
        return nr::report_error(NR_E_HIP, "nr_group_render_batch: RCCL gather: %s",
                                ncclGetErrorString(e != ncclSuccess ? e : e2));
    // ---- re-interleave on the first device: frame i's shard s sits at gather + s * per_rank + i * shard_px
    for (int i = 0; i < nframes; ++i) {
        uint32_t *dst = loc == NR_DEVICE ? frames[i].out : g->staging + (size_t)i * W * H;
        const int a = nr_assemble_shards(g->ctx[0], g->gather + (size_t)i * shard_px, per_rank, dst, W, H, band, n,
                                         NR_DEVICE);
        if (a != NR_OK) return a;
    }
    if (loc != NR_DEVICE) {
        hipStream_t s0 = (hipStream_t)nr::ctx_stream(g->ctx[0]);
        for (int i = 0; i < nframes; ++i)
            if (hipMemcpyAsync(frames[i].out, g->staging + (size_t)i * W * H, (size_t)W * H * 4, hipMemcpyDeviceToHost, s0) !=
                hipSuccess)
                return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "copy to host");
    }
    const int s = nr_synchronize(g->ctx[0]);
    if (s != NR_OK) return s;
    if (stats) {
        nr_stats t{};
        for (int r = 0; r < n; ++r) {
            t.ray_steps += st[r].ray_steps;
            t.shade_evals += st[r].shade_evals;
            t.rays_hit += st[r].rays_hit;
            t.rays_shaded += st[r].rays_shaded;
            t.iterations = std::max(t.iterations, st[r].iterations);
            t.launches += st[r].launches;
            t.ms_total = std::max(t.ms_total, st[r].ms_total);
            t.endgame_evals += st[r].endgame_evals;
        }
        *stats = t;
    }
    return NR_OK;
}

}  // extern "C"
