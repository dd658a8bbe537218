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
//     ncclRecv from every rank, ncclGroupEnd) brings all frames' shards to the first GPU, on a
//     communication stream per GPU, not the render streams;
//   * one re-interleave launch per frame (launch_assemble) writes the frames there, on the first
//     GPU's communication stream.
// The shard and gather buffers are double-buffered (call k uses set k & 1): with NR_GROUP_ASYNC a
// call returns once its gather and re-interleave are enqueued, so call k + 1's render runs while
// call k's shards travel; a render into a set waits (device-side, hipStreamWaitEvent) until the
// transfer of the call before last that used it has read it.  NR_GROUP_COPY moves the shards with
// hipMemcpyPeerAsync instead of RCCL -- the same layout, offsets and re-interleave with another
// transport -- and lets several contexts share one GPU, which is how a one-GPU box runs 2- and
// 3-rank groups (tests/test_gpu_group.py).  Rays are independent, so nothing is exchanged while
// the frames march.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "nr_internal.h"
#include "nr_kernels.h"

struct nr_group {
    int n = 0;
    int flags = 0;
    std::vector<nr_ctx *> ctx;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;              // empty with NR_GROUP_COPY
    std::vector<hipStream_t> cs;               // per rank: its communication stream (on its device)
    std::vector<uint32_t *> shard[2];          // per set, per rank, on its device: its shards of a call
    std::vector<size_t> shard_cap[2];          // pixels
    std::vector<hipEvent_t> sent[2];           // per set, per rank: the set's shards have been read
                                               // (created on the device whose stream records it:
                                               // rank r's with RCCL, the first device's with NR_GROUP_COPY)
    std::vector<hipEvent_t> rendered[2];       // per set, per rank (on its device): its shards are written
    uint32_t *gather[2] = {nullptr, nullptr};  // first device: N x frames x shard pixels
    size_t gather_cap[2] = {0, 0};
    uint32_t *staging[2] = {nullptr, nullptr}; // first device: frames for a host destination
    size_t staging_cap[2] = {0, 0};
    unsigned long long calls = 0;
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

void release(nr_group *g) {
    for (int r = 0; r < (int)g->dev.size(); ++r) {
        (void)hipSetDevice(g->dev[r]);
        if (r < (int)g->cs.size() && g->cs[r]) (void)hipStreamSynchronize(g->cs[r]);
        for (int b = 0; b < 2; ++b) {
            if (r < (int)g->shard[b].size() && g->shard[b][r]) (void)hipFree(g->shard[b][r]);
            if (r < (int)g->sent[b].size() && g->sent[b][r]) (void)hipEventDestroy(g->sent[b][r]);
            if (r < (int)g->rendered[b].size() && g->rendered[b][r]) (void)hipEventDestroy(g->rendered[b][r]);
        }
        if (r < (int)g->cs.size() && g->cs[r]) (void)hipStreamDestroy(g->cs[r]);
        if (r < (int)g->comm.size() && g->comm[r]) ncclCommDestroy(g->comm[r]);
    }
    if (!g->dev.empty()) {
        (void)hipSetDevice(g->dev[0]);
        for (int b = 0; b < 2; ++b) {
            if (g->gather[b]) (void)hipFree(g->gather[b]);
            if (g->staging[b]) (void)hipFree(g->staging[b]);
        }
    }
    delete g;
}

}  // namespace

extern "C" {

int nr_group_create_ex(nr_ctx *const *ctxs, int n, int flags, nr_group **out) {
    if (!ctxs || n < 1 || !out || (flags & ~(NR_GROUP_COPY | NR_GROUP_ASYNC)))
        return nr::report_error(NR_E_INVALID, "nr_group_create: bad arguments");
    nr_group *g = new nr_group();
    g->n = n;
    g->flags = flags;
    for (int r = 0; r < n; ++r) {
        if (!ctxs[r]) {
            release(g);
            return nr::report_error(NR_E_INVALID, "nr_group_create: context %d is NULL", r);
        }
        for (int q = 0; q < r; ++q)
            if (ctxs[q] == ctxs[r]) {
                release(g);
                return nr::report_error(NR_E_INVALID, "nr_group_create: context %d appears twice", r);
            }
        const int d = nr::ctx_device(ctxs[r]);
        if (!(flags & NR_GROUP_COPY) && std::find(g->dev.begin(), g->dev.end(), d) != g->dev.end()) {
            release(g);
            return nr::report_error(NR_E_INVALID, "nr_group_create: two contexts on device %d (one GPU per rank "
                                                  "for RCCL; NR_GROUP_COPY shares a GPU)", d);
        }
        g->ctx.push_back(ctxs[r]);
        g->dev.push_back(d);
    }
    g->cs.assign(n, nullptr);
    for (int b = 0; b < 2; ++b) {
        g->shard[b].assign(n, nullptr);
        g->shard_cap[b].assign(n, 0);
        g->sent[b].assign(n, nullptr);
        g->rendered[b].assign(n, nullptr);
    }
    // an event is recorded on a stream of the device it was created on: rank r's transfer stream
    // records its `sent` events with RCCL, the first device's with NR_GROUP_COPY (the peer copies
    // all run there); the render streams only wait on them (a cross-device wait is legal)
    const bool copy = (flags & NR_GROUP_COPY) != 0;
    for (int r = 0; r < n; ++r) {
        bool ok = hipSetDevice(g->dev[r]) == hipSuccess && hipStreamCreateWithFlags(&g->cs[r], hipStreamNonBlocking) == hipSuccess;
        for (int b = 0; b < 2 && ok; ++b)
            ok = hipEventCreateWithFlags(&g->rendered[b][r], hipEventDisableTiming) == hipSuccess &&
                 hipSetDevice(copy ? g->dev[0] : g->dev[r]) == hipSuccess &&
                 hipEventCreateWithFlags(&g->sent[b][r], hipEventDisableTiming) == hipSuccess &&
                 hipSetDevice(g->dev[r]) == hipSuccess;
        if (!ok) {
            release(g);
            return nr::report_error(NR_E_HIP, "nr_group_create: streams / events on device %d", g->dev[r]);
        }
    }
    if (!(flags & NR_GROUP_COPY)) {
        g->comm.assign(n, nullptr);
        const ncclResult_t rc = ncclCommInitAll(g->comm.data(), n, g->dev.data());
        if (rc != ncclSuccess) {
            g->comm.clear();
            release(g);
            return nr::report_error(NR_E_HIP, "nr_group_create: ncclCommInitAll: %s", ncclGetErrorString(rc));
        }
    }
    *out = g;
    return NR_OK;
}

int nr_group_create(nr_ctx *const *ctxs, int n, nr_group **out) { return nr_group_create_ex(ctxs, n, 0, out); }

int nr_group_destroy(nr_group *g) {
    if (g) release(g);
    return NR_OK;
}

int nr_group_size(const nr_group *g) { return g ? g->n : 0; }

int nr_group_synchronize(nr_group *g) {
    if (!g) return nr::report_error(NR_E_INVALID, "nr_group_synchronize: NULL group");
    for (int r = 0; r < g->n; ++r)
        if (hipSetDevice(g->dev[r]) != hipSuccess || hipStreamSynchronize(g->cs[r]) != hipSuccess)
            return nr::report_error(NR_E_HIP, "nr_group_synchronize: device %d", g->dev[r]);
    return NR_OK;
}

// The gather layout: every rank's set holds frame i's shard at i * shard_px, shard_px = the rows
// of shard 0 (the most) x W; the gather buffer holds rank r's set at r * per_rank, per_rank =
// shard_px x nframes; frame i is re-interleaved from gather + i * shard_px with stride per_rank.
int nr_group_layout(int W, int H, int band, int n, int nframes, size_t *shard_px, size_t *per_rank) {
    if (W < 1 || H < 1 || band < 1 || n < 1 || nframes < 1 || !shard_px || !per_rank)
        return nr::report_error(NR_E_INVALID, "nr_group_layout: bad arguments");
    *shard_px = (size_t)nr_shard_rows(H, band, n, 0) * (size_t)W;
    *per_rank = *shard_px * (size_t)nframes;
    return NR_OK;
}

int nr_group_render_batch(nr_group *g, const nr_frame *frames, int nframes, int W, int H, int band, int max_steps,
                          int loc, nr_stats *stats) {
    if (!g || !frames || nframes < 1 || W < 1 || H < 1 || band < 1 || max_steps < 0)
        return nr::report_error(NR_E_INVALID, "nr_group_render_batch: bad arguments");
    for (int i = 0; i < nframes; ++i)
        if (!frames[i].out) return nr::report_error(NR_E_INVALID, "nr_group_render_batch: frame %d has no output", i);
    const int n = g->n;
    size_t shard_px = 0, per_rank = 0;
    nr_group_layout(W, H, band, n, nframes, &shard_px, &per_rank);
    const int b = (int)(g->calls & 1);  // this call's buffer set
    // a set's buffers are reallocated only once the transfers that read them have finished
    bool grow = per_rank * n > g->gather_cap[b] || (loc != NR_DEVICE && (size_t)W * H * nframes > g->staging_cap[b]);
    for (int r = 0; r < n; ++r) grow = grow || per_rank > g->shard_cap[b][r];
    if (grow && nr_group_synchronize(g) != NR_OK) return NR_E_HIP;
    for (int r = 0; r < n; ++r)
        if (ensure(g->dev[r], g->shard[b][r], g->shard_cap[b][r], per_rank) != NR_OK)
            return nr::report_error(NR_E_HIP, "nr_group_render_batch: shard buffer on device %d", g->dev[r]);
    if (ensure(g->dev[0], g->gather[b], g->gather_cap[b], per_rank * n) != NR_OK ||
        (loc != NR_DEVICE && ensure(g->dev[0], g->staging[b], g->staging_cap[b], (size_t)W * H * nframes) != NR_OK))
        return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "gather buffer");
    // ---- a fault of an earlier asynchronous call (its renders or transfers) ends this one first
    const bool async = (g->flags & NR_GROUP_ASYNC) != 0;
    if (async)
        for (int r = 0; r < n; ++r) {
            hipError_t q = hipSetDevice(g->dev[r]);
            if (q == hipSuccess) q = hipStreamQuery(g->cs[r]);
            if (q != hipSuccess && q != hipErrorNotReady)
                return nr::report_error(NR_E_HIP, "nr_group_render_batch: an earlier call failed on device %d: %s", g->dev[r],
                                        hipGetErrorString(q));
        }
    // ---- every context renders its shard of every frame, in parallel, into set b once the
    // transfer that last read set b is done.  Synchronous groups (and calls that ask for the
    // statistics, which are read from the device) wait for each render here, so that a fault
    // surfaces before any transfer; NR_GROUP_ASYNC only enqueues it: the transfer streams wait
    // for it device-side (`rendered`), and the host returns to submit the next call while this
    // one renders.  Its launch errors still end the call before the gather; a fault during the
    // march surfaces at the next call or at nr_group_synchronize.
    std::vector<int> rc(n, NR_OK);
    std::vector<nr_stats> st(n);
    std::vector<std::string> msg(n);
    auto work = [&](int r) {
        if (hipSetDevice(g->dev[r]) != hipSuccess) {
            rc[r] = NR_E_HIP;
            msg[r] = "hipSetDevice failed";
            return;
        }
        const hipStream_t rs = (hipStream_t)nr::ctx_stream(g->ctx[r]);
        if (g->calls >= 2 && hipStreamWaitEvent(rs, g->sent[b][r], 0) != hipSuccess) {
            rc[r] = NR_E_HIP;
            msg[r] = "hipStreamWaitEvent failed";
            return;
        }
        std::vector<nr_frame> fr(frames, frames + nframes);
        for (int i = 0; i < nframes; ++i) fr[i].out = g->shard[b][r] + (size_t)i * shard_px;
        rc[r] = nr_render_batch(g->ctx[r], fr.data(), nframes, W, H, band, n, r, max_steps, NR_DEVICE, stats ? &st[r] : nullptr);
        if (rc[r] == NR_OK && !async) rc[r] = nr_synchronize(g->ctx[r]);  // a fault surfaces here, before the gather
        if (rc[r] != NR_OK) {
            msg[r] = nr_last_error(g->ctx[r]);
            return;
        }
        if (hipEventRecord(g->rendered[b][r], rs) != hipSuccess) {
            rc[r] = NR_E_HIP;
            msg[r] = "hipEventRecord failed";
            return;
        }
        const hipError_t q = hipStreamQuery(rs);  // a fault already known on this context's stream
        if (q != hipSuccess && q != hipErrorNotReady) {
            rc[r] = NR_E_HIP;
            msg[r] = hipGetErrorString(q);
        }
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
    // ---- the transfers of set b start once its shards are rendered (device-side waits)
    const bool copy = (g->flags & NR_GROUP_COPY) != 0;
    for (int r = 0; r < n; ++r)
        if (hipSetDevice(copy ? g->dev[0] : g->dev[r]) != hipSuccess ||
            hipStreamWaitEvent(copy ? g->cs[0] : g->cs[r], g->rendered[b][r], 0) != hipSuccess)
            return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "transfer wait");
    ++g->calls;
    hipStream_t c0 = g->cs[0];
    // ---- one gather of every frame's shards to the first device, on the communication streams
    if (copy) {
        if (hipSetDevice(g->dev[0]) != hipSuccess)
            return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "hipSetDevice");
        for (int r = 0; r < n; ++r)
            if (hipMemcpyPeerAsync(g->gather[b] + (size_t)r * per_rank, g->dev[0], g->shard[b][r], g->dev[r], per_rank * 4,
                                   c0) != hipSuccess)
                return nr::report_error(NR_E_HIP, "nr_group_render_batch: shard copy from device %d", g->dev[r]);
        for (int r = 0; r < n; ++r)
            if (hipEventRecord(g->sent[b][r], c0) != hipSuccess)
                return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "event");
    } else {
        ncclResult_t e = ncclGroupStart();
        for (int r = 0; r < n && e == ncclSuccess; ++r)
            e = ncclSend(g->shard[b][r], per_rank, ncclUint32, 0, g->comm[r], g->cs[r]);
        for (int r = 0; r < n && e == ncclSuccess; ++r)
            e = ncclRecv(g->gather[b] + (size_t)r * per_rank, per_rank, ncclUint32, r, g->comm[0], c0);
        const ncclResult_t e2 = ncclGroupEnd();
        if (e != ncclSuccess || e2 != ncclSuccess)
            return nr::report_error(NR_E_HIP, "nr_group_render_batch: RCCL gather: %s",
                                    ncclGetErrorString(e != ncclSuccess ? e : e2));
        for (int r = 0; r < n; ++r)
            if (hipSetDevice(g->dev[r]) != hipSuccess || hipEventRecord(g->sent[b][r], g->cs[r]) != hipSuccess)
                return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "event");
    }
    // ---- re-interleave on the first device: frame i's shard s sits at gather + s * per_rank + i * shard_px
    if (hipSetDevice(g->dev[0]) != hipSuccess) return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "hipSetDevice");
    for (int i = 0; i < nframes; ++i) {
        uint32_t *dst = loc == NR_DEVICE ? frames[i].out : g->staging[b] + (size_t)i * W * H;
        if (nr::launch_assemble(g->gather[b] + (size_t)i * shard_px, per_rank, dst, W, H, band, n, c0) != hipSuccess)
            return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "re-interleave launch");
    }
    if (loc != NR_DEVICE) {
        for (int i = 0; i < nframes; ++i)
            if (hipMemcpyAsync(frames[i].out, g->staging[b] + (size_t)i * W * H, (size_t)W * H * 4, hipMemcpyDeviceToHost, c0) !=
                hipSuccess)
                return nr::report_error(NR_E_HIP, "nr_group_render_batch: %s", "copy to host");
    }
    // host outputs are the caller's pageable memory: such a call returns with them written
    if (!(g->flags & NR_GROUP_ASYNC) || loc != NR_DEVICE) {
        const int s = nr_group_synchronize(g);
        if (s != NR_OK) return s;
    }
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
            t.endgame_switches += st[r].endgame_switches;
        }
        *stats = t;
    }
    return NR_OK;
}

}  // extern "C"
