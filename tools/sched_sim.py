"""Offline model of the persistent tracer's schedule (k_trace), driven by a measured
per-pixel iteration map (tools/itmap.py).  Used to rank scheduling policies before
building them; not part of the product path.

Model: 1024 SIMDs, `bpc` waves each, 64 ray slots per wave.  All waves of a SIMD
advance one iteration per round; a round costs
    max(sum_w tiles_w * T_TILE,  max_w (tiles_w * T_TILE + V_WAVE))
(the matrix pipe is shared; a wave's own VALU work overlaps its partners' MFMAs).
Refills come from one global pixel queue in dispense order, in time order across SIMDs.

    python tools/sched_sim.py gpurun_out/itmap_plane_1_1024.npy
"""
import heapq
import sys

import numpy as np

T_TILE = 2.36   # us per 16-point tile-iteration of the MLP on one SIMD's matrix pipe
V_WAVE = 1.6    # us of per-wave-iteration VALU work (scene, step, refill)
NSIMD = 1024


def block_order(m, key=None):
    """Pixels in block-major order (8x8 blocks, raster), optionally blocks sorted by key desc."""
    H, W = m.shape
    bh, bw = H // 8, W // 8
    blocks = np.arange(bh * bw)
    if key is not None:
        blocks = blocks[np.argsort(-key.reshape(-1), kind="stable")]
    by, bx = blocks // bw, blocks % bw
    py = (by[:, None] * 8 + (np.arange(64) // 8)[None, :]).reshape(-1)
    px = (bx[:, None] * 8 + (np.arange(64) % 8)[None, :]).reshape(-1)
    return m[py, px]


def spread_order(m, G=16):
    H, W = m.shape
    b = block_order(m).reshape(-1, 64)          # [blocks][64]
    out = []
    for g in range(0, b.shape[0], G):
        out.append(b[g:g + G].T.reshape(-1))    # pixel-major within the group
    return np.concatenate(out)


def simulate(costs, bpc=2, merge_pairs=False, take=64, share=0):
    """costs: iteration counts in dispense order.  Returns (frame_us, drain_us).
    share > 0: once the queue is drained, a wave holding more than `share` rays moves the rest to a
    global pool and a wave holding fewer takes from it (tail sharing through HBM, ideal)."""
    q = 0
    n = len(costs)
    pool = []
    waves = [[np.zeros(64, np.int32) for _ in range(bpc)] for _ in range(NSIMD)]
    ev = [(0.0, s) for s in range(NSIMD)]
    heapq.heapify(ev)
    t_end = 0.0
    drain = None
    while ev:
        t, s = heapq.heappop(ev)
        ws = waves[s]
        mfma, crit = 0.0, 0.0
        any_live = False
        qempty = q >= n
        if qempty and drain is None:
            drain = t
        if qempty and merge_pairs and len(ws) > 1:
            live = np.concatenate([w[w > 0] for w in ws])
            if len(live) <= 64:
                w0 = np.zeros(64, np.int32)
                w0[:len(live)] = live
                ws[:] = [w0]
        for w in ws:
            free = np.flatnonzero(w == 0)
            if len(free) and q < n:
                k = min(len(free), n - q, take)
                w[free[:k]] = costs[q:q + k]
                q += k
            if share and q >= n:
                live = np.flatnonzero(w > 0)
                if len(live) > share:
                    pool.extend(w[live[share:]].tolist())
                    w[live[share:]] = 0
                elif len(live) < share and pool:
                    k = min(share - len(live), len(pool))
                    fr = np.flatnonzero(w == 0)[:k]
                    w[fr] = pool[-k:]
                    del pool[-k:]
            nl = int((w > 0).sum())
            if nl == 0:
                continue
            any_live = True
            if q >= n:   # compaction in the tail
                tiles = (nl + 15) // 16
            else:
                tiles = int((w.reshape(4, 16) > 0).any(axis=1).sum())
            mfma += tiles * T_TILE
            crit = max(crit, tiles * T_TILE + V_WAVE)
        if not any_live:
            if q >= n and not pool:
                t_end = max(t_end, t)
                continue
            heapq.heappush(ev, (t + 0.5, s))
            continue
        R = max(mfma, crit)
        for w in ws:
            w[w > 0] -= 1
        heapq.heappush(ev, (t + R, s))
    return t_end, drain


def simulate_promote(m, age=24, dilate=True, bpc=2):
    """Interleaved dispensing (one pixel of every block per round) with hot-block
    promotion: when a ray reaches `age` iterations its block (and, with `dilate`, the
    8 neighbours) jumps the queue: its remaining pixels are dealt before anything else."""
    H, W = m.shape
    bh, bw = H // 8, W // 8
    nb = bh * bw
    pix = m.reshape(bh, 8, bw, 8).transpose(0, 2, 1, 3).reshape(nb, 64)
    ptr = np.zeros(nb, np.int32)
    hot = np.zeros(nb, bool)
    hotq = []          # blocks, FIFO
    hq = 0
    cur = [0]          # main-queue position (block index cycling)
    left = [int(nb * 64)]

    def take(k):
        nonlocal hq
        out_c, out_b = [], []
        while k > 0 and left[0] > 0:
            if hq < len(hotq):
                b = hotq[hq]
                r = 64 - ptr[b]
                if r <= 0:
                    hq += 1
                    continue
                t = min(r, k)
                out_c.extend(pix[b, ptr[b]:ptr[b] + t]); out_b.extend([b] * t)
                ptr[b] += t; k -= t; left[0] -= t
                continue
            b = cur[0] % nb
            cur[0] += 1
            if ptr[b] < 64:
                out_c.append(pix[b, ptr[b]]); out_b.append(b)
                ptr[b] += 1; k -= 1; left[0] -= 1
        return out_c, out_b

    def promote(b):
        by, bx = divmod(b, bw)
        cand = [b] if not dilate else [(y * bw + x) for y in range(by - 1, by + 2) for x in range(bx - 1, bx + 2)
                                        if 0 <= y < bh and 0 <= x < bw]
        for c in cand:
            if not hot[c]:
                hot[c] = True
                if ptr[c] < 64:
                    hotq.append(c)

    rem = [[np.zeros(64, np.int32) for _ in range(bpc)] for _ in range(NSIMD)]
    cst = [[np.zeros(64, np.int32) for _ in range(bpc)] for _ in range(NSIMD)]
    blk = [[np.zeros(64, np.int32) for _ in range(bpc)] for _ in range(NSIMD)]
    ev = [(0.0, s) for s in range(NSIMD)]
    heapq.heapify(ev)
    t_end, drain = 0.0, None
    while ev:
        t, s = heapq.heappop(ev)
        mfma, crit, any_live = 0.0, 0.0, False
        if left[0] == 0 and drain is None:
            drain = t
        for w, c, bb in zip(rem[s], cst[s], blk[s]):
            free = np.flatnonzero(w == 0)
            if len(free) and left[0] > 0:
                oc, ob = take(len(free))
                k = len(oc)
                w[free[:k]] = oc; c[free[:k]] = oc; bb[free[:k]] = ob
            nl = int((w > 0).sum())
            if nl == 0:
                continue
            any_live = True
            tiles = (nl + 15) // 16 if left[0] == 0 else int((w.reshape(4, 16) > 0).any(axis=1).sum())
            mfma += tiles * T_TILE
            crit = max(crit, tiles * T_TILE + V_WAVE)
        if not any_live:
            if left[0] == 0:
                t_end = max(t_end, t)
                continue
            heapq.heappush(ev, (t + 0.5, s))
            continue
        for w, c, bb in zip(rem[s], cst[s], blk[s]):
            w[w > 0] -= 1
            aged = np.flatnonzero((w > 0) & (c - w == age))
            for i in aged:
                if not hot[bb[i]]:
                    promote(int(bb[i]))
        heapq.heappush(ev, (t + max(mfma, crit), s))
    return t_end, drain


def main():
    m = np.load(sys.argv[1]).astype(np.int32)
    H, W = m.shape
    bmax = m.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
    cases = [
        ("block-major", block_order(m), 2, False),
        ("spread16", spread_order(m, 16), 2, False),
        ("spread16 bpc3", spread_order(m, 16), 3, False),
        ("temporal", block_order(m, bmax), 2, False),
        ("temporal bpc3", block_order(m, bmax), 3, False),
        ("spread16 merge", spread_order(m, 16), 2, True),
        ("spread16 bpc3 merge", spread_order(m, 16), 3, True),
        ("spread16 share16", spread_order(m, 16), 2, 16),
        ("spread16 share8", spread_order(m, 16), 2, 8),
        ("spread16 bpc3 share16", spread_order(m, 16), 3, 16),
        ("spread16 bpc3 share32", spread_order(m, 16), 3, 32),
    ]
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for name, costs, bpc, merge in cases:
        if only and name not in only:
            continue
        t, d = simulate(costs, bpc, merge is True, share=merge if not isinstance(merge, bool) else 0)
        print(f"{name:24s} frame {t / 1e3:.3f} ms  drain {d / 1e3:.3f} ms  tail {(t - d) / 1e3:.3f} ms", flush=True)
    for age, dil in [(16, True), (24, True), (32, True), (24, False)]:
        t, d = simulate_promote(m, age, dil)
        print(f"promote age {age} dilate {dil}: frame {t / 1e3:.3f} ms  drain {d / 1e3:.3f} ms  tail {(t - d) / 1e3:.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
