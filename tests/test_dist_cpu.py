"""Multi-rank plumbing of the sharded frame on CPU (gloo, world size 2 and 3).

Each rank produces its row-band shards of n frames (the rows nr_render_shard /
nr_render_batch render: bands of `band` rows dealt round-robin), rank 0 gathers the
n frames' shards in one torch.distributed.gather and re-interleaves each frame with
nr_assemble_shards -- the same sequence and buffer layout bench.py runs over RCCL.  The shard content comes from the CPU oracle's full frame (test stand-in for
the GPU render, whose shard == rows-of-full-frame property is a GPU test)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, band, W, H, nframes, result_path):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "oracle"))
    import torch
    import torch.distributed as dist

    import cudaneuralrender_amd as nr
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dims, K, B = nr.read_keras_h5(nr.geometry_path("plane_1"))
    fulls = []
    for f in range(nframes):   # frames of a short camera orbit
        iv, nm = nr.camera(-10.0, 25.0 + 40.0 * f, 2.0)
        fulls.append(oracle.OracleNet(K, B).render(W, H, iv, nm, color_type=0, max_steps=64, nthreads=2)[0])
    rows = [y for y in range(H) if (y // band) % world == rank]
    assert len(rows) == nr.shard_rows(H, band, world, rank)
    max_rows = max(nr.shard_rows(H, band, world, s) for s in range(world))
    shard_px = max_rows * W
    # bench.py's layout: this rank's shards of the n frames back to back, ONE gather
    buf = torch.zeros(nframes, shard_px, dtype=torch.int64)
    for f in range(nframes):
        buf[f, : len(rows) * W] = torch.from_numpy(fulls[f][rows].astype(np.int64).reshape(-1))
    gl = [torch.zeros(nframes * shard_px, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
    dist.gather(buf.reshape(-1), gl, dst=0)
    if rank == 0:
        flat = torch.stack(gl).numpy().astype(np.uint32).reshape(-1)
        out = []
        for f in range(nframes):
            # frame f of shard s at flat[s * nframes * shard_px + f * shard_px]
            src = flat[f * shard_px:]
            shards = [src[s * nframes * shard_px: s * nframes * shard_px + shard_px].reshape(max_rows, W)
                      for s in range(world)]
            out.append(nr.assemble_shards(shards, W, H, band, world))
        if H % (band * world) == 0:
            # bench.py's single assembly: when every frame is a whole number of band rounds,
            # the n frames stacked are one (n*H)-row image whose shard s is rank s's gathered
            # n x max_rows rows
            stacked = [flat[s * nframes * shard_px:(s + 1) * nframes * shard_px].reshape(nframes * max_rows, W)
                       for s in range(world)]
            one = nr.assemble_shards(stacked, W, nframes * H, band, world).reshape(nframes, H, W)
            assert np.array_equal(one, np.stack(out))
        np.save(result_path, np.stack([np.stack(out), np.stack(fulls)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band,nframes,H", [(2, 8, 1, 41), (3, 5, 1, 41), (2, 8, 3, 41), (3, 1, 2, 41),
                                                (2, 1, 3, 41), (2, 1, 3, 48), (3, 1, 4, 48), (2, 8, 2, 48)])
def test_gloo_gather_assemble(tmp_path, world, band, nframes, H):
    import torch.multiprocessing as mp
    W = 48
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), band, W, H, nframes, out), nprocs=world, join=True)
    frames, fulls = np.load(out)
    assert np.array_equal(frames, fulls)
    assert (fulls != 0).sum() > 0


def _fail_worker(rank, world, port, bad, result_dir):
    """bench.py's per-batch step on gloo: rank `bad` raises inside its render; every rank then
    reaches the gather only if the status all-reduce says every rank rendered."""
    import sys
    import time
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import torch
    import torch.distributed as dist

    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = torch.full((16,), rank, dtype=torch.int64)
    batch = [0]

    def render():
        batch[0] += 1
        if rank == bad and batch[0] == 2:
            raise RuntimeError("nr_render_batch failed (injected)")
        buf.add_(1)

    t0 = time.time()
    outcome = "gathered"
    try:
        for _ in range(3):      # three batches: the failure comes in the second
            bench.checked_step(dist, world, "cpu", render)
            gl = [torch.zeros(16, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
            dist.gather(buf, gl, dst=0)
    except bench.RankFailed:
        outcome = "RankFailed"
    except RuntimeError as e:
        outcome = "own error" if "injected" in str(e) else f"other: {e}"
    with open(os.path.join(result_dir, f"rank{rank}"), "w") as f:
        f.write(f"{outcome} {time.time() - t0:.2f}")


@pytest.mark.parametrize("world,bad", [(2, 1), (2, 0), (3, 2)])
def test_failed_rank_fails_fast(tmp_path, world, bad):
    """a rank whose render raises must not leave the others blocked in the gather.
    With bench.checked_step before every gather, the failing rank re-raises its error and every
    other rank raises RankFailed, all within seconds (the gloo default timeout is 30 minutes)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, bad, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank is still blocked"
    res = {r: open(tmp_path / f"rank{r}").read().split() for r in range(world)}
    for r in range(world):
        want = "own" if r == bad else "RankFailed"
        assert res[r][0] == want, res
        assert float(res[r][-1]) < 60, res


@pytest.mark.parametrize("n,band,nframes,H", [(2, 1, 3, 131), (3, 8, 3, 131), (3, 5, 2, 41), (2, 8, 1, 7),
                                              (8, 1, 4, 1024), (3, 1, 1, 1)])
def test_group_layout_reassembles(n, band, nframes, H):
    """nr_group_render_batch's gather layout (nr_group_layout: frame i's shard at i * shard_px of
    every rank's set, rank r's set at r * per_rank) re-interleaved the way it calls the kernel --
    nr_assemble_shards from gather + i * shard_px with stride per_rank -- gives every frame back,
    uneven shards (shard_px from shard 0 while the others hold fewer rows) included."""
    import cudaneuralrender_amd as nr
    W = 37
    rng = np.random.default_rng(n * 100 + band)
    fulls = rng.integers(1, 2**32, size=(nframes, H, W), dtype=np.uint64).astype(np.uint32)
    shard_px, per_rank = nr.group_layout(W, H, band, n, nframes)
    assert shard_px == nr.shard_rows(H, band, n, 0) * W and per_rank == shard_px * nframes
    assert all(nr.shard_rows(H, band, n, s) * W <= shard_px for s in range(n))
    gather = np.zeros(n * per_rank, np.uint32)
    for r in range(n):
        rows = [y for y in range(H) if (y // band) % n == r]
        for i in range(nframes):   # rank r's set: frame i's shard rows at i * shard_px
            o = r * per_rank + i * shard_px
            gather[o:o + len(rows) * W] = fulls[i][rows].reshape(-1)
    L = nr.lib()
    for i in range(nframes):
        out = np.zeros((H, W), np.uint32)
        src = gather[i * shard_px:]
        assert L.nr_assemble_shards(None, src.ctypes.data, per_rank, out.ctypes.data, W, H, band, n, 0) == 0
        assert np.array_equal(out, fulls[i]), (n, band, i)
