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
