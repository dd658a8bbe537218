"""Multi-rank plumbing of the sharded frame on CPU (gloo, world size 2 and 3).

Each rank produces its row-band shard (the rows nr_render_shard renders: bands of
`band` rows dealt round-robin), rank 0 gathers them with torch.distributed.gather and
re-interleaves them with nr_assemble_shards -- the same sequence bench.py runs over
RCCL.  The shard content comes from the CPU oracle's full frame (test stand-in for
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


def _worker(rank, world, port, band, W, H, result_path):
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
    iv, nm = nr.camera(-10.0, 25.0, 2.0)
    full, _ = oracle.OracleNet(K, B).render(W, H, iv, nm, color_type=0, max_steps=64, nthreads=2)
    rows = [y for y in range(H) if (y // band) % world == rank]
    assert len(rows) == nr.shard_rows(H, band, world, rank)
    max_rows = max(nr.shard_rows(H, band, world, s) for s in range(world))
    buf = torch.zeros(max_rows * W, dtype=torch.int64)
    buf[: len(rows) * W] = torch.from_numpy(full[rows].astype(np.int64).reshape(-1))
    gl = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gl, dst=0)
    if rank == 0:
        shards = [g.numpy().astype(np.uint32) for g in gl]
        frame = nr.assemble_shards(shards, W, H, band, world)
        np.save(result_path, np.stack([frame, full]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 8), (3, 5)])
def test_gloo_gather_assemble(tmp_path, world, band):
    import torch.multiprocessing as mp
    W, H = 48, 41
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), band, W, H, out), nprocs=world, join=True)
    frame, full = np.load(out)
    assert np.array_equal(frame, full)
    assert (full != 0).sum() > 0
