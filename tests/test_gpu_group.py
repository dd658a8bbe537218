"""Multi-GPU frames from one process behind the C ABI (nr_group, csrc/nr_group.hip): row-band
shards rendered by one context per rank, one gather, one re-interleave per frame.

  * RCCL groups over every visible GPU count from 1 up (ncclCommInitAll, grouped ncclSend /
    ncclRecv over xGMI): the 1-rank group runs on any box, N > 1 wherever the box has N GPUs
    (skipped otherwise);
  * NR_GROUP_COPY groups of 2 and 3 contexts that share GPU 0 (hipMemcpyPeerAsync transfers): the
    same layout, uneven shards, threads and re-interleave as the RCCL path, on a one-GPU box;
  * NR_GROUP_ASYNC: consecutive calls overlap (call k + 1 renders while call k's shards travel,
    double-buffered), every frame of every call identical after nr_group_synchronize.
Every frame must equal the single-context nr_render of its camera, bit for bit, and the stats
the sum of the shards'.  The CPU side of the layout: tests/test_dist_cpu.py
test_group_layout_reassembles."""
import numpy as np
import pytest
import torch

import cudaneuralrender_amd as nr

pytestmark = pytest.mark.gpu
NGPU = torch.cuda.device_count()


def _setup(r, prec, chrome):
    r.load_h5(nr.geometry_path("plane_1")).set_precision(prec)
    r.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
    return r


def _refs(r, cams, W, H, steps):
    out = []
    for iv, nm, f in cams:
        r.set_view(iv, nm, f)
        out.append(r.render(W, H, steps))
    return out


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_group_rccl_equals_render(chrome, prec, n):
    if n > NGPU:
        pytest.skip(f"{n} GPUs needed, {NGPU} visible")
    cams = [(*nr.camera(-10.0 + 5 * i, 20.0 + 33 * i, 2.0), i) for i in range(3)]
    rs = [_setup(nr.Renderer(d), prec, chrome) for d in range(n)]
    try:
        refs = _refs(rs[0], cams, 200, 131, 128)
        with nr.Group(rs) as g:
            assert g.size() == n
            for band in (1, 8):
                imgs, st = g.render_batch(200, 131, cams, 128, band=band)
                assert all(np.array_equal(a, b[0]) for a, b in zip(imgs, refs)), band
                assert st["ray_steps"] == sum(b[1]["ray_steps"] for b in refs)
    finally:
        for r in rs:
            r.close()


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("n", [2, 3])
def test_group_copy_multi_rank_on_one_gpu(chrome, prec, n):
    """n contexts on GPU 0 joined with NR_GROUP_COPY: uneven shards (131 rows), bands 1 / 8 / 5,
    host and device outputs."""
    cams = [(*nr.camera(7.0 * i, 15.0 + 29 * i, 2.1), 2 * i) for i in range(4)]
    rs = [_setup(nr.Renderer(0), prec, chrome) for _ in range(n)]
    try:
        refs = _refs(rs[0], cams, 200, 131, 128)
        with nr.Group(rs, copy=True) as g:
            for band in (1, 8, 5):
                imgs, st = g.render_batch(200, 131, cams, 128, band=band)
                for i, (a, b) in enumerate(zip(imgs, refs)):
                    assert np.array_equal(a, b[0]), (band, i, int((a != b[0]).sum()))
                assert st["ray_steps"] == sum(b[1]["ray_steps"] for b in refs)
            outs = torch.zeros(len(cams), 131 * 200, dtype=torch.int32, device="cuda")
            g.render_batch_device([o.data_ptr() for o in outs], 200, 131, cams, 128, band=1)
            torch.cuda.synchronize()
            for o, b in zip(outs, refs):
                assert np.array_equal(o.cpu().numpy().view(np.uint32).reshape(131, 200), b[0])
    finally:
        for r in rs:
            r.close()


@pytest.mark.parametrize("asynchronous", [False, True])
def test_group_copy_over_distinct_gpus(chrome, asynchronous):
    """NR_GROUP_COPY with its contexts on different GPUs (the COPY-mode events are
    created on GPU 0 and waited on by every rank's streams): 2 ranks on GPUs 0 and 1, host and
    device outputs, synchronous and NR_GROUP_ASYNC.  Needs 2 GPUs (skipped on a one-GPU box)."""
    if NGPU < 2:
        pytest.skip(f"2 GPUs needed, {NGPU} visible")
    cams = [(*nr.camera(5.0 * i, 12.0 + 31 * i, 2.0), i) for i in range(3)]
    rs = [_setup(nr.Renderer(d), "fp32", chrome) for d in (0, 1)]
    try:
        refs = _refs(rs[0], cams, 200, 131, 128)
        with nr.Group(rs, copy=True, asynchronous=asynchronous) as g:
            imgs, _ = g.render_batch(200, 131, cams, 128, band=1)
            assert all(np.array_equal(a, b[0]) for a, b in zip(imgs, refs))
            outs = torch.zeros(len(cams), 131 * 200, dtype=torch.int32, device="cuda:0")
            g.render_batch_device([o.data_ptr() for o in outs], 200, 131, cams, 128, band=8)
            g.synchronize()
            torch.cuda.synchronize()
            for o, b in zip(outs, refs):
                assert np.array_equal(o.cpu().numpy().view(np.uint32).reshape(131, 200), b[0])
    finally:
        for r in rs:
            r.close()


def test_group_async_calls_overlap_and_stay_exact(chrome):
    """NR_GROUP_ASYNC: five calls back to back (set k & 1 reused every other call, its render
    waiting on the transfer of the call before last), then one synchronize: every frame of every
    call equals its single render."""
    n = min(max(NGPU, 2), 3)
    devs = list(range(n)) if NGPU >= n else [0] * n
    rs = [_setup(nr.Renderer(d), "fp32", chrome) for d in devs]
    calls = [[(*nr.camera(3.0 * k, 40.0 * k + 11 * i, 2.0), k) for i in range(2)] for k in range(5)]
    try:
        refs = [_refs(rs[0], cams, 160, 96, 96) for cams in calls]
        outs = torch.zeros(5, 2, 96 * 160, dtype=torch.int32, device="cuda:0")
        with nr.Group(rs, copy=NGPU < n, asynchronous=True) as g:
            for k, cams in enumerate(calls):
                g.render_batch_device([o.data_ptr() for o in outs[k]], 160, 96, cams, 96, band=1)
            g.synchronize()
        for k in range(5):
            for i in range(2):
                got = outs[k, i].cpu().numpy().view(np.uint32).reshape(96, 160)
                assert np.array_equal(got, refs[k][i][0]), (k, i)
    finally:
        for r in rs:
            r.close()


def test_group_async_host_outputs_are_complete_on_return(chrome):
    """NR_GROUP_ASYNC with host outputs: the call returns with the frames written (no
    nr_group_synchronize needed), call after call."""
    n = min(max(NGPU, 2), 3)
    devs = list(range(n)) if NGPU >= n else [0] * n
    rs = [_setup(nr.Renderer(d), "fp32", chrome) for d in devs]
    calls = [[(*nr.camera(9.0 * k, 30.0 * k + 7 * i, 2.0), k) for i in range(2)] for k in range(3)]
    try:
        with nr.Group(rs, copy=NGPU < n, asynchronous=True) as g:
            for cams in calls:
                imgs, _ = g.render_batch(128, 80, cams, 96, band=1)
                refs = _refs(rs[0], cams, 128, 80, 96)
                for a, b in zip(imgs, refs):
                    assert np.array_equal(a, b[0])
    finally:
        for r in rs:
            r.close()


def test_group_rejects_two_contexts_on_one_gpu_without_copy():
    with nr.Renderer(0) as a, nr.Renderer(0) as b:
        with pytest.raises(nr.NRError):
            nr.Group([a, b])
        with pytest.raises(nr.NRError):
            nr.Group([a, a], copy=True)


def test_group_shard_failure_returns_error_before_the_gather():
    """A shard whose render fails (here: no network loaded on rank 1) ends the call with its error;
    no transfer is started (a later valid call still works)."""
    with nr.Renderer(0) as r0, nr.Renderer(0) as r1:
        r0.load_h5(nr.geometry_path("plane_1")).set_static(nr.NR_COLOR_FACING, 3).set_scene("v1")
        with nr.Group([r0, r1], copy=True) as g:
            iv, nm = nr.camera(0, 0, 2)
            with pytest.raises(nr.NRError, match="shard 1"):
                g.render_batch(32, 32, [(iv, nm, 0)], 64)
            r1.load_h5(nr.geometry_path("plane_1")).set_static(nr.NR_COLOR_FACING, 3).set_scene("v1")
            imgs, _ = g.render_batch(32, 32, [(iv, nm, 0)], 64)
            r0.set_view(iv, nm, 0)
            assert np.array_equal(imgs[0], r0.render(32, 32, 64)[0])
