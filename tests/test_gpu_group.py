"""Multi-GPU frames from one process behind the C ABI (nr_group, csrc/nr_group.hip): row-band
shards rendered by one context per GPU, one RCCL gather, one re-interleave.  The box has one
GPU, so the group has one rank here (the RCCL send/recv to itself still runs); the 2- and 3-rank
assembly of the same layout is checked on gloo (tests/test_dist_cpu.py) and the shards
themselves on one GPU (test_gpu_parity.py)."""
import numpy as np
import pytest

import cudaneuralrender_amd as nr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_group_one_rank_equals_render(prec):
    chrome = nr.load_png(nr.matcap_path("Chrome"))
    cams = [(*nr.camera(-10.0 + 5 * i, 20.0 + 33 * i, 2.0), i) for i in range(3)]
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path("plane_1")).set_precision(prec)
        r.set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        refs = []
        for iv, nm, f in cams:
            r.set_view(iv, nm, f)
            refs.append(r.render(200, 131, 128))
        with nr.Group([r]) as g:
            assert g.size() == 1
            for band in (1, 8):
                imgs, st = g.render_batch(200, 131, cams, 128, band=band)
                assert all(np.array_equal(a, b[0]) for a, b in zip(imgs, refs)), band
                assert st["ray_steps"] == sum(b[1]["ray_steps"] for b in refs)


def test_group_rejects_two_contexts_on_one_gpu():
    with nr.Renderer(0) as a, nr.Renderer(0) as b:
        with pytest.raises(nr.NRError):
            nr.Group([a, b])


def test_group_shard_failure_returns_error_before_the_gather():
    """A shard whose render fails (here: no network loaded) ends the call with its error; no
    collective is started (a later valid call still works)."""
    with nr.Renderer(0) as r:
        with nr.Group([r]) as g:
            iv, nm = nr.camera(0, 0, 2)
            with pytest.raises(nr.NRError, match="shard 0"):
                g.render_batch(32, 32, [(iv, nm, 0)], 64)
            r.load_h5(nr.geometry_path("plane_1")).set_static(nr.NR_COLOR_FACING, 3).set_scene("v1")
            imgs, _ = g.render_batch(32, 32, [(iv, nm, 0)], 64)
            r.set_view(iv, nm, 0)
            assert np.array_equal(imgs[0], r.render(32, 32, 64)[0])
