"""Threading contract (neural_render.h header; SURVEY.md §8(b) "one ctx per GPU, different
contexts are thread-safe"): two contexts on one device, each driven from its own host thread
at the same time (ctypes releases the GIL inside every libnr call), render exactly what each
renders alone.  The reference keeps its render state in process globals
(volumeRender_kernel.cu:31-35, :578-585) and could not do this."""
import threading

import numpy as np
import pytest

import cudaneuralrender_amd as nr

pytestmark = pytest.mark.gpu


def make(geom, prec, scene, color, chrome):
    r = nr.Renderer(0).load_h5(nr.geometry_path(geom)).set_precision(prec)
    r.set_static(color, 3).set_scene(scene).set_matcap(chrome)
    return r


def test_two_contexts_two_threads(chrome):
    cams = [(*nr.camera(10.0 * i, 37.0 * i, 2.0 + 0.1 * i), i) for i in range(6)]
    jobs = [("plane_1", "fp32", "v1", nr.NR_COLOR_MATCAP), ("car_1", "bf16", "tanh", nr.NR_COLOR_FACING)]
    rends = [make(*j, chrome) for j in jobs]
    try:
        # alone, one context at a time
        alone = []
        for r in rends:
            out = []
            for iv, nm, f in cams:
                r.set_view(iv, nm, f)
                out.append(r.render(200, 150, 128))
            out.append(r.render_batch(200, 150, cams, 128))
            out.append(r.mlp_forward(np.random.default_rng(1).uniform(-1, 1, (5000, 3)).astype(np.float32)))
            alone.append(out)
        # together: both threads issue all their work at once, three rounds
        results = [[None] * 3 for _ in rends]
        errors = []
        start = threading.Barrier(len(rends))

        def work(k):
            try:
                r = rends[k]
                start.wait()
                for rnd in range(3):
                    out = []
                    for iv, nm, f in cams:
                        r.set_view(iv, nm, f)
                        out.append(r.render(200, 150, 128))
                    out.append(r.render_batch(200, 150, cams, 128))
                    out.append(r.mlp_forward(np.random.default_rng(1).uniform(-1, 1, (5000, 3)).astype(np.float32)))
                    results[k][rnd] = out
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append((k, repr(e)))

        ts = [threading.Thread(target=work, args=(k,)) for k in range(len(rends))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in ts), "a render thread hung"
        assert not errors, errors
        for k in range(len(rends)):
            for rnd in range(3):
                got = results[k][rnd]
                for i in range(len(cams)):
                    (img, st), (ref, rst) = got[i], alone[k][i]
                    assert np.array_equal(img, ref), (k, rnd, i)
                    assert st["ray_steps"] == rst["ray_steps"]
                (bimgs, bst), (brefs, brst) = got[len(cams)], alone[k][len(cams)]
                assert all(np.array_equal(a, b) for a, b in zip(bimgs, brefs)), (k, rnd)
                assert bst["ray_steps"] == brst["ray_steps"]
                assert np.array_equal(got[-1], alone[k][-1]), (k, rnd)
        # single-frame renders of a batch's cameras equal the batch (cross-check of the two paths)
        for k in range(len(rends)):
            assert all(np.array_equal(alone[k][i][0], alone[k][len(cams)][0][i]) for i in range(len(cams)))
    finally:
        for r in rends:
            r.close()


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))
