"""Bounded search for the shading that produced the reference's own renders
(/root/reference/neuralGeometries/{plane_1,car_1}.h5.ppm).

Every foreground pixel of those renders is an exact texel of skin-matcap.png / Car Paint
Red.png, so a shading variant is scored by how many golden foreground pixels
carry the colour of the texel the variant picks (exactly, or anywhere within a (2r+1)^2 texel
window for r = 2, which absorbs the small error of the camera recovered from the silhouette).

The CPU oracle renders the pure-neural scene at the recovered camera with a coordinate-encoding
matcap (texel (tx, ty) holds tx, ty in its bytes), which returns the texel matCapColor
(volumeRender_kernel.cu:387-413) picks for each pixel; with the normal matrix of the camera that
gives the view-space normal ne (x, y from the texel, z >= 0 facing the eye) and the world-space
normal n.  Variants: the texel from ne or n, each axis from x / y / z of it, flipped or not
(u = (c . 0.5 + 0.5)(mw - 1), or 1 - that), and the uv swap.  Needs /root/reference (runs in the
build container, not on the GPU box); writes a summary to stdout.

    python tools/shading_search.py [--res 256]"""
import argparse
import itertools
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import cudaneuralrender_amd as nr  # noqa: E402
import oracle  # noqa: E402

REF = "/root/reference/neuralGeometries"


def read_ppm(path):
    """P6 reader (the header is whitespace-separated tokens, sdkSavePPM4ub)"""
    data = open(path, "rb").read()
    toks, pos = [], 0
    while len(toks) < 4:
        while data[pos:pos + 1].isspace():
            pos += 1
        end = pos
        while not data[end:end + 1].isspace():
            end += 1
        toks.append(data[pos:end])
        pos = end
    w, h = int(toks[1]), int(toks[2])
    return np.frombuffer(data, np.uint8, w * h * 3, pos + 1).reshape(h, w, 3)


# cameras: refined from SURVEY App. A by maximising the silhouette IoU (tools/camera_fit.py)
CASES = {"plane_1": ("skin-matcap", (-18.8021, 149.7984, 2.2702)), "car_1": ("Car Paint Red", (80.047, 140.0488, 3.1031))}

ap = argparse.ArgumentParser()
ap.add_argument("--res", type=int, default=256)
ap.add_argument("--radius", type=int, default=2)
a = ap.parse_args()


def rgb(img):
    return np.stack([(img >> (8 * c)) & 0xff for c in range(3)], -1).astype(np.int32)


for name, (mc, (rx, ry, zoom)) in CASES.items():
    gold = read_ppm(os.path.join(REF, name + ".h5.ppm")).astype(np.int32)  # [1024, 1024, 3]
    k = gold.shape[0] // a.res
    gold = gold[::k, ::k]
    gfg = gold.any(-1)
    matcap = nr.load_png(nr.matcap_path(mc))
    mh, mw = matcap.shape
    mrgb = rgb(matcap)
    # coordinate matcap: r = tx & 255, g = ty & 255, b = (tx >> 8) | (ty >> 8) << 4, alpha 255
    ty, tx = np.mgrid[0:mh, 0:mw]
    coord = (255 << 24 | (((tx >> 8) | ((ty >> 8) << 4)) << 16) | ((ty & 255) << 8) | (tx & 255)).astype(np.uint32)
    iv, nm = nr.camera(rx, ry, zoom)
    dims, K, B = nr.read_keras_h5(nr.geometry_path(name))
    img, st = oracle.OracleNet(K, B).render(a.res, a.res, iv, nm, color_type=1, matcap=coord, scene=1,
                                            max_steps=6000, nthreads=8)
    fg = img != 0
    both = fg & gfg
    ptx = (img & 255) | (((img >> 16) & 15) << 8)
    pty = ((img >> 8) & 255) | (((img >> 20) & 15) << 8)
    # view-space normal from the texel (matCapColor: texel = (ne.x .5 + .5)(mw - 1)); z >= 0
    nex = ptx[both] / (mw - 1) * 2 - 1
    ney = pty[both] / (mh - 1) * 2 - 1
    nez = np.sqrt(np.clip(1 - nex ** 2 - ney ** 2, 0, 1))
    ne = np.stack([nex, ney, nez], -1)
    N = np.asarray(nm, np.float64).reshape(4, 4)[:3, :3]  # ne = normalize(N n)
    nw = ne @ np.linalg.inv(N).T
    nw /= np.linalg.norm(nw, axis=1, keepdims=True)
    g = gold[both]
    print(f"{name}: {a.res}^2, coverage IoU {(fg & gfg).sum() / (fg | gfg).sum():.4f}, "
          f"{both.sum()} pixels in both; matcap {mc} {mw}x{mh}")

    def score(u, v):
        """fraction of pixels whose golden colour is the texel at (u, v) (exact), or within radius"""
        ix = np.clip(np.floor(u * (mw - 1)).astype(int), 0, mw - 1)
        iy = np.clip(np.floor(v * (mh - 1)).astype(int), 0, mh - 1)
        exact = (mrgb[iy, ix] == g).all(-1).mean()
        near = np.zeros(len(g), bool)
        r = a.radius
        for dy in range(-r, r + 1):
            for dx in range(-r, r + 1):
                near |= (mrgb[np.clip(iy + dy, 0, mh - 1), np.clip(ix + dx, 0, mw - 1)] == g).all(-1)
        return exact, near.mean()

    res = []
    nt = nw @ N  # the transpose of the normal matrix applied (rows: N^T n)
    nt /= np.linalg.norm(nt, axis=1, keepdims=True)
    for space, vec in (("view", ne), ("world", nw), ("viewT", nt)):
        for (cu, cv) in itertools.permutations(range(3), 2):
            for fu, fv in itertools.product((False, True), repeat=2):
                u = vec[:, cu] * 0.5 + 0.5
                v = vec[:, cv] * 0.5 + 0.5
                u = 1 - u if fu else u
                v = 1 - v if fv else v
                e, n_ = score(u, v)
                res.append((n_, e, f"{space:5s} u={'-' if fu else '+'}{'xyz'[cu]} v={'-' if fv else '+'}{'xyz'[cv]}"))
    # sphere-map variants on the reflected view ray (camera space: the eye looks down -z; the
    # pixel's direction normalize(u, v, -2), initMarcher :315-320): r = d - 2 (d . n) n,
    # m = 2 sqrt(r.x^2 + r.y^2 + (r.z + 1)^2), uv = r.xy / m + 1/2 (flips included)
    yy, xx = np.nonzero(both)
    du = xx / a.res * 2 - 1
    dv = yy / a.res * 2 - 1
    dc = np.stack([du, dv, -2 * np.ones_like(du)], -1)
    dc /= np.linalg.norm(dc, axis=1, keepdims=True)
    for zs in (1, -1):
        r_ = dc - 2 * (dc * ne).sum(1, keepdims=True) * ne
        m = 2 * np.sqrt(r_[:, 0] ** 2 + r_[:, 1] ** 2 + (r_[:, 2] + zs) ** 2)
        for fu, fv in itertools.product((False, True), repeat=2):
            for sw in (False, True):
                u, v = r_[:, 0] / m + 0.5, r_[:, 1] / m + 0.5
                if sw:
                    u, v = v, u
                u = 1 - u if fu else u
                v = 1 - v if fv else v
                e, n_ = score(u, v)
                res.append((n_, e, f"spheremap(z{'+' if zs > 0 else '-'}1) {'swap ' if sw else ''}"
                                   f"u{'-' if fu else '+'} v{'-' if fv else '+'}"))
    res.sort(reverse=True)
    for n_, e, lab in res[:8]:
        print(f"   {lab}: exact {e:.4f}  within {a.radius} texels {n_:.4f}")
    # how many golden pixels match ANY texel within the window of the best variant's texel is
    # bounded by how often a colour recurs: the chance level of the window test
    rng = np.random.default_rng(0)
    e, n_ = score(rng.uniform(0, 1, len(g)), rng.uniform(0, 1, len(g)))
    print(f"   random texels (chance level): exact {e:.4f}  within {a.radius} texels {n_:.4f}")

    # data-driven: the texel from (R n)_x, (R n)_y for a rotation R of the world normal (any
    # camera convention, mirror or axis order is some R, with det -1 for mirrors): coarse grid
    # over ZYZ Euler angles, then a local refinement of the best
    def rot(a1, a2, a3):
        def rz(t):
            c, s = np.cos(t), np.sin(t)
            return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])

        def ry_(t):
            c, s = np.cos(t), np.sin(t)
            return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
        return rz(a1) @ ry_(a2) @ rz(a3)

    def rscore(R):
        m = nw @ R.T
        return score(m[:, 0] * 0.5 + 0.5, m[:, 1] * 0.5 + 0.5)[1]

    best = []
    for mirror in (1, -1):
        Mx = np.diag([mirror, 1, 1])
        for a1 in np.radians(np.arange(0, 360, 20)):
            for a2 in np.radians(np.arange(0, 181, 20)):
                for a3 in np.radians(np.arange(0, 360, 20)):
                    R = Mx @ rot(a1, a2, a3)
                    best.append((rscore(R), mirror, a1, a2, a3))
    best.sort(reverse=True)
    s0, mirror, a1, a2, a3 = best[0]
    step = np.radians(10)
    while step > np.radians(0.5):
        improved = False
        for d in itertools.product((-1, 0, 1), repeat=3):
            c = (a1 + d[0] * step, a2 + d[1] * step, a3 + d[2] * step)
            sc = rscore(np.diag([mirror, 1, 1]) @ rot(*c))
            if sc > s0:
                s0, (a1, a2, a3), improved = sc, c, True
        if not improved:
            step /= 2
    R = np.diag([mirror, 1, 1]) @ rot(a1, a2, a3)
    m = nw @ R.T
    e, n_ = score(m[:, 0] * 0.5 + 0.5, m[:, 1] * 0.5 + 0.5)
    print(f"   best rotation of the world normal (mirror {mirror}, ZYZ {np.degrees([a1, a2, a3]).round(1)}): "
          f"exact {e:.4f}  within {a.radius} texels {n_:.4f}; R =\n{np.round(R, 3)}")
