"""Pixel contract of the reduced-precision configurations (BASELINE C3-C5) against the oracle.

The oracle marches with the GPU's bf16/fp16 MLP arithmetic (oracle/nr_oracle.c
mlp_point_gpu_lowp: 16-bit operands rounded as the kernels round them, each MFMA / dot2 step an
exact sum rounded once to f32 -- the hardware's internal summation order is not documented,
so this is an emulation, not a bit-exact restatement) and fp32 normals, on a row crop of the
full-size frame (the same rays as the full frame).  Per crop we report the identical-pixel
fraction, the per-channel mean and max |delta| over pixels both sides cover, the coverage IoU,
and the same figures against the fp32 oracle (what reduced precision costs in total).

Contract, per configuration crop, against the emulation:
                      bf16 (C3, C4)   fp16 (C5)     measured r2 (profiles/r2_lowp_contract.json)
  identical pixels    >= 99.9 %       >= 98 %       bf16 99.97-99.99 %, fp16 98.7-99.9 %
  coverage IoU        >= 0.9999       >= 0.995      bf16 >= 0.99996, fp16 >= 0.9978
  mean |delta|/chan.  <= 0.02         <= 0.3        bf16 0.006, fp16 0.05-0.21 (of 255)
and the emulation must be closer to the GPU than the fp32 oracle is (fp32: 76-99 % identical,
mean |delta| 1.2-10).

Quality bound: what reduced precision costs is measured against the oracle's
exact-MLP frame (precision 3, oracle/nr_oracle.c mlp_point_f64: the whole network in f64,
only the SDF rounded to f32 -- the network as written, not as any f32 or 16-bit machine
evaluates it).  Per precision:
                      bf16 (C3, C4)   fp16 (C5)     measured r4 (profiles/r4_lowp_contract.json)
  identical pixels    >= 0.72         >= 0.75       bf16 0.760 / 0.849, fp16 0.789-0.993
  coverage IoU        >= 0.90         >= 0.78       bf16 0.998 / 0.931, fp16 0.817-0.997
  mean |delta|/chan.  <= 12           <= 3.2        bf16 5.44 / 10.24, fp16 1.15-2.72
and per crop no worse than r4's figure by more than 2 points of identical pixels, 0.01 of IoU
or 1.25x the mean |delta| (EXACT_R4).  For scale, the fp32 MLP itself (fp32 oracle vs exact)
is 89-99.8 % identical, IoU >= 0.9995, mean |delta| 0.34-1.33, and the fp32 oracle built with
and without FMA contraction differs in 1-4 % of its pixels (profiles/r2_fp32_contraction_drift.txt).
A single differing MLP rounding moves one ray's step, which can change its pixel completely
(a silhouette ray hits or misses, a grazing ray converges one step later), so max |delta| is
reported, not bounded."""
import json
import os

import numpy as np
import pytest

import cudaneuralrender_amd as nr
import oracle
from conftest import GEOMS, REPO
from conftest import compare_frames as compare

pytestmark = pytest.mark.gpu
PREC = {"bf16": 1, "fp16": 2}


@pytest.fixture(scope="module")
def chrome():
    return nr.load_png(nr.matcap_path("Chrome"))


def contract(name, geom, size, steps, prec, rows, chrome, record):
    dims, K, B = nr.read_keras_h5(nr.geometry_path(geom))
    iv, nm = nr.camera(0.0, 0.0, 2.0)
    with nr.Renderer(0) as r:
        r.load_h5(nr.geometry_path(geom)).set_precision(prec)
        r.set_view(iv, nm, 0).set_static(nr.NR_COLOR_MATCAP, 3).set_scene("v1").set_matcap(chrome)
        img, st = r.render(size, size, steps)
    gpu = img[rows[0]:rows[1]]
    # the emulation computes the normals as the bf16/fp16 tracers do: fp32x3 from the library's pack
    # (nr_pack_x3; nr_oracle.c mlp_point_gpu_x3), fp32 where the pack is not valid
    pack = nr.pack_x3(dims, K, B)
    net = oracle.OracleNet(K, B, x3_pack=pack[:2] if pack[2] else None)
    kw = dict(color_type=1, matcap=chrome, max_steps=steps, nthreads=16, rows=rows)
    emu, _ = net.render(size, size, iv, nm, precision=PREC[prec], **kw)
    f32, _ = net.render(size, size, iv, nm, precision=0, **kw)
    exact, _ = net.render(size, size, iv, nm, precision=3, **kw)
    res = {"config": name, "geometry": geom, "size": size, "steps": steps, "precision": prec, "rows": list(rows),
           "vs_emulation": compare(gpu, emu), "vs_fp32_oracle": compare(gpu, f32),
           "vs_exact_mlp": compare(gpu, exact), "emulation_vs_fp32_oracle": compare(emu, f32),
           "fp32_oracle_vs_exact_mlp": compare(f32, exact)}
    record.append(res)
    e = res["vs_emulation"]
    ident, iou, mean = {"bf16": (0.999, 0.9999, 0.02), "fp16": (0.98, 0.995, 0.3)}[prec]
    assert e["identical"] >= ident, res
    assert e["iou"] >= iou, res
    assert max(e["mean_abs"]) <= mean, res
    assert e["identical"] > res["vs_fp32_oracle"]["identical"], res
    # the quality bound against the exact-MLP frame: per precision, and per crop against r4
    x = res["vs_exact_mlp"]
    qi, qiou, qmean = EXACT_BOUND[prec]
    assert x["identical"] >= qi and x["iou"] >= qiou and max(x["mean_abs"][:3]) <= qmean, res
    ri, riou, rmean = EXACT_R4[(name, geom)]
    assert x["identical"] >= ri - 0.02, res
    assert x["iou"] >= riou - 0.01, res
    assert max(x["mean_abs"][:3]) <= 1.25 * rmean, res
    # the fp32 MLP is the yardstick's own distance from the exact one: it must stay far closer
    y = res["fp32_oracle_vs_exact_mlp"]
    assert y["identical"] >= 0.85 and y["iou"] >= 0.999, res
    return res


# (identical, IoU, max per-channel mean |delta|) against the exact-MLP frame
EXACT_BOUND = {"bf16": (0.72, 0.90, 12.0), "fp16": (0.75, 0.78, 3.2)}
EXACT_R4 = {("C3", "car_1"): (0.7601, 0.99801, 5.437), ("C4", "plane_2"): (0.8493, 0.93107, 10.240),
            ("C5", "plane_1"): (0.8784, 0.86754, 2.720), ("C5", "plane_2"): (0.9325, 0.97787, 2.603),
            ("C5", "plane_3"): (0.9931, 0.81736, 1.150), ("C5", "car_1"): (0.7893, 0.99674, 2.433),
            ("C5", "3a3d4a90a2db90b4203936772104a82d.obj"): (0.8386, 0.88365, 2.507)}


@pytest.fixture(scope="module")
def record():
    out = []
    yield out
    d = os.path.join(REPO, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "lowp_contract.json"), "w") as f:
        json.dump(out, f, indent=1)


def test_c3_bf16_contract(chrome, record):
    # C3: car_1 2048^2, 256 steps, bf16; the 256 rows through the object's centre
    contract("C3", "car_1", 2048, 256, "bf16", (896, 1152), chrome, record)


@pytest.mark.parametrize("geom", GEOMS)
def test_c5_fp16_contract(chrome, record, geom):
    # C5: each geometry 2048^2, 128 steps, fp16; 128 rows through the centre
    contract("C5", geom, 2048, 128, "fp16", (960, 1088), chrome, record)


def test_c4_bf16_contract(chrome, record):
    # C4: plane_2 4096^2, 128 steps, bf16; 128 rows through the centre
    contract("C4", "plane_2", 4096, 128, "bf16", (1984, 2112), chrome, record)
