"""Diagnostic (GPU box): does v_mfma_f32_16x16x32_{f16,bf16} sum its K = 32 products as two
chained K = 16 steps of the round-4 matrix-core model (oracle/nr_oracle.c mfma_sum_e, fitted on
v_mfma_f32_32x32x16)?  Random matrices of the kinds tools/mfma_model.py fits on (wide exponent
spreads, x3-like, cancellation, tiny, residual) through tools/mfma_k32_probe.hip, each output
against or_mfma_sum(or_mfma_sum(c, k 0-15), k 16-31) from the oracle library.  Prints, per
precision and kind, the share of outputs equal bit for bit (and the f64-reference error scale,
a check on the operand layout).

    python tools/mfma_k32_check.py [--n 48]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SO = os.path.join(HERE, "bin", "libmfma_k32_probe.so")
sys.path.insert(0, HERE)
from mfma_model import to16  # noqa: E402


def kinds(n, prec, rng):
    sgn = lambda s: rng.choice([-1.0, 1.0], size=s)  # noqa: E731
    lo = -20 if prec == "f16" else -70
    return [
        ("generic", sgn((n, 16, 32)) * np.exp2(rng.uniform(-8, 3, (n, 16, 32))),
         sgn((n, 32, 16)) * np.exp2(rng.uniform(-8, 3, (n, 32, 16))), sgn((n, 16, 16)) * np.exp2(rng.uniform(-6, 5, (n, 16, 16)))),
        ("x3_like", rng.standard_normal((n, 16, 32)) * 0.3, rng.uniform(0, 1, (n, 32, 16)) ** 3,
         rng.standard_normal((n, 16, 16)) * 2.0),
        ("cancel", sgn((n, 16, 32)) * rng.uniform(0.5, 1.0, (n, 16, 32)), rng.uniform(0.5, 1.0, (n, 32, 16)),
         sgn((n, 16, 16)) * np.exp2(rng.uniform(-30, -10, (n, 16, 16)))),
        ("tiny", sgn((n, 16, 32)) * np.exp2(rng.uniform(lo, lo + 8, (n, 16, 32))),
         sgn((n, 32, 16)) * np.exp2(rng.uniform(-4, 0, (n, 32, 16))), sgn((n, 16, 16)) * np.exp2(rng.uniform(lo - 10, lo + 2, (n, 16, 16)))),
        ("residual", sgn((n, 16, 32)) * rng.uniform(0.5, 1.0, (n, 16, 32)), np.exp2(rng.uniform(-30, -20, (n, 32, 16))),
         sgn((n, 16, 16)) * rng.uniform(1.0, 2.0, (n, 16, 16))),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    a = ap.parse_args()
    P = ctypes.CDLL(SO)
    O = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    dp = ctypes.POINTER(ctypes.c_double)
    O.or_mfma_sum.restype = ctypes.c_float
    O.or_mfma_sum.argtypes = [ctypes.c_float, dp, dp, ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(32)
    res = {}
    for prec in ("bf16", "f16"):
        emin = -14 if prec == "f16" else -126
        for kind, A, B, C in kinds(a.n, prec, rng):
            ua, va = to16(A, prec)
            ub, vb = to16(B, prec)
            c32 = C.astype(np.float32)
            D = np.zeros((a.n, 16, 16), np.float32)
            rc = P.mfma_k32_probe(ua.ctypes.data_as(ctypes.c_void_p), ub.ctypes.data_as(ctypes.c_void_p),
                                  c32.ctypes.data_as(ctypes.c_void_p), D.ctypes.data_as(ctypes.c_void_p), a.n,
                                  1 if prec == "bf16" else 0)
            assert rc == 0, rc
            same = tot = 0
            ref_err = []
            for m in range(a.n):
                for i in range(16):
                    ai = np.ascontiguousarray(va[m, i, :])
                    for j in range(16):
                        bj = np.ascontiguousarray(vb[m, :, j])
                        r = O.or_mfma_sum(float(c32[m, i, j]), ai[:16].ctypes.data_as(dp), bj[:16].ctypes.data_as(dp), emin, 1)
                        r = O.or_mfma_sum(r, ai[16:].ctypes.data_as(dp), bj[16:].ctypes.data_as(dp), emin, 1)
                        g = float(D[m, i, j])
                        same += np.float32(r).view(np.uint32) == np.float32(g).view(np.uint32)
                        tot += 1
                        exact = float(c32[m, i, j]) + float(ai @ bj)
                        ref_err.append(abs(g - exact) / max(abs(exact), 1e-30))
            res[f"{prec}/{kind}"] = {"identical": same / tot, "outputs": tot,
                                     "median_rel_err_vs_f64": float(np.median(ref_err))}
            print(json.dumps({"prec": prec, "kind": kind, **res[f"{prec}/{kind}"]}), flush=True)
    allsame = all(v["identical"] == 1.0 for v in res.values())
    print(json.dumps({"all_identical": allsame}))


if __name__ == "__main__":
    main()
