"""Diagnostic (GPU box): hand-built dot products through one v_mfma_f32_32x32x16_{f16,bf16}
(tools/mfma_probe.hip), each case on the diagonal of its own 32x32 matrix slot (row i, column i),
printed as exact hex floats -- to pin the matrix core's alignment window, truncation and
rounding that tools/mfma_model.py's statistical fit narrows down.

    python tools/mfma_cases.py [--prec f16|bf16]"""
import argparse
import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "bin", "libmfma_probe.so")


def cases():
    """(name, [(a, b) x <= 16 at k positions], c) -- a, b exact in f16 (and bf16)"""
    C = []
    two = lambda e: 2.0 ** e  # noqa: E731

    S = 14  # every value scaled by 2^14, so that the small terms stay products of normal f16 values

    def prod(e):  # 2^(S + e) as an exact product of two normal f16 values (e >= -42)
        t = S + e
        return (two(t // 2), two(t - t // 2))
    one = prod(0)

    for k in range(24, 43):  # sticky bit: 1 + 2^-24 (a tie) + 2^-k, all products in half 0
        C.append((f"pos_sticky_k{k}", {0: one, 1: prod(-24), 2: prod(-k)}, 0.0))
    for k in range(24, 43):  # the same with 1 as the accumulator
        C.append((f"acc_sticky_k{k}", {1: prod(-24), 2: prod(-k)}, two(S)))
    for k in range(24, 43):  # the 1 in half 1, the small terms in half 0
        C.append((f"cross_sticky_k{k}", {8: one, 1: prod(-24), 2: prod(-k)}, 0.0))
    for k in range(24, 43):  # negative: 1 + 2^-23 + 2^-24 (a tie, odd) - 2^-k
        C.append((f"neg_sticky_k{k}", {0: one, 1: prod(-23), 2: prod(-24), 3: (-prod(-k)[0], prod(-k)[1])}, 0.0))
    for k in range(24, 43):  # negative, the 1 + 2^-23 + 2^-24 in the accumulator
        C.append((f"negacc_sticky_k{k}", {3: (-prod(-k)[0], prod(-k)[1])}, two(S) * (1.0 + 2.0 ** -23 + 2.0 ** -24)))
    for k in range(20, 40):  # two products only, no tie
        C.append((f"pair_k{k}", {0: one, 5: prod(-k)}, 0.0))
    for k in range(20, 40):  # accumulator small, products big
        C.append((f"smallacc_k{k}", {0: one, 1: prod(-24)}, two(S - k)))
    # rounding direction: exact sums just above / below a tie, and the tie itself
    C.append(("tie_even", {0: one, 1: prod(-24)}, 0.0))
    C.append(("tie_odd", {0: one, 1: prod(-23), 2: prod(-24)}, 0.0))
    C.append(("neg_tie_even", {0: (-one[0], one[1]), 1: (-prod(-24)[0], prod(-24)[1])}, 0.0))
    C.append(("neg_tie_odd", {0: (-one[0], one[1]), 1: (-prod(-23)[0], prod(-23)[1]), 2: (-prod(-24)[0], prod(-24)[1])}, 0.0))
    # cancellation: big terms cancel, small remainder
    for k in range(20, 34):
        C.append((f"cancel_k{k}", {0: one, 1: (-one[0], one[1]), 2: prod(-k)}, 0.0))
        C.append((f"cancel_acc_k{k}", {1: (-one[0], one[1]), 2: prod(-k)}, two(S)))
    return C


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="f16")
    a = ap.parse_args()
    cs = cases()
    n = (len(cs) + 31) // 32
    A = np.zeros((n, 32, 16), np.float64)
    B = np.zeros((n, 16, 32), np.float64)
    Cm = np.zeros((n, 32, 32), np.float32)
    for i, (_, terms, c) in enumerate(cs):
        m, d = divmod(i, 32)
        for k, (x, y) in terms.items():
            A[m, d, k], B[m, k, d] = x, y
        Cm[m, d, d] = c
    if a.prec == "f16":
        Au, Bu = A.astype(np.float16).view(np.uint16), B.astype(np.float16).view(np.uint16)
        assert np.array_equal(A.astype(np.float16).astype(np.float64), A)
    else:
        Au = (A.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
        Bu = (B.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16)
    D = np.zeros((n, 32, 32), np.float32)
    L = ctypes.CDLL(SO)
    L.mfma_probe.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_int]
    Au, Bu = np.ascontiguousarray(Au), np.ascontiguousarray(Bu)
    assert L.mfma_probe(Au.ctypes.data, Bu.ctypes.data, Cm.ctypes.data, D.ctypes.data, n, int(a.prec == "bf16")) == 0
    for i, (name, terms, c) in enumerate(cs):
        m, d = divmod(i, 32)
        exact = sum(x * y for x, y in terms.values()) + c  # fine for display (float64)
        v = float(D[m, d, d])
        print(json.dumps({"case": name, "hw_units": (v / 2.0 ** 14 - 1.0) * 2.0 ** 24,
                          "exact_units": (exact / 2.0 ** 14 - 1.0) * 2.0 ** 24, "hw": v.hex(), "exact_f64": exact.hex(),
                          "rne_of_exact": float(np.float32(exact)).hex()}), flush=True)


if __name__ == "__main__":
    main()
