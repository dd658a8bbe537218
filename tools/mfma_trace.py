"""Diagnostic: replay the oracle's MFMA calls for chosen points on the GPU's matrix core.

    python tools/mfma_trace.py collect gpurun_out/mlp_dump.npz out.npz   (here: the oracle's
        fp32x3 MFMA operands for the points where it differs from the dumped GPU output)
    python tools/mfma_trace.py replay out.npz                              (GPU box: each call
        through tools/mfma_probe.hip, printed where the hardware differs from the oracle's model)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def collect(dump, out):
    import cudaneuralrender_amd as nr
    import oracle
    z = np.load(dump)
    X = z["X"]
    recs = []
    for g in sorted({k.split("/")[0] for k in z.files if "/" in k}):
        d, K, B = nr.read_keras_h5(nr.geometry_path(g))
        pack = nr.pack_x3(d, K, B)
        net = oracle.OracleNet(K, B, x3_pack=pack[:2])
        e = net.forward(X, precision=4, nthreads=1)[:, 0]
        for i in np.nonzero(e != z[f"{g}/fp32x3"])[0]:
            buf = np.zeros((4096, 34), np.float64)
            oracle.lib().or_trace_mfma(buf.ctypes.data, 4096)
            net.forward(X[i:i + 1], precision=4, nthreads=1)
            n = oracle.lib().or_trace_count()
            oracle.lib().or_trace_mfma(None, 0)
            recs.append(buf[:n])
            print(g, i, n, "calls")
    np.savez(out, recs=np.concatenate(recs))


def replay(fn):
    r = np.load(fn)["recs"]
    n = (len(r) + 31) // 32
    A = np.zeros((n, 32, 16), np.float64)
    B = np.zeros((n, 16, 32), np.float64)
    C = np.zeros((n, 32, 32), np.float32)
    for i, t in enumerate(r):
        m, d = divmod(i, 32)
        A[m, d, :], B[m, :, d], C[m, d, d] = t[1:17], t[17:33], t[0]
    Au = np.ascontiguousarray(A.astype(np.float16).view(np.uint16))
    Bu = np.ascontiguousarray(B.astype(np.float16).view(np.uint16))
    assert np.array_equal(A.astype(np.float16).astype(np.float64), A) and np.array_equal(B.astype(np.float16).astype(np.float64), B)
    D = np.zeros((n, 32, 32), np.float32)
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libmfma_probe.so"))
    L.mfma_probe.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_int]
    assert L.mfma_probe(Au.ctypes.data, Bu.ctypes.data, C.ctypes.data, D.ctypes.data, n, 0) == 0
    bad = 0
    for i, t in enumerate(r):
        m, d = divmod(i, 32)
        hw = float(D[m, d, d])
        if hw != t[33]:
            bad += 1
            print("call", i, "acc", t[0].hex(), "model", t[33].hex(), "hw", hw.hex())
            print("  a", [x.hex() for x in t[1:17]])
            print("  b", [x.hex() for x in t[17:33]])
    print("calls", len(r), "differ", bad)


if __name__ == "__main__":
    collect(sys.argv[2], sys.argv[3]) if sys.argv[1] == "collect" else replay(sys.argv[2])
