"""Builds tests/golden/mfma_{f16,bf16}.npz: gfx950 MFMA outputs measured on the GPU box, the
fixtures that pin the oracle's matrix-core summation model (oracle/nr_oracle.c mfma_sum_e).

  hand cases: tools/mfma_cases.py's hand-built dot products (its --prec f16 / bf16 output);
  random:     the first 2 matrices of each kind of tools/mfma_model.py --save (2,048 outputs per
              kind, 5 kinds), stored as 16-bit operand patterns, accumulators and results.

    python tests/golden/make_mfma_golden.py gpurun_out/mfma_cases_f16.txt gpurun_out/mfma_f16.npz f16
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tools"))
import mfma_cases  # noqa: E402

cases_txt, rand_npz, prec = sys.argv[1:4]
hw = {json.loads(l)["case"]: float.fromhex(json.loads(l)["hw"]) for l in open(cases_txt)}
A, B, C, D = [], [], [], []
for name, terms, c in mfma_cases.cases():
    a = np.zeros(16)
    b = np.zeros(16)
    for k, (x, y) in terms.items():
        a[k], b[k] = x, y
    A.append(a)
    B.append(b)
    C.append(c)
    D.append(hw[name])
out = {"hand_a": np.array(A), "hand_b": np.array(B), "hand_c": np.array(C, np.float32),
       "hand_d": np.array(D, np.float32)}
z = np.load(rand_npz)
for kind in sorted({k.rsplit("_", 1)[0] for k in z.files}):
    for n in "ABCD":
        out[f"{kind}_{n}"] = z[f"{kind}_{n}"][:2]
np.savez_compressed(os.path.join(HERE, f"mfma_{prec}.npz"), **out)
print("wrote", f"mfma_{prec}.npz", {k: v.shape for k, v in out.items()})
