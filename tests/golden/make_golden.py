"""Generate the committed golden fixtures under tests/golden/.

Run ONCE in the build container (it reads /root/reference, which the GPU box does
not have), with the conda interpreter that carries h5py:

    env -i PATH=/opt/conda/bin:/usr/bin /opt/conda/bin/python3.9 tests/golden/make_golden.py

Outputs (all data, no reference source):
  weights_h5py.npz  every dataset of the five bundled Keras weight files, read by
                    h5py 3.3.0 / HDF5 1.10.6 (an HDF5 implementation independent of
                    this repo's reader), keyed "<geometry>/<group>/<dataset>", plus
                    "<geometry>/__order__" = root groups in HDF5 name order -- the
                    order NeuralNetwork::load iterates (neuralNetwork.cpp:85-91).
  mlp_kat.npz       MLP known-answer test: per geometry, 4096 points from
                    numpy.random.default_rng(0) U[-1.2, 1.2]^3 followed by the
                    simpleInfer points (0,0,0) and (0.1,0.2,0.3)
                    (simpleInfer.cpp:112-126, :81-95); outputs of the network in
                    float64 (numpy), ReLU hidden layers, LINEAR last layer
                    (denseLayer.cu:150-166 -- the "Tanh" tag takes the linear branch).
  silhouettes.npz   foreground masks (any channel != 0) of the reference's own
                    renders neuralGeometries/{plane_1,car_1,plane_2}.h5.ppm
                    (P6 1024x1024, buffer row 0 first), np.packbits'ed, plus the
                    cameras recovered for them in SURVEY.md App. A.
"""
import os
import sys

import h5py
import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
GEOMS = ["plane_1", "plane_2", "plane_3", "car_1", "3a3d4a90a2db90b4203936772104a82d.obj"]


def read_weights(path):
    out = {}
    order = []
    with h5py.File(path, "r") as f:
        for name in f.keys():          # h5py iterates links in name order
            order.append(name)
            g = f[name][name]
            for ds in g.keys():
                out[f"{name}/{ds}"] = np.array(g[ds], dtype=np.float32)
    return out, order


def mlp64(weights, order, X):
    a = X.astype(np.float64)
    for i, name in enumerate(order):
        K = weights[f"{name}/kernel:0"].astype(np.float64)   # (in, out)
        b = weights[f"{name}/bias:0"].astype(np.float64)
        a = a @ K + b
        if i != len(order) - 1:
            a = np.maximum(a, 0.0)
    return a


def read_ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    # header: "P6" w h maxval, whitespace separated (sdkSavePPM4ub writes one per line)
    toks, pos = [], 0
    while len(toks) < 4:
        while data[pos:pos + 1].isspace():
            pos += 1
        end = pos
        while not data[end:end + 1].isspace():
            end += 1
        toks.append(data[pos:end])
        pos = end
    pos += 1
    assert toks[0] == b"P6", toks[0]
    w, h, maxval = int(toks[1]), int(toks[2]), int(toks[3])
    assert maxval == 255
    img = np.frombuffer(data, dtype=np.uint8, count=w * h * 3, offset=pos).reshape(h, w, 3)
    return img


def main():
    wts = {}
    kat = {}
    rng = np.random.default_rng(0)
    X = rng.uniform(-1.2, 1.2, size=(4096, 3)).astype(np.float32)
    X = np.concatenate([X, np.array([[0, 0, 0], [0.1, 0.2, 0.3]], np.float32)], 0)
    kat["X"] = X
    for g in GEOMS:
        w, order = read_weights(os.path.join(REF, "neuralGeometries", g + ".h5"))
        for k, v in w.items():
            wts[f"{g}/{k}"] = v
        wts[f"{g}/__order__"] = np.array(order)
        kat[g] = mlp64(w, order, X)[:, 0]
    np.savez_compressed(os.path.join(HERE, "weights_h5py.npz"), **wts)
    np.savez_compressed(os.path.join(HERE, "mlp_kat.npz"), **kat)

    sil = {}
    for g in ["plane_1", "car_1", "plane_2"]:
        img = read_ppm(os.path.join(REF, "neuralGeometries", g + ".h5.ppm"))
        fg = (img != 0).any(axis=2)
        sil[g] = np.packbits(fg.reshape(-1))
        sil[g + "/shape"] = np.array(fg.shape)
        sil[g + "/count"] = np.array(int(fg.sum()))
    # cameras recovered by silhouette search: rx, ry (deg), zoom
    sil["plane_1/camera"] = np.array([-18.3, 150.7, 2.25], np.float32)
    sil["car_1/camera"] = np.array([-79.0, 229.0, 3.05], np.float32)
    np.savez_compressed(os.path.join(HERE, "silhouettes.npz"), **sil)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    sys.exit(main())
