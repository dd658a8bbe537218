"""The HighFive subset (include/highfive/, over libnr's nr_h5_* C ABI) against h5py.

tests/cpp/highfive_load.cpp restates the reference's loadModelFromH5
(simpleInfer.cpp:13-79 = NeuralNetwork::load, neuralNetwork.cpp:86-129) with the same
HighFive calls, compiled with g++ against include/ and linked to libnr.so.  Its dump of
every layer (Keras kernel order + bias, hex floats) must equal h5py's reading of all five
bundled geometries bit for bit (tests/golden/weights_h5py.npz).  CPU only: the loader
builds host-only DenseLayers, so no GPU call is made."""
import os
import subprocess

import numpy as np
import pytest

import cudaneuralrender_amd as nr
from conftest import GEOMS, REPO


@pytest.fixture(scope="module")
def loader(tmp_path_factory):
    nr.lib()  # libnr.so must be built
    exe = str(tmp_path_factory.mktemp("hf") / "highfive_load")
    libdir = os.path.join(REPO, "cudaneuralrender_amd", "lib")
    cmd = ["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", os.path.join(REPO, "tests", "cpp", "highfive_load.cpp"),
           "-o", exe, "-L", libdir, "-lnr", f"-Wl,-rpath,{libdir}", "-L/opt/rocm/lib", "-lamdhip64"]
    subprocess.run(cmd, check=True)
    return exe


def run(exe, path):
    return subprocess.run([exe, path], capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("geom", GEOMS)
def test_highfive_loader_matches_h5py(loader, golden, geom):
    r = run(loader, nr.geometry_path(geom))
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "layers 9 weights 7296 biases 257"
    w = golden["weights"]
    order = [str(x) for x in w[f"{geom}/__order__"]]
    i = 1
    for li, name in enumerate(order):
        lname, din, dout, act = lines[i].split()
        assert lname == f"Dense_{li}" and act == ("tanh" if li == len(order) - 1 else "relu")
        din, dout = int(din), int(dout)
        K = np.array([[float.fromhex(v) for v in lines[i + 1 + x].split()] for x in range(din)], dtype=np.float32)
        b = np.array([float.fromhex(v) for v in lines[i + 1 + din].split()], dtype=np.float32)
        assert np.array_equal(K, w[f"{geom}/{name}/kernel:0"]), name
        assert np.array_equal(b, w[f"{geom}/{name}/bias:0"]), name
        i += 2 + din
    assert i == len(lines)


def test_highfive_errors(loader, tmp_path):
    r = run(loader, str(tmp_path / "missing.h5"))
    assert r.returncode == 3 and "Unable to open file" in r.stdout and "cannot open" in r.stdout
    bad = tmp_path / "bad.h5"
    bad.write_bytes(b"not an hdf5 file" * 10)
    r = run(loader, str(bad))
    assert r.returncode == 3 and "not an HDF5 file" in r.stdout


def test_h5_tree_c_abi():
    """The C ABI the headers wrap, driven directly: names in HDF5 name order, types, dims."""
    import ctypes
    L = nr.lib()
    f = ctypes.c_void_p()
    assert L.nr_h5_open(nr.geometry_path("plane_1").encode(), ctypes.byref(f)) == 0
    try:
        root = ctypes.c_uint64()
        assert L.nr_h5_root(f, ctypes.byref(root)) == 0
        n = ctypes.c_size_t()
        assert L.nr_h5_num_members(f, root, ctypes.byref(n)) == 0 and n.value == 9
        names = []
        for i in range(n.value):
            buf = ctypes.create_string_buffer(64)
            obj = ctypes.c_uint64()
            assert L.nr_h5_member(f, root, i, buf, 64, None, ctypes.byref(obj)) == 0
            t = ctypes.c_int()
            assert L.nr_h5_object_type(f, obj, ctypes.byref(t)) == 0 and t.value == 1  # NR_H5_GROUP
            names.append(buf.value.decode())
        assert names == sorted(names) and names[0] == "dense"  # name order, as HighFive lists them
        # a too-small name buffer and an out-of-range index are errors, not overflows
        assert L.nr_h5_member(f, root, 0, ctypes.create_string_buffer(2), 2, None, None) == -1
        assert L.nr_h5_member(f, root, 99, None, 0, None, None) == -1
        # a dataset is not a group
        obj = ctypes.c_uint64()
        L.nr_h5_member(f, root, 0, None, 0, None, ctypes.byref(obj))
        inner = ctypes.c_uint64()
        assert L.nr_h5_member(f, obj, 0, None, 0, None, ctypes.byref(inner)) == 0
        ds = ctypes.c_uint64()
        assert L.nr_h5_member(f, inner, 1, None, 0, None, ctypes.byref(ds)) == 0  # kernel:0
        nd = ctypes.c_int()
        dims = (ctypes.c_uint64 * 4)()
        assert L.nr_h5_dims(f, ds, dims, 4, ctypes.byref(nd)) == 0 and nd.value == 2
        assert (dims[0], dims[1]) == (3, 32)
        assert L.nr_h5_num_members(f, ds, ctypes.byref(n)) == -1
        out = (ctypes.c_float * 96)()
        assert L.nr_h5_read_f32(f, ds, out, 95) == -1
        assert L.nr_h5_read_f32(f, ds, out, 96) == 0
    finally:
        L.nr_h5_close(f)
