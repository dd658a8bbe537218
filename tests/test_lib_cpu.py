"""CPU tests of libnr.so's host side: the C ABI loads and exports every declared symbol,
and the pieces that need no GPU (HDF5 reader errors, PNG/PPM codecs, camera, shard
arithmetic, host re-assembly) behave like the reference's host code."""
import ctypes
import os
import re

import numpy as np
import pytest

import cudaneuralrender_amd as nr
from cudaneuralrender_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "neural_render.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = nr.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == syms, "Python binding out of sync with the header"
    assert L.nr_abi_version() == 1


def test_create_without_gpu_fails_cleanly():
    # no exit()/abort() inside the library: a missing device is an error code
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    ctx = ctypes.c_void_p()
    rc = nr.lib().nr_create(0, ctypes.byref(ctx))
    assert rc == -2 and not ctx
    assert b"device" in nr.lib().nr_last_error(None)


def test_hdf5_errors(tmp_path):
    with pytest.raises(nr.NRError) as e:
        nr.read_keras_h5(str(tmp_path / "missing.h5"))
    assert e.value.code == -3
    bad = tmp_path / "bad.h5"
    bad.write_bytes(b"not an hdf5 file" * 10)
    with pytest.raises(nr.NRError) as e:
        nr.read_keras_h5(str(bad))
    assert e.value.code == -4
    # truncated real file
    data = open(nr.geometry_path("plane_1"), "rb").read()
    trunc = tmp_path / "trunc.h5"
    trunc.write_bytes(data[:9000])
    with pytest.raises(nr.NRError):
        nr.read_keras_h5(str(trunc))


@pytest.mark.parametrize("name", ["Chrome", "skin-matcap", "Car Paint Red"])
def test_png_decode_matches_pil(name):
    from PIL import Image
    path = nr.matcap_path(name)
    got = nr.load_png(path)
    im = np.asarray(Image.open(path).convert("RGBA")).astype(np.uint32)
    # Image::loadPNG packing (image.cu:57-58): a<<24 | b<<16 | g<<8 | r
    want = (im[..., 3] << 24) | (im[..., 2] << 16) | (im[..., 1] << 8) | im[..., 0]
    assert got.shape == want.shape == (512, 512)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("flip", [True, False])
def test_png_save_roundtrip(tmp_path, flip):
    from PIL import Image
    rng = np.random.default_rng(1)
    img = rng.integers(0, 2 ** 32, size=(37, 53), dtype=np.uint64).astype(np.uint32)
    p = str(tmp_path / "x.png")
    nr.save_png(p, img, flip=flip)
    back = nr.load_png(p)
    # savePNG with doFlip reverses the byte stream: a 180-degree rotation (quirk Q9)
    want = img[::-1, ::-1] if flip else img
    assert np.array_equal(back, want)
    pil = np.asarray(Image.open(p).convert("RGBA")).astype(np.uint32)
    assert np.array_equal((pil[..., 3] << 24) | (pil[..., 2] << 16) | (pil[..., 1] << 8) | pil[..., 0], want)


def test_ppm_writer(tmp_path):
    img = np.arange(6 * 4, dtype=np.uint32).reshape(4, 6) * 0x01020305
    p = str(tmp_path / "x.ppm")
    nr.save_ppm(p, img)
    data = open(p, "rb").read()
    # sdkSavePPM4ub (helper_image.h:310-328): "P6\n<w>\n<h>\n255\n", RGB, row 0 first
    assert data.startswith(b"P6\n6\n4\n255\n")
    rgb = np.frombuffer(data[len(b"P6\n6\n4\n255\n"):], np.uint8).reshape(4, 6, 3)
    assert np.array_equal(rgb[..., 0], (img & 0xff).astype(np.uint8))
    assert np.array_equal(rgb[..., 2], ((img >> 16) & 0xff).astype(np.uint8))


def camera_ref(rx, ry, zoom):
    """numpy restatement of updateViewMatrices (main.cpp:207-222)."""
    ax, ay = -np.radians(rx), -np.radians(ry)
    Rx = np.array([[1, 0, 0], [0, np.cos(ax), -np.sin(ax)], [0, np.sin(ax), np.cos(ax)]])
    Ry = np.array([[np.cos(ay), 0, np.sin(ay)], [0, 1, 0], [-np.sin(ay), 0, np.cos(ay)]])
    R = Rx @ Ry
    M = np.eye(4)
    M[:3, :3] = R
    M[:3, 3] = R @ np.array([0, 0, zoom])
    return M[:3].reshape(-1), np.linalg.inv(M).reshape(-1)


@pytest.mark.parametrize("rx,ry,zoom", [(0, 0, 2), (-18.3, 150.7, 2.25), (45, -30, 3.0), (-79, 229, 3.05)])
def test_camera(rx, ry, zoom):
    iv, nm = nr.camera(rx, ry, zoom)
    riv, rnm = camera_ref(rx, ry, zoom)
    assert np.allclose(iv, riv, atol=1e-6) and np.allclose(nm, rnm, atol=1e-6)
    if rx == 0 and ry == 0:
        # default camera: eye at (0, 0, 2)
        assert list(iv) == [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 2]


@pytest.mark.parametrize("H,band,n", [(1024, 8, 8), (1024, 8, 3), (83, 5, 3), (7, 8, 2), (1, 1, 4), (100, 1, 7)])
def test_shard_rows_partition(H, band, n):
    rows = [nr.shard_rows(H, band, n, s) for s in range(n)]
    assert sum(rows) == H
    # band b goes to shard b % n
    expect = [0] * n
    for y in range(H):
        expect[(y // band) % n] += 1
    assert rows == expect


def test_assemble_shards_host():
    W, H, band, n = 13, 29, 4, 3
    full = np.arange(W * H, dtype=np.uint32).reshape(H, W)
    shards = []
    for s in range(n):
        ys = [y for y in range(H) if (y // band) % n == s]
        shards.append(full[ys])
    assert np.array_equal(nr.assemble_shards(shards, W, H, band, n), full)


def assert_no_packed_fp32(lib_path, tmp_path):
    """The gfx950 code objects of lib_path hold reduced-precision MFMAs and no packed-FP32 VALU."""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    so = tmp_path / "libnr.so"
    shutil.copy(lib_path, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    objs = sorted(p for p in tmp_path.iterdir() if "amdgcn" in p.name and "gfx950" in p.name)
    assert objs, "no gfx950 code object in libnr.so"
    n_mfma = 0
    for p in objs:
        dis = subprocess.run([objdump, "-d", str(p)], check=True, capture_output=True, text=True).stdout
        bad = re.findall(r"v_pk_(?:mul|add|fma)_f32|v_pk_mov_b32", dis)
        assert not bad, f"{p.name}: {len(bad)} packed-FP32 instructions"
        n_mfma += len(re.findall(r"v_mfma_f32_32x32x16_(?:bf16|f16)", dis))
    assert n_mfma > 0


def test_device_code_has_no_packed_fp32(tmp_path):
    """libnr.so's gfx950 code objects contain no packed-FP32 VALU instructions: beside
    reduced-precision MFMAs on the same SIMD a packed op consuming a packed op's result can
    read stale data in lanes 48-63 (profiles/r2_lowp_determinism.txt), so the Makefile builds
    with -packed-fp32-ops.  A rebuild without that flag fails here."""
    assert_no_packed_fp32(_lib.LIB_PATH, tmp_path)


def test_batch_frames_per_launch_fits_the_queue_counters():
    """nr_render_batch caps the frames of one launch so that the busiest pixel-queue shard's
    positions (plus the waves' over-reservation) stay below 2^32 (16384^2 x 16
    frames on one queue shard, or 32768^2 x 32 frames on 8, used to wrap the counter)."""
    f = nr.batch_frames_per_launch
    assert f(1024, 1024, 1, 1, 0, 32) == 32
    assert f(1024, 1024, 1, 1, 0, 5) == 5
    assert f(1024, 1024, 1, 1, 0, 100) == 32
    for W, H, q, n in [(16384, 16384, 1, 16), (32768, 32768, 8, 32), (46340, 46340, 1, 32), (8192, 8192, 8, 32)]:
        k = f(W, H, 1, 1, 0, n, q)
        per_frame = -(-((W + 7) // 8) * ((H + 7) // 8) // q) * 64
        assert 1 <= k <= min(n, 32)
        assert k * per_frame + 256 * 8 * 4 * 64 < 2 ** 32, (W, H, q, k)
        if k < min(n, 32):
            assert (k + 1) * per_frame + 256 * 8 * 4 * 64 >= 2 ** 32
    assert f(16384, 16384, 1, 1, 0, 16, 1) == 15
    assert f(0, 16, 1, 1, 0, 4) == 0
