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
    assert L.nr_abi_version() == 3
    # the ctypes mirror of nr_stats and the header's default endgame threshold
    txt = open(os.path.join(REPO, "include", "neural_render.h")).read()
    assert float(re.search(r"#define NR_ENDGAME_DEFAULT ([0-9.]+)f", txt).group(1)) == nr.NR_ENDGAME_DEFAULT
    assert ctypes.sizeof(_lib.NRStats) == 64 and _lib.NRStats.endgame_evals.offset == 48
    assert _lib.NRStats.endgame_switches.offset == 56


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
    """numpy f64 restatement of updateViewMatrices (main.cpp:207-222) on the float arguments."""
    rx, ry, zoom = float(np.float32(rx)), float(np.float32(ry)), float(np.float32(zoom))
    ax, ay = -np.radians(rx), -np.radians(ry)
    Rx = np.array([[1, 0, 0], [0, np.cos(ax), -np.sin(ax)], [0, np.sin(ax), np.cos(ax)]])
    Ry = np.array([[np.cos(ay), 0, np.sin(ay)], [0, 1, 0], [-np.sin(ay), 0, np.cos(ay)]])
    R = Rx @ Ry
    M = np.eye(4)
    M[:3, :3] = R
    M[:3, 3] = R @ np.array([0, 0, zoom])
    return M[:3].reshape(-1), np.linalg.inv(M).reshape(-1)


CAMS = [(0, 0, 2), (-18.3, 150.7, 2.25), (45, -30, 3.0), (-79, 229, 3.05), (90, 180, 2.0), (-18.8021, 149.7984, 2.2702),
        (0, 37.0, 4.0), (12.5, 0, 1.5)]


def _ulps(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64))


@pytest.mark.parametrize("rx,ry,zoom", CAMS)
def test_camera(rx, ry, zoom):
    """NR_CAMERA_F64 (nr_camera): the f64 rotation and its exact transpose-inverse, rounded once:
    within 1 ulp of numpy's f64 evaluation rounded to f32 (where both are not ~0), and M^-1 M = I."""
    iv, nm = nr.camera(rx, ry, zoom)
    riv, rnm = camera_ref(rx, ry, zoom)
    for got, ref in ((iv, riv), (nm, rnm)):
        big = np.abs(ref) > 1e-6
        assert (_ulps(got[big], ref[big].astype(np.float32)) <= 1).all(), (got, ref)
        assert np.abs(got[~big] - ref[~big]).max(initial=0) <= 1e-6
    M = np.eye(4)
    M[:3] = iv.reshape(3, 4)
    assert np.abs(M @ nm.reshape(4, 4).astype(np.float64) - np.eye(4)).max() < 1e-6
    if rx == 0 and ry == 0:
        # default camera: eye at (0, 0, 2)
        assert list(iv) == [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, zoom]


def camera_eigen_np(rx, ry, zoom, tx=0.0, ty=0.0):
    """numpy float32 restatement of main.cpp:207-222 through Eigen 3.3's scalar paths (the
    independent check of nr_pack.cpp camera_matrices_eigen): AngleAxisf * AngleAxisf as a
    quaternion product, toRotationMatrix, rotate, translate (3-term redux x0 + (x1 + x2)),
    cofactor 4x4 inverse with det = (c0 + c1) + (c2 + c3)."""
    import math
    f = np.float32
    ax = f(float(-f(rx)) * math.pi / 180.0)
    ay = f(float(-f(ry)) * math.pi / 180.0)
    hx, hy = f(0.5) * ax, f(0.5) * ay
    w1, x1 = f(math.cos(hx)), f(math.sin(hx))
    w2, y2 = f(math.cos(hy)), f(math.sin(hy))
    z = f(0)
    qw = w1 * w2 - x1 * z - z * y2 - z * z
    qx = w1 * z + x1 * w2 + z * z - z * y2
    qy = w1 * y2 + z * w2 + z * z - x1 * z
    qz = w1 * z + z * z + x1 * y2 - z * z
    tx_, ty_, tz_ = f(2) * qx, f(2) * qy, f(2) * qz
    twx, twy, twz = tx_ * qw, ty_ * qw, tz_ * qw
    txx, txy, txz = tx_ * qx, ty_ * qx, tz_ * qx
    tyy, tyz, tzz = ty_ * qy, tz_ * qy, tz_ * qz
    L = [[f(1) - (tyy + tzz), txy - twz, txz + twy],
         [txy + twz, f(1) - (txx + tzz), tyz - twx],
         [txz - twy, tyz + twx, f(1) - (txx + tyy)]]
    v = [-f(tx), -f(ty), -(-f(zoom))]
    T = [f(0) + (L[i][0] * v[0] + (L[i][1] * v[1] + L[i][2] * v[2])) for i in range(3)]
    M = [[L[0][0], L[0][1], L[0][2], T[0]], [L[1][0], L[1][1], L[1][2], T[1]],
         [L[2][0], L[2][1], L[2][2], T[2]], [z, z, z, f(1)]]

    def det3(i1, i2, i3, j1, j2, j3):
        return M[i1][j1] * (M[i2][j2] * M[i3][j3] - M[i2][j3] * M[i3][j2])

    def cof(i, j):
        i1, i2, i3, j1, j2, j3 = (i + 1) % 4, (i + 2) % 4, (i + 3) % 4, (j + 1) % 4, (j + 2) % 4, (j + 3) % 4
        return det3(i1, i2, i3, j1, j2, j3) + det3(i2, i3, i1, j1, j2, j3) + det3(i3, i1, i2, j1, j2, j3)

    R = [[z] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            R[j][i] = -cof(i, j) if (i + j) % 2 else cof(i, j)
    det = (M[0][0] * R[0][0] + M[1][0] * R[0][1]) + (M[2][0] * R[0][2] + M[3][0] * R[0][3])
    iv = np.array([M[i][j] for i in range(3) for j in range(4)], np.float32)
    nm = np.array([R[i][j] / det for i in range(4) for j in range(4)], np.float32)
    return iv, nm


@pytest.mark.parametrize("rx,ry,zoom", CAMS)
def test_camera_eigen_float(rx, ry, zoom):
    """NR_CAMERA_EIGEN restates the reference's float Eigen camera.  Parity with
    Eigen itself is unpinned (Eigen is not in this image); checked here: bit-equal to an
    independent numpy float32 restatement of the same Eigen 3.3 code paths, a few ulps from the
    f64 form, a rotation (R R^T = I to float precision), and M^-1 M = I."""
    iv, nm = nr.camera(rx, ry, zoom, mode="eigen")
    riv, rnm = camera_eigen_np(rx, ry, zoom)
    assert np.array_equal(iv, riv), (iv, riv)
    assert np.array_equal(nm, rnm), (nm, rnm)
    fiv, fnm = nr.camera(rx, ry, zoom)
    assert np.abs(iv - fiv).max() <= 4e-6 * max(1.0, zoom) and np.abs(nm - fnm).max() <= 4e-6 * max(1.0, zoom)
    R = iv.reshape(3, 4)[:, :3].astype(np.float64)
    assert np.abs(R @ R.T - np.eye(3)).max() < 1e-6
    M = np.eye(4)
    M[:3] = iv.reshape(3, 4)
    assert np.abs(M @ nm.reshape(4, 4).astype(np.float64) - np.eye(4)).max() < 1e-5
    if rx == 0 and ry == 0:
        assert list(iv) == [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, zoom]


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


def kernel_resources(lib_path, tmp_path):
    """{kernel symbol: {vgpr_count, private_segment_fixed_size, vgpr_spill_count, ...}} from the
    code-object metadata of lib_path's gfx950 objects"""
    import shutil
    import subprocess
    readelf, objdump = "/opt/rocm/lib/llvm/bin/llvm-readelf", "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not (os.path.exists(readelf) and os.path.exists(objdump)):
        pytest.skip("llvm-readelf / llvm-objdump not available")
    so = tmp_path / "libnr.so"
    shutil.copy(lib_path, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    out = {}
    for p in sorted(p for p in tmp_path.iterdir() if "amdgcn" in p.name and "gfx950" in p.name):
        notes = subprocess.run([readelf, "--notes", str(p)], check=True, capture_output=True, text=True).stdout
        for blk in notes.split(".name:")[1:]:
            name = blk.split("\n")[0].strip()
            out[name] = {k: int(v) for k, v in re.findall(r"\.(\w+):\s+(\d+)\s*$", blk, re.M)}
    return out


def test_batched_fp32_tracer_has_no_scratch(tmp_path):
    """the bench's kernel -- the batched fp32 k_trace, built for 4 workgroups per
    CU (<= 128 VGPRs) -- keeps every value in registers: no spill, no scratch.  (Its spills were
    per-lane loop invariants the compiler hoisted: the lanemask of popcount(m & lanemask_lt()) and
    the ds_bpermute addresses of the quad and lane-group shuffles; mbcnt, DPP quad_perm and
    v_permlane swaps need none.)  The stand-alone MLP's fp32 and bf16 instances stay spill-free."""
    res = kernel_resources(_lib.LIB_PATH, tmp_path)
    want = {"_ZN2nr7k_traceILi0ELb0ELb0ELb1ELb0ELb0ELb1EEEvNS_10RenderArgsENS_7MlpArgsENS_9TraceArgsE": 128,
            "_ZN2nr7k_mlp16ILi0ELi3ELb0EEEvNS_7MlpArgsEPKfPfi": 512,
            # round 6: the 16x16x32 instances (128 pinned registers), the default for bf16 / fp16
            "_ZN2nr7k_mlp16ILi1ELi3ELb1EEEvNS_7MlpArgsEPKfPfi": 168,
            "_ZN2nr7k_mlp16ILi2ELi3ELb1EEEvNS_7MlpArgsEPKfPfi": 168}
    for name, cap in want.items():
        r = res[name]
        assert r["private_segment_fixed_size"] == 0 and r["vgpr_spill_count"] == 0, (name, r)
        assert r["vgpr_count"] <= cap, (name, r)
    # the bf16 MLP pins 144 registers for its pipelined stream (nr_mlp16_asm.h); one or two loop
    # invariants of its builtin-form path (nr_set_debug bit 11) go to scratch
    r = res["_ZN2nr7k_mlp16ILi1ELi3ELb0EEEvNS_7MlpArgsEPKfPfi"]
    assert r["private_segment_fixed_size"] <= 16 and r["vgpr_count"] <= 168, r


def test_trace_kernarg_layout_matches_trace_kargs(tmp_path):
    """Round 6 (nr_trace.hip fresh_kargs): k_trace re-reads its arguments through a TraceKargs
    {RenderArgs A; MlpArgs M; TraceArgs T;} view of the kernarg segment, which holds iff the code
    object puts the three by-value arguments where that struct's layout does: back to back, each
    at the next 8-byte boundary (every one holds pointers / doubles), from offset 0.  Checked
    here on every k_trace instance's metadata in the built library."""
    import shutil
    import subprocess
    readelf, objdump = "/opt/rocm/lib/llvm/bin/llvm-readelf", "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not (os.path.exists(readelf) and os.path.exists(objdump)):
        pytest.skip("llvm-readelf / llvm-objdump not available")
    so = tmp_path / "libnr.so"
    shutil.copy(_lib.LIB_PATH, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    seen = 0
    for p in sorted(p for p in tmp_path.iterdir() if "amdgcn" in p.name and "gfx950" in p.name):
        notes = subprocess.run([readelf, "--notes", str(p)], check=True, capture_output=True, text=True).stdout
        for kern in notes.split("  - .agpr_count:")[1:]:
            m = re.search(r"\.name:\s+(\S+)", kern)
            if not m or "k_trace" not in m.group(1):
                continue
            args = re.findall(r"\.offset:\s+(\d+)\s+\.size:\s+(\d+)\s+\.value_kind:\s+(\w+)", kern)
            byval = [(int(o), int(s)) for o, s, k in args if k == "by_value"]
            assert len(byval) == 3, (m.group(1), byval)
            off = 0
            for o, s in byval:
                assert o == off, (m.group(1), byval)
                off = (o + s + 7) // 8 * 8
            seen += 1
    assert seen >= 8, seen


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
        # every wave nr_set_occupancy allows: two pending reservations of 64 + a blocking one of 64
        slop = 512 * 16 * 4 * 192
        assert k * per_frame + slop < 2 ** 32, (W, H, q, k)
        if k < min(n, 32):
            assert (k + 1) * per_frame + slop >= 2 ** 32
    assert f(16384, 16384, 1, 1, 0, 16, 1) == 15
    assert f(0, 16, 1, 1, 0, 4) == 0


_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def _regs(ops):
    """{('v'|'a', index)} named by an operand string (v7, v[8:11], a[0:15])"""
    out = set()
    for kind, lo, hi, one in _REG.findall(ops):
        lo, hi = (int(lo), int(hi)) if lo else (int(one), int(one))
        out |= {(kind, i) for i in range(lo, hi + 1)}
    return out


def _parse(line):
    """(address, mnemonic, dst regs, src regs, MFMA SrcC regs) of one llvm-objdump -d line, or None"""
    m = re.match(r"\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
    if not m:
        return None
    mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
    parts = [p.strip() for p in re.split(r",(?![^\[]*\])", ops)] if ops else []
    dst = _regs(parts[0]) if parts and not mn.startswith(("s_", "ds_write", "global_store", "buffer_store")) else set()
    src = set().union(*[_regs(p) for p in parts[1:]]) if len(parts) > 1 else set()
    srcc = _regs(parts[3]) if mn.startswith("v_mfma") and len(parts) > 3 else set()
    return addr, mn, dst, src, srcc


def _wait_states(mn, line):
    m = re.match(r"\s+s_nop\s+(?:0x)?([0-9a-f]+)", line)
    return int(m.group(1), 16) + 1 if m else 1


# MFMA -> VALU distances (wait states; tools/gen_mlp_asm.py): a VALU read or write of a register a
# v_mfma_f32_32x32x16 writes needs 12 (hipcc's own padding; 13 required here), a VALU write of a
# register it reads as SrcC 16 and as SrcA/B 8 (conservative); within the window every older MFMA
# of the path is checked too, unless a VALU read of its result (a 'touch') proves it complete.
RAW_STATES, SRCC_WAR_STATES, SRCAB_WAR_STATES = 13, 16, 8


def check_clamp_runs(lines):
    """Checks every v_cvt_pk_bf16_f32 ... clamp run of one disassembly (test below); returns the count."""
    runs_checked = 0
    ins = [(ln, _parse(ln)) for ln in lines]
    ins = [(ln, x) for ln, x in ins if x]
    # predecessors of every instruction: the one before it (unless that one is an
    # unconditional jump or the end of the program) and every branch that targets it
    addr_ix = {x[0]: n for n, (_, x) in enumerate(ins)}
    preds = {n: ([n - 1] if n > 0 and ins[n - 1][1][1] not in ("s_branch", "s_endpgm") else [])
             for n in range(len(ins))}
    for n, (ln, (addr, mn, _, _, _)) in enumerate(ins):
        m = re.match(r"\s+s_(?:c)?branch\w*\s+(-?\d+)", ln)
        if m:
            off = int(m.group(1))
            off = off - 65536 if off >= 32768 else off
            t = addr_ix.get(addr + 4 + 4 * off)
            if t is not None:
                preds[t].append(n)
    i = 0
    while i < len(ins):
        if not (ins[i][1][1] == "v_cvt_pk_bf16_f32" and " clamp" in ins[i][0]):
            i += 1
            continue
        j = i
        while j < len(ins) and ins[j][1][1] == "v_cvt_pk_bf16_f32" and " clamp" in ins[j][0]:
            j += 1
        run = ins[i:j]
        S = set().union(*[x[3] for _, x in run])
        D = set().union(*[x[2] for _, x in run])
        where = f"run @ {run[0][1][0]:#x}"
        # backward walk over every path into the run, up to 24 wait states deep
        stack, seen = [(k, 0, frozenset()) for k in preds[i]], set()
        while stack:
            k, W, read_since = stack.pop()
            if (k, W, read_since) in seen:
                continue
            seen.add((k, W, read_since))
            ln, (addr, mn, dst, src, srcc) = ins[k]
            if mn.startswith("v_mfma"):
                if dst & read_since:
                    continue  # touched: it completed, and every MFMA of this path before it
                # distance to the first instruction of the run that touches each register involved
                for q in range(i, j):
                    qd, qs = ins[q][1][2], ins[q][1][3]
                    need = RAW_STATES if dst & (qs | qd) else 0
                    if src & qd:
                        need = max(need, SRCC_WAR_STATES if srcc & qd else SRCAB_WAR_STATES)
                    assert W + (q - i) >= need, f"{where}: MFMA at {addr:#x} ({W + q - i} wait states before) not touched"
            if mn.startswith("v_") and not mn.startswith("v_mfma"):
                read_since = read_since | frozenset(src)
            W += _wait_states(mn, ln)
            if W < 24:
                stack.extend((q, W, read_since) for q in preds[k])
        # forward: first MFMA reading a result of the run, counted from the run's last write of
        # a register it reads
        W, k = 0, j
        while k < len(ins):
            ln, (addr, mn, dst, src, _) = ins[k]
            if mn.startswith("v_mfma") and src & D:
                last = max(q for q in range(i, j) if ins[q][1][2] & src)
                assert W + (j - 1 - last) >= 2, f"{where}: MFMA {W + j - 1 - last} wait states after the run"
                break
            if mn.startswith(("s_branch", "s_cbranch", "s_endpgm")):
                break
            W += _wait_states(mn, ln)
            k += 1
        runs_checked += 1
        i = j
    return runs_checked


def test_bf16_clamp_conversions_are_hazard_free(tmp_path):
    """the bf16 ReLU folded into the conversion is inline asm (nr_mlp16.h
    relu_clamp_bf16_x*), invisible to the compiler's hazard recognizer.  Its safety rests on a
    VALU 'touch' of every accumulator the block converts (the compiler puts the MFMA -> VALU wait
    states before the touch) and on the block's trailing s_nop 1 (a VALU write needs 2 wait
    states before an MFMA reads it).  Checked on the generated code of every instance:
      * on every path into each run of v_cvt_pk_bf16_f32 ... clamp (control flow followed
        through branches and branch targets), every MFMA that writes a register the run reads,
        or reads or writes a register the run writes, is either followed before the run by a VALU
        read of its result (the touch) or far enough ahead of it (RAW_STATES / *_WAR_STATES: the
        pipelined streams of nr_mlp16_asm.h, whose runs sit between MFMAs, rely on distance); a
        path is followed until 24 wait states separate it from the run (beyond every window);
      * the first MFMA after the run that reads one of its results is >= 2 wait states after it."""
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    so = tmp_path / "libnr.so"
    shutil.copy(_lib.LIB_PATH, so)
    subprocess.run([objdump, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    objs = sorted(p for p in tmp_path.iterdir() if "amdgcn" in p.name and "gfx950" in p.name)
    assert objs
    runs, caught = 0, 0
    for p in objs:
        lines = subprocess.run([objdump, "-d", str(p)], check=True, capture_output=True, text=True).stdout.splitlines()
        n = check_clamp_runs(lines)
        runs += n
        if n:
            # the checker itself: without the touches (v_and_b32 vX, 1, vY) it must object
            # wherever a run reads MFMA results in place (runs that read v_accvgpr_read copies
            # of AGPR accumulators are safe without them: the copies are the touch)
            cut = [ln for ln in lines if not re.match(r"\s+v_and_b32_e32 v\d+, 1, v\d+\s", ln)]
            try:
                check_clamp_runs(cut)
            except AssertionError as e:
                assert "not touched" in str(e)
                caught += 1
    assert runs > 0 and caught > 0


def test_mlp_stream_header_is_current_and_hazard_checked():
    """nr_mlp16_asm.h (the 16-bit MLP's pipelined instruction streams) is what
    tools/gen_mlp_asm.py generates today, and the generator's hazard check accepts every stream
    (it raises on a violation before writing or comparing)."""
    import subprocess
    import sys
    gen = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "gen_mlp_asm.py")
    r = subprocess.run([sys.executable, gen, "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_mlp_stream_checker_rejects_hazards():
    """The generator's checker catches each hazard class it guards (a stream edited to break it)."""
    import importlib.util
    gen = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "gen_mlp_asm.py")
    spec = importlib.util.spec_from_file_location("gen_mlp_asm", gen)
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    for nt in (4, 2):
        _broken_streams(g, g.build("bf16", True, nt))


def _broken_streams(g, st):
    ins = st.ins

    def broken(edit):
        s2 = g.Stream(st.nt)
        s2.ins = edit(list(ins))
        with pytest.raises(AssertionError):
            g.check(s2)

    first_nop = next(i for i, x in enumerate(ins) if x[1] == "nop")
    broken(lambda l: l[:first_nop] + l[first_nop + 1:])                          # MFMA -> VALU read too soon
    first_wait = next(i for i, x in enumerate(ins) if x[1] == "wait")
    broken(lambda l: l[:first_wait] + l[first_wait + 1:])                        # LDS data used before the wait
    last_cvt = max(i for i, x in enumerate(ins) if x[1] == "valu")
    broken(lambda l: l[:last_cvt - 20])                                          # MFMA still in flight at the exit
