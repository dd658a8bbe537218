"""AddressSanitizer + UndefinedBehaviorSanitizer build of the code that reads untrusted files --
the Keras HDF5 reader (csrc/h5_keras.cpp) and the PNG decoder (csrc/png_codec.cpp) -- and of the
CPU oracle (oracle/nr_oracle.c), run over truncated and bit-flipped copies of the bundled .h5 and
.png files.  Every malformed file must be rejected with an error
message; the sanitizers abort on any out-of-bounds access, leak, overflow or undefined behaviour.
Host code only (g++/gcc on the CPU; GPU sanitizers are not available on this pool)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "cudaneuralrender_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    d = tmp_path_factory.mktemp("san")
    inc = ["-I" + CSRC, "-I" + os.path.join(REPO, "include"), "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    objs = []
    for src in ("h5_keras.cpp", "png_codec.cpp"):
        o = str(d / (src + ".o"))
        subprocess.run(["g++", "-std=c++17", *SAN, *inc, "-c", os.path.join(CSRC, src), "-o", o], check=True)
        objs.append(o)
    o = str(d / "nr_oracle.o")
    subprocess.run(["gcc", "-std=c11", *SAN, "-fopenmp", "-ffp-contract=off", "-c", os.path.join(REPO, "oracle", "nr_oracle.c"),
                    "-o", o], check=True)
    objs.append(o)
    exe = str(d / "parser_sanitize")
    subprocess.run(["g++", "-std=c++17", *SAN, *inc, os.path.join(REPO, "tests", "cpp", "parser_sanitize.cpp"), *objs,
                    "-fopenmp", "-lz", "-lm", "-o", exe], check=True)
    return exe


def corrupt_copies(src, outdir, seed, n_trunc=40, n_flip=160):
    """Truncations at spread lengths (every header field boundary region included) and copies with
    1-8 random bit flips, the flips biased towards the first 4 KiB (superblock, object headers,
    PNG chunk headers) where a parser's offsets and sizes come from."""
    data = open(src, "rb").read()
    rng = np.random.default_rng(seed)
    paths = []
    cuts = sorted(set([0, 1, 7, 8, 9, 16, 33, 64, 100, 200, 512, 1024, 2048, 4096] +
                      [int(x) for x in rng.integers(1, len(data), n_trunc)]))
    for k, c in enumerate(c for c in cuts if c < len(data)):
        p = os.path.join(outdir, f"{os.path.basename(src)}.t{k}")
        open(p, "wb").write(data[:c])
        paths.append(p)
    for k in range(n_flip):
        b = bytearray(data)
        for _ in range(int(rng.integers(1, 9))):
            lim = min(len(b), 4096) if rng.random() < 0.7 else len(b)
            i = int(rng.integers(0, lim))
            b[i] ^= 1 << int(rng.integers(0, 8))
        p = os.path.join(outdir, f"{os.path.basename(src)}.f{k}")
        open(p, "wb").write(bytes(b))
        paths.append(p)
    return paths


def run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    env.pop("LD_PRELOAD", None) if "libasan" in env.get("LD_PRELOAD", "") else None
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, \
        (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_h5_reader_on_corrupted_files(driver, tmp_path):
    import cudaneuralrender_amd as nr
    files = []
    for k, g in enumerate(("plane_1", "car_1")):
        files += corrupt_copies(nr.geometry_path(g), str(tmp_path), seed=k)
    out = run(driver, "h5", nr.geometry_path("plane_1"), *files)
    ok, failed = (int(v) for v in out.split()[2::2])
    assert ok >= 1 and failed > len(files) // 4, out   # the intact file reads; most damage is caught


def test_png_decoder_on_corrupted_files(driver, tmp_path):
    import cudaneuralrender_amd as nr
    files = []
    for k, m in enumerate(("Chrome", "skin-matcap")):
        try:
            path = nr.matcap_path(m)
        except Exception:
            continue
        if os.path.exists(path):
            files += corrupt_copies(path, str(tmp_path), seed=10 + k, n_flip=120)
    assert files
    out = run(driver, "png", nr.matcap_path("Chrome"), *files)
    ok, failed = (int(v) for v in out.split()[2::2])
    assert ok >= 1 and failed > len(files) // 4, out


def test_oracle_under_sanitizers(driver):
    import cudaneuralrender_amd as nr
    assert "oracle ok" in run(driver, "oracle", nr.geometry_path("plane_1"))
