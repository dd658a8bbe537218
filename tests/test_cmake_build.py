"""The top-level CMakeLists.txt (north_star: the host side stays C++ with CMake) builds
libnr.so and the reference's two drivers (reference src/CMakeLists.txt:47-83:
neuralSDFRenderer, simpleInfer) for gfx950, plus the HighFive-loader check.  CPU only:
the build is a cross-compile; the drivers are not run (they need a GPU), the HighFive
loader is (host-only layers)."""
import ctypes
import os
import shutil
import subprocess

import pytest

from conftest import REPO
from test_lib_cpu import assert_no_packed_fp32, header_symbols


@pytest.fixture(scope="module")
def cmake_build(tmp_path_factory):
    if not shutil.which("cmake"):
        pytest.skip("cmake not available")
    b = tmp_path_factory.mktemp("cmake")
    env = dict(os.environ)
    subprocess.run(["cmake", "-S", REPO, "-B", str(b), "-DCMAKE_PREFIX_PATH=/opt/rocm"], check=True,
                   capture_output=True, env=env, timeout=300)
    r = subprocess.run(["cmake", "--build", str(b), "-j", str(min(8, os.cpu_count() or 2))], capture_output=True,
                       text=True, env=env, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return b


def test_cmake_targets(cmake_build):
    for exe in ("neuralSDFRenderer", "simpleInfer", "highfive_load"):
        assert os.access(cmake_build / "bin" / exe, os.X_OK), exe
    lib = ctypes.CDLL(str(cmake_build / "lib" / "libnr.so"))
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_cmake_libnr_device_code(cmake_build, tmp_path):
    assert_no_packed_fp32(cmake_build / "lib" / "libnr.so", tmp_path)


def test_cmake_highfive_loader_runs(cmake_build):
    from conftest import GEOMS
    import cudaneuralrender_amd as nr
    for g in GEOMS:
        r = subprocess.run([str(cmake_build / "bin" / "highfive_load"), nr.geometry_path(g)], capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0 and r.stdout.splitlines()[0] == "layers 9 weights 7296 biases 257", r.stdout[:200]
