"""Torch-free native build (CMakeLists.txt): configure + build the C library, the driver and
the unit tests with CMake's HIP language for gfx950, then run the CPU unit tests through ctest
(the reference builds its driver with the toolkit alone, reference CMakeLists.txt:1-14)."""
import os
import shutil
import subprocess

import pytest

from cuda_knearests_amd.utils import REPO

BUILD = REPO / "build_cmake"


def _cmake():
    return shutil.which("cmake")


@pytest.mark.skipif(_cmake() is None, reason="cmake not installed")
def test_cmake_build_and_ctest_cpu():
    BUILD.mkdir(exist_ok=True)
    env = dict(os.environ)
    r = subprocess.run([_cmake(), "-S", str(REPO), "-B", str(BUILD), "-DCMAKE_BUILD_TYPE=Release"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run([_cmake(), "--build", str(BUILD), "-j", "8"], capture_output=True, text=True, timeout=1500,
                       env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for exe in ("knn_cli", "knn_unit"):
        assert (BUILD / exe).exists()
    assert (BUILD / "libknearests.so").exists()
    # no libtorch anywhere in the dependency closure of the CMake-built library
    ldd = subprocess.run(["ldd", str(BUILD / "libknearests.so")], capture_output=True, text=True).stdout
    assert "torch" not in ldd and "amdhip64" in ldd
    r = subprocess.run(["ctest", "--test-dir", str(BUILD), "-LE", "gpu", "--output-on-failure"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
