"""C++ host mirror (include/chunkfs_amd.hpp) over the C ABI.

CPU: the header-only mirror and the example compile and link against
libchunkfs_amd.so.  GPU: the example runs (FSChunker known answer, FastCDC
tiling, write-path segmentation invariance)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "_build", "cdc_example")


def _build_example():
    from chunkfs_amd import _lib  # ensures the library exists
    assert os.path.exists(_lib.LIB_PATH)
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "cdc_example.cpp"),
                    "-L", os.path.dirname(_lib.LIB_PATH), "-lchunkfs_amd",
                    "-Wl,-rpath," + os.path.dirname(_lib.LIB_PATH), "-o", EXE], check=True)


def test_cpp_mirror_compiles_and_links():
    _build_example()
    assert os.access(EXE, os.X_OK)


@pytest.mark.gpu
def test_cpp_mirror_runs_on_gpu():
    _build_example()
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Fixed size chunking" in r.stdout and "write path" in r.stdout
