"""In-tree build of libchunkfs_amd.so for gfx950 (hipcc cross-compiles without a GPU).

The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libchunkfs_amd.so")
SOURCES = ["fastcdc.hip", "fastcdc_ovl.hip", "small.hip", "walk.hip", "util_kernels.hip", "sha256.hip", "index.hip", "engine.cpp", "hostpath.cpp", "capi.cpp",
           "index_host.cpp"]
HEADERS = ["fastcdc.hpp", "small.hpp", "walk.hpp", "cdc_kernels.hpp", "sha256.hpp", "index.hpp", "engine.hpp"]
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result"]


def source_digest():
    """SHA-256 (first 16 hex digits) over every source and header the library
    is built from: ties a profile under profiles/ to the build it measured."""
    import hashlib
    h = hashlib.sha256()
    files = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [
        os.path.join(ROOT, "include", f) for f in ("chunkfs_amd.h", "chunkfs_amd_tables.h", "chunkfs_amd_debug.h", "chunkfs_amd_cdc_params.h")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force=False, defines=(), lib=None, build_dir=None):
    """Compile every source for gfx950 and link LIB (or `lib`: experiment
    builds with extra -D `defines` into their own `build_dir`)."""
    bdir = build_dir or BUILD
    out_lib = lib or LIB
    os.makedirs(bdir, exist_ok=True)
    common = [os.path.join(CSRC, h) for h in HEADERS] + [
        os.path.join(ROOT, "include", "chunkfs_amd.h"),
        os.path.join(ROOT, "include", "chunkfs_amd_tables.h"),
        os.path.join(ROOT, "include", "chunkfs_amd_debug.h"),
        os.path.join(ROOT, "include", "chunkfs_amd_cdc_params.h"),
    ]
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(bdir, src + ".o")
        objs.append(o)
        deps = [s] + common + ([os.path.join(CSRC, "fastcdc.hip")] if src == "fastcdc_ovl.hip" else [])
        if force or _newer(o, deps):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            _run([HIPCC] + CFLAGS + [f"-D{d}" for d in defines] + lang + ["-c", s, "-o", o])
    if force or _newer(out_lib, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out_lib] + objs)
    return out_lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
