"""CPU suite: the C-ABI library builds, loads and exports every declared symbol.

No compute calls are made here (no GPU in this container); creating a handle
must fail LOUDLY (CDC_EDEVICE) rather than fall back to the CPU.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "chunkfs_amd.h")
DEBUG_HEADER = os.path.join(ROOT, "include", "chunkfs_amd_debug.h")


def _declared(path=HEADER):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cdc_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from chunkfs_amd import _lib
    L = _lib.lib()
    declared = _declared()
    assert declared, "header parse failed"
    assert sorted(_lib.EXPORTS) == declared
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (cdc_[a-z0-9_]+)$", out, flags=re.M))
    for name in declared:
        assert name in exported, name
        assert hasattr(L, name)
    debug = _declared(DEBUG_HEADER)
    assert sorted(_lib.DEBUG_EXPORTS) == debug
    for name in debug:
        assert name in exported, name


def test_version_string():
    import chunkfs_amd
    assert "gfx950" in chunkfs_amd.version()


def test_abi_version_matches_header():
    from chunkfs_amd import _lib
    m = re.search(r"#define CHUNKFS_AMD_ABI_VERSION (\d+)", open(HEADER).read())
    assert m and _lib.lib().cdc_abi_version() == int(m.group(1))
    assert f"abi {m.group(1)}" in _lib.lib().cdc_version().decode()


def test_header_compiles_as_c():
    src = '#include "chunkfs_amd.h"\nint main(void){cdc_chunk_t c={0,0};(void)c;return sizeof(cdc_chunk_t)==16?0:1;}\n'
    exe = "/tmp/_abi_c_test"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-x", "c", "-", "-o", exe], input=src.encode(), check=True)
    assert subprocess.call([exe]) == 0


def test_code_object_is_gfx950():
    from chunkfs_amd import _lib
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={_lib.LIB_PATH}"], capture_output=True, text=True)
    txt = out.stdout + out.stderr
    if "gfx950" not in txt:  # fall back: search the embedded bundle id
        data = open(_lib.LIB_PATH, "rb").read()
        assert b"gfx950" in data
    else:
        assert "gfx950" in txt


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK),
                    reason="a GPU is visible: the no-GPU failure mode is not observable")
def test_no_gpu_fails_loudly():
    import chunkfs_amd
    with pytest.raises(chunkfs_amd.CdcError) as ei:
        chunkfs_amd.FastChunker(chunkfs_amd.SizeParams(4096, 8192, 16384))
    assert ei.value.code == -3  # CDC_EDEVICE


def test_invalid_sizes_rejected_before_device():
    import chunkfs_amd
    with pytest.raises(chunkfs_amd.CdcError) as ei:
        chunkfs_amd.FastChunker(chunkfs_amd.SizeParams(32, 8192, 16384))
    assert ei.value.code == -1


def test_unsupported_algorithms_raise():
    import chunkfs_amd
    with pytest.raises(NotImplementedError):
        chunkfs_amd.SuperChunker()


def test_walk_chunkers_need_explicit_sizes():
    import chunkfs_amd as c
    for cls in (c.RabinChunker, c.UltraChunker, c.LeapChunker):
        with pytest.raises(TypeError):
            cls()
    with pytest.raises(TypeError):
        c.SeqChunker(c.OperationMode.Increasing)


def test_walk_chunkers_reject_bad_sizes_before_device():
    import chunkfs_amd as c
    bad = [(c.RabinChunker, (0, 10, 20)), (c.UltraChunker, (4, 8, 16)), (c.LeapChunker, (16, 64, 128)),
           (c.RabinChunker, (100, 50, 200))]
    for cls, s in bad:
        with pytest.raises(c.CdcError) as ei:
            cls(c.SizeParams(*s))
        assert ei.value.code == -1
    with pytest.raises(c.CdcError) as ei:
        c.SeqChunker(c.OperationMode.Decreasing, c.SizeParams(64, 128, 256), c.SeqConfig(0, 50, 256))
    assert ei.value.code == -1
    with pytest.raises(c.CdcError) as ei:
        c.SeqChunker(c.OperationMode.Increasing, c.SizeParams(64, 128, 256), c.SeqConfig(5, 1, 0))
    assert ei.value.code == -1


def test_python_mirror_debug_strings():
    import chunkfs_amd as c
    assert repr(c.SizeParams(4096, 8192, 16384)) == "SizeParams { min: 4096, avg: 8192, max: 16384 }"
    assert repr(c.Chunk(3, 4)) == "Chunk { offset: 3, length: 4 }"
    assert list(c.Chunk(3, 4).range()) == [3, 4, 5, 6]
    assert c.SEG_SIZE == 1 << 20
