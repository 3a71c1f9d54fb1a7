"""The parity suite against pipeline 2 (cdc_kernels.hip: per-lane sub-span
scan, record links, lane-per-span walk), selected with CHUNKFS_AMD_PIPELINE=2.

Pipeline 2 was written while the GPU pool was unreachable, so it is not the
default and this module only runs when CHUNKFS_AMD_TEST_PIPELINE2=1 (an
explicit, time-limited GPU run), never as part of an unattended `-m gpu`
pass.  It re-runs every test of test_gpu_parity.py with pipeline 2.
"""
import os

import pytest

if os.environ.get("CHUNKFS_AMD_TEST_PIPELINE2") != "1":
    pytest.skip("pipeline 2 parity: set CHUNKFS_AMD_TEST_PIPELINE2=1", allow_module_level=True)

import ctypes  # noqa: E402

import numpy as np  # noqa: E402

import oracle  # noqa: E402

pytestmark = pytest.mark.gpu


def _handle(pipeline, sizes=(4096, 8192, 16384)):
    os.environ["CHUNKFS_AMD_PIPELINE"] = pipeline
    import chunkfs_amd as c
    return c.FastChunker(c.SizeParams(*sizes))


def _copy(ch, what, count, dtype):
    from chunkfs_amd import _lib
    out = np.zeros(count, dtype=dtype)
    got = _lib.check(_lib.lib().cdc_debug_copy(ch._h, what, out.ctypes.data, out.nbytes))
    assert got == out.nbytes
    return out


def _stage(ch, data):
    from chunkfs_amd import _lib
    chunks = ch.chunk_array(data)
    cap = _lib.lib().cdc_debug_record_cap(ch._h)
    spans = (data.size + 65535) // 65536
    counts = _copy(ch, 0, spans, np.uint32)
    recs = _copy(ch, 1, spans * cap, np.uint32).reshape(spans, cap)
    return chunks, cap, counts, recs


def test_stage1_scan_records_match_pipeline1():
    """Stage 1: the sub-span scan must emit exactly pipeline 1's candidate
    records (offset | hit flags; pipeline 1's bits 24..29 are its truncated
    precompute and are masked off)."""
    from chunkfs_amd import _lib
    data = oracle.splitmix64_bytes((4 << 20) + 12345, 17)
    c1, cap1, n1, r1 = _stage(_handle("1"), data)
    h2 = _handle("2")
    assert _lib.lib().cdc_debug_pipeline(h2._h) == 2
    c2, cap2, n2, r2 = _stage(h2, data)
    assert cap1 == cap2
    assert (n1 == n2).all(), np.nonzero(n1 != n2)[0][:10]
    m = np.uint32(0xC0FFFFFF)
    for g in range(n1.size):
        k = min(int(n1[g]), cap1)
        assert ((r1[g, :k] & m) == (r2[g, :k] & m)).all(), g
    assert (c1 == c2).all()


def test_stage2_links_match_cpu_model():
    """Stage 2: every record link equals the CPU model's next-chunk start."""
    from test_resolve_model import Model
    sizes = (4096, 8192, 16384)
    data = oracle.splitmix64_bytes(2 << 20, 23)
    ch = _handle("2", sizes)
    chunks, cap, counts, recs = _stage(ch, data)
    nxt = _copy(ch, 2, counts.size * cap, np.uint64).reshape(counts.size, cap)
    model = Model(data, *sizes)
    checked = 0
    for g in range(counts.size):
        for k in range(min(int(counts[g]), cap)):
            v = int(nxt[g, k])
            if not v >> 63:
                continue  # left to the walk (overflowed neighbour)
            c = g * 65536 + (int(recs[g, k]) & 0xFFFFFF)
            assert c + (v & ((1 << 25) - 1)) == model.step(c), (g, k, c)
            checked += 1
    assert checked > 100
    assert (chunks == oracle.fastcdc(data, *sizes)).all()


os.environ["CHUNKFS_AMD_PIPELINE"] = "2"
from test_gpu_parity import *  # noqa: E402,F401,F403  (same tests, pipeline 2 handles)
