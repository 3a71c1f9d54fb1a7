"""One-launch small-stream FastCDC (chunkfs_amd/csrc/small.hip) on the GPU.

The reference's StorageWriter calls chunk_data once per 1 MiB segment plus
the carried chunk (storage.rs:302-357); such calls (one stream of at most
4 MiB) run as ONE kernel -- scan, links, chain walk -- reading the pinned ring
slot over PCIe (cdc_chunk_data) or device memory (cdc_chunk_batch_device).
Every result is compared bit-exactly with the oracle's restatement of
fastcdc v2020 (parity vs the crate unpinned: GEAR placeholder), including
the inputs that make the kernel fall back to the regular pipeline."""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SIZES = [(4096, 8192, 16384), (2048, 4096, 8192), (8192, 16384, 32768), (1024, 2048, 8192),
         (8192, 4096, 16384), (16384, 65536, 262144)]


def _fast(sizes, env=None):
    import chunkfs_amd as c
    old = {}
    for k, v in (env or {}).items():
        old[k] = os.environ.get(k)
        os.environ[k] = v
    try:
        return c.FastChunker(c.SizeParams(*sizes))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(got, ref, what):
    got = np.asarray(got, dtype=np.uint64).reshape(-1, 2)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert bad.size == 0, (what, int(bad[0]), got[bad[0]], ref[bad[0]])


def _inputs(n, seed):
    rng = np.random.default_rng(seed)
    rnd = oracle.splitmix64_bytes(n, seed)
    lowent = rng.integers(0, 3, n, dtype=np.uint8)
    mixed = rnd.copy()
    if n > 64:
        a = int(rng.integers(0, n // 2))
        mixed[a:a + n // 3] = 0
    per = np.resize(oracle.splitmix64_bytes(61, 7), n)
    return {"random": rnd, "zeros": np.zeros(n, np.uint8), "lowent": lowent, "zero_region": mixed, "period61": per}


@pytest.mark.parametrize("sizes", SIZES)
def test_small_chunk_data_matches_oracle(sizes):
    import chunkfs_amd as c
    ch = _fast(sizes)
    st0 = c.host_stats(ch)
    lens = [1, 47, 4095, 4096, 4097, 16385, 65536 + 17, (1 << 20) + 4097, (1 << 20) + 16384, (4 << 20) - 1, 4 << 20]
    for n in lens:
        for name, data in _inputs(n, n & 0xFFFF).items():
            _check(ch.chunk_array(data), oracle.fastcdc(data, *sizes), (sizes, n, name))
    st1 = c.host_stats(ch)
    assert st1["small_calls"] - st0["small_calls"] >= len(lens)  # the one-launch kernel took them
    ch.close()


def test_small_reference_loop_1MiB_segments():
    """StorageWriter's loop (buffer = rest ++ 1 MiB segment) through chunk_data:
    every call is one small-kernel launch, and the spans are the oracle's."""
    import chunkfs_amd as c
    sizes = (4096, 8192, 16384)
    data = oracle.splitmix64_bytes((32 << 20) + 777, 2024)
    ch = _fast(sizes)
    st0 = c.host_stats(ch)
    spans, rest = [], np.empty(0, dtype=np.uint8)
    for off in range(0, data.size, 1 << 20):
        buf = np.concatenate([rest, data[off:off + (1 << 20)]])
        chunks = ch.chunk_array(buf)
        spans += [int(x) for x in chunks[:-1, 1]]
        o, ln = (int(x) for x in chunks[-1])
        rest = buf[o:o + ln]
    spans.append(rest.size)
    ref, _ = oracle.fs_write("fast", data, *sizes)
    assert spans == [int(x) for x in ref]
    st1 = c.host_stats(ch)
    # every call went to the small kernel; a feed wait past its poll limit (a
    # descheduled host thread) falls back to the pipeline, exact all the same:
    # a few are tolerated, not required to be 0
    assert st1["small_calls"] - st0["small_calls"] == 33
    t = ch.last_timing()
    assert t["path"] in (1, 0) and (t["path"] == 0 or t["timed"] == 0)  # small kernel: not timed, said so
    assert st1["small_fallbacks"] - st0["small_fallbacks"] <= 3
    ch.close()


def test_small_device_stream_and_ab():
    """cdc_chunk_batch_device on one small device stream (the kernel reads HBM),
    and the same bytes with the small kernel off (CHUNKFS_AMD_SMALL=0) and with
    the host path's device copy (CHUNKFS_AMD_SMALL_ZC=0): identical chunks."""
    import torch
    sizes = (4096, 8192, 16384)
    on, off, dma = _fast(sizes), _fast(sizes, {"CHUNKFS_AMD_SMALL": "0"}), _fast(sizes, {"CHUNKFS_AMD_SMALL_ZC": "0"})
    for n in (4096 * 3 + 5, (1 << 20) + 12345, (3 << 20) + 1):
        data = oracle.splitmix64_bytes(n, n)
        ref = oracle.fastcdc(data, *sizes)
        buf = torch.from_numpy(data).cuda()
        for ch in (on, off):
            cap = ch.batch_max_chunks([n])
            out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
            first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
            _check(out[:int(first[1])].cpu().numpy().view(np.uint64), ref, ("device", n))
        for ch in (on, off, dma):
            _check(ch.chunk_array(data), ref, ("host", n))
    for ch in (on, off, dma):
        ch.close()


def test_small_fallback_dense_records():
    """A GEAR table whose entry 0 is 0 makes every position of a zero run a
    record: the kernel's budgets overflow, it raises the fallback word and the
    regular pipeline answers -- still bit-exact."""
    import chunkfs_amd as c
    sizes = (4096, 8192, 16384)
    gear = oracle.splitmix64_bytes(256 * 8, 99).view(np.uint64).copy()
    gear[0] = 0
    ch = _fast(sizes)
    ch.set_gear(gear)
    st0 = c.host_stats(ch)
    data = oracle.splitmix64_bytes((1 << 20) + 333, 5)
    data[100000:400000] = 0
    _check(ch.chunk_array(data), oracle.fastcdc(data, *sizes, gear=gear), "dense")
    st1 = c.host_stats(ch)
    assert st1["small_fallbacks"] - st0["small_fallbacks"] == 1
    data = oracle.splitmix64_bytes((1 << 20) + 333, 6)
    _check(ch.chunk_array(data), oracle.fastcdc(data, *sizes, gear=gear), "random, custom gear")
    assert c.host_stats(ch)["small_fallbacks"] == st1["small_fallbacks"]
    ch.close()
