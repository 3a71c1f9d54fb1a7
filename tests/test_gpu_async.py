"""Asynchronous FastCDC batches (cdc_chunk_batch_device_async / cdc_batch_sync).

Batches of more than 8 MiB are enqueued back to back with no host wait, each
with its own host staging block (three in rotation) and device table slot
(two); results are collected later.  Every batch's chunks must equal the
oracle's, whatever the interleaving: multi-stream batches,
ragged and empty streams, different outputs per batch, bursts ended by
cdc_batch_sync or by a synchronous call, and small batches that complete
inside the call.  Parity vs the fastcdc crate is unpinned (GEAR placeholder,
DESIGN.md); these tests pin the GPU path to the oracle (oracle/cdc_oracle.c).
"""
import ctypes

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SIZES = (4096, 8192, 16384)


def _dev_stream(torch, n, seed):
    import chunkfs_amd as c
    b = torch.empty(max(n, 16), dtype=torch.uint8, device="cuda:0")
    c._lib.check(c._lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, seed, None))
    return b


def _check(out, first, bufs, lens):
    for i, (b, n) in enumerate(zip(bufs, lens)):
        got = out[int(first[i]):int(first[i + 1])].cpu().numpy().view(np.uint64)
        ref = oracle.fastcdc(b[:n].cpu().numpy(), *SIZES) if n else np.zeros((0, 2), np.uint64)
        assert got.shape == ref.shape and (got == ref).all(), f"stream {i} ({n} B)"


def test_async_burst_multi_stream_batches():
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*SIZES))
    lens_all = [(64 << 20) + 1, 20 << 20, (33 << 20) + 12345, 0, 9 << 20]
    bufs = [_dev_stream(torch, n, 300 + i) for i, n in enumerate(lens_all)]
    batches = [[0], [1, 2], [3, 4, 1], [2], [0, 1, 2, 3, 4]]
    outs, firsts = [], []
    for idx in batches:
        lens = [lens_all[i] for i in idx]
        cap = ch.batch_max_chunks(lens)
        out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
        firsts.append(ch.chunk_batch_device_async([bufs[i].data_ptr() for i in idx], lens, out.data_ptr(), cap))
        outs.append(out)
    total = ch.batch_sync()
    torch.cuda.synchronize()
    assert total == int(firsts[-1][-1])
    for idx, out, first in zip(batches, outs, firsts):
        _check(out, first, [bufs[i] for i in idx], [lens_all[i] for i in idx])
    assert ch.batch_sync() == 0  # nothing in flight
    ch.close()


def test_async_repeated_batch_and_sync_call_drains():
    """The bench's shape (one buffer, one output, back-to-back) ended by a
    synchronous call, then by cdc_batch_sync."""
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*SIZES))
    n = (96 << 20) + 7
    buf = _dev_stream(torch, n, 77)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    fs = [ch.chunk_batch_device_async([buf.data_ptr()], [n], out.data_ptr(), cap) for _ in range(7)]
    first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)  # drains, then runs
    for f in fs:
        assert (f == first).all()
    _check(out, first, [buf], [n])
    t = ch.last_timing()
    assert t["scan_ms"] > 0 and t["total_ms"] >= t["scan_ms"]
    for _ in range(3):
        f = ch.chunk_batch_device_async([buf.data_ptr()], [n], out.data_ptr(), cap)
    assert ch.batch_sync() == int(first[-1])
    assert (f == first).all()
    ch.close()


def test_async_small_batches_complete_in_call():
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*SIZES))
    big = (40 << 20) + 3
    small = (1 << 20) + 5
    b0, b1 = _dev_stream(torch, big, 5), _dev_stream(torch, small, 6)
    cap0, cap1 = ch.batch_max_chunks([big]), ch.batch_max_chunks([small])
    o0 = torch.empty((cap0, 2), dtype=torch.int64, device="cuda:0")
    o1 = torch.empty((cap1, 2), dtype=torch.int64, device="cuda:0")
    f0 = ch.chunk_batch_device_async([b0.data_ptr()], [big], o0.data_ptr(), cap0)
    f1 = ch.chunk_batch_device_async([b1.data_ptr()], [small], o1.data_ptr(), cap1)  # drains f0, then runs
    assert int(f1[-1]) > 0 and int(f0[-1]) > 0  # both filled on return
    _check(o0, f0, [b0], [big])
    _check(o1, f1, [b1], [small])
    assert ch.batch_sync() == 0
    ch.close()


def test_async_other_algorithms_are_synchronous():
    import torch
    import chunkfs_amd as c
    ch = c.RabinChunker(c.SizeParams(*SIZES))
    n = 24 << 20
    b = _dev_stream(torch, n, 9)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    f = ch.chunk_batch_device_async([b.data_ptr()], [n], out.data_ptr(), cap)
    got = out[:int(f[-1])].cpu().numpy().view(np.uint64)
    ref = oracle.cdc("rabin", b[:n].cpu().numpy(), *SIZES)
    assert got.shape == ref.shape and (got == ref).all()
    ch.close()


def test_async_batches_sample_events():
    """Async batches record their HIP events one in four (an event costs the
    stream ~4 us); synchronous ones always do.  The unsampled report 0 ms."""
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*SIZES))
    n = 24 << 20
    buf = _dev_stream(torch, n, 11)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    for _ in range(8):
        ch.chunk_batch_device_async([buf.data_ptr()], [n], out.data_ptr(), cap)
    ch.batch_sync()
    hist = [ch.timing_back(k) for k in range(8)]
    timed = [h for h in hist if h["total_ms"] > 0]
    assert len(timed) == 2 and all(h["scan_ms"] > 0 and h["resolve_ms"] > 0 for h in timed)
    assert sum(h["timed"] for h in hist) == 2 and all(h["path"] == 0 for h in hist)
    ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
    assert ch.last_timing()["scan_ms"] > 0
    ch.close()
