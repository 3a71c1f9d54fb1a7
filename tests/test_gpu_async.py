"""Asynchronous FastCDC batches (cdc_chunk_batch_device_async / cdc_batch_sync).

Batches of more than 8 MiB are enqueued back to back with no host wait, each
with its own host staging block (three in rotation) and device table slot
(four); results are collected later.  Where the sizes allow (avg 8 KiB and up
at max <= 64 KiB) each batch's resolve runs on a second stream beside the
next batch's scan (the overlap kernel set, fastcdc_ovl.hip).  Every batch's chunks must equal the
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
    # the small call drained f0 on the caller's behalf: its count is what the
    # next cdc_batch_sync reports, once
    assert ch.batch_sync() == int(f0[-1])
    assert ch.batch_sync() == 0
    ch.close()


def test_async_other_algorithms():
    """Segment-walk batches past 8 MiB are in flight until batch_sync (two
    internal contexts, tests/test_gpu_walk_async.py); smaller ones complete
    inside the call."""
    import torch
    import chunkfs_amd as c
    ch = c.RabinChunker(c.SizeParams(*SIZES))
    for n, inside in ((24 << 20, False), (4 << 20, True)):
        b = _dev_stream(torch, n, 9)
        cap = ch.batch_max_chunks([n])
        out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
        f = ch.chunk_batch_device_async([b.data_ptr()], [n], out.data_ptr(), cap)
        if inside:
            assert int(f[-1]) > 0 and ch.batch_sync() == 0
        else:
            assert ch.batch_sync() == int(f[-1]) > 0
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


def test_async_then_host_chunk_data_small_path():
    """cdc_chunk_data on a 1 MiB host buffer (the one-launch small kernel, which
    reuses host staging block 0) while async batches are in flight: the call
    completes them first, and both results are exact."""
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*SIZES))
    n = (24 << 20) + 5
    bufs = [_dev_stream(torch, n, 500 + k) for k in range(4)]
    cap = ch.batch_max_chunks([n])
    outs = [torch.empty((cap, 2), dtype=torch.int64, device="cuda:0") for _ in bufs]
    fs = [ch.chunk_batch_device_async([b.data_ptr()], [n], o.data_ptr(), cap) for b, o in zip(bufs, outs)]
    host = np.frombuffer(np.random.default_rng(3).bytes((1 << 20) + 17), dtype=np.uint8)
    got = ch.chunk_array(host)  # drains the four batches, then the small path
    ref = oracle.fastcdc(host, *SIZES)
    assert got.shape == ref.shape and (got == ref).all()
    assert ch.batch_sync() == int(fs[-1][-1])
    for b, o, f in zip(bufs, outs, fs):
        _check(o, f, [b], [n])
    ch.close()


def test_async_implicit_drain_result_held_for_batch_sync():
    """cdc_last_timing completes the batches in flight; the next cdc_batch_sync
    returns the last batch's count (not 0), then 0."""
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*SIZES))
    n = 40 << 20
    buf = _dev_stream(torch, n, 21)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    fs = [ch.chunk_batch_device_async([buf.data_ptr()], [n], out.data_ptr(), cap) for _ in range(5)]
    ch.last_timing()
    assert int(fs[-1][-1]) > 0 and all((f == fs[-1]).all() for f in fs)
    assert ch.batch_sync() == int(fs[-1][-1])
    assert ch.batch_sync() == 0
    _check(out, fs[-1], [buf], [n])
    ch.close()


@pytest.mark.parametrize("overlap", ["2", "1", "0"])
def test_async_long_burst_overlap_on_and_off(monkeypatch, overlap):
    """Twelve back-to-back batches of varying shape (every device slot and host
    block reused several times) on two streams with the regular kernels (the
    default), with the overlap set, and on one stream: identical, exact
    chunks."""
    import torch
    import chunkfs_amd as c
    monkeypatch.setenv("CHUNKFS_AMD_OVERLAP", overlap)
    ch = c.FastChunker(c.SizeParams(*SIZES))
    lens_all = [(48 << 20) + 3, 9 << 20, (17 << 20) + 1000, 0, (12 << 20) + 64]
    bufs = [_dev_stream(torch, n, 700 + i) for i, n in enumerate(lens_all)]
    shapes = [[0], [1, 2], [4], [2, 3, 1], [0, 4], [1], [3, 0], [2], [4, 1, 0], [0], [1, 2, 4], [2, 0]]
    res = []
    for idx in shapes:
        lens = [lens_all[i] for i in idx]
        cap = ch.batch_max_chunks(lens)
        out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
        res.append((idx, out, ch.chunk_batch_device_async([bufs[i].data_ptr() for i in idx], lens, out.data_ptr(),
                                                          cap)))
    assert ch.batch_sync() == int(res[-1][2][-1])
    torch.cuda.synchronize()
    for idx, out, first in res:
        _check(out, first, [bufs[i] for i in idx], [lens_all[i] for i in idx])
    ch.close()


def test_async_dense_sizes_take_the_standard_set():
    """2/4/8 KiB: records too dense for the overlap set's windows; the async
    batches run the standard kernels, still exact."""
    import torch
    import chunkfs_amd as c
    sizes = (2048, 4096, 8192)
    ch = c.FastChunker(c.SizeParams(*sizes))
    n = (20 << 20) + 9
    buf = _dev_stream(torch, n, 31)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    fs = [ch.chunk_batch_device_async([buf.data_ptr()], [n], out.data_ptr(), cap) for _ in range(5)]
    ch.batch_sync()
    got = out[int(fs[-1][0]):int(fs[-1][1])].cpu().numpy().view(np.uint64)
    ref = oracle.fastcdc(buf[:n].cpu().numpy(), *sizes)
    assert got.shape == ref.shape and (got == ref).all()
    ch.close()
