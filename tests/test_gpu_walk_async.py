"""Async batches of the segment-walk algorithms (-m gpu): cdc_chunk_batch_device_async
on Rabin / UltraCDC / LeapCDC / SeqCDC handles runs alternate batches on two
contexts (Engine::walk_submit), each on its own stream and host worker thread.
Every batch bit-exact vs the CPU oracle, whatever its context, and the drain
semantics those of the FastCDC pipeline (batch_sync, implicit drains)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ALGOS = ["rabin", "ultra", "leap", "seq"]
SIZES = (4096, 8192, 16384)


def make(algo, sizes=SIZES):
    import chunkfs_amd as c
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(algo)
    p = c.SizeParams(*sizes)
    return cls(p) if cls else c.SeqChunker(c.OperationMode.Increasing, p)


def _dev(torch, n, seed):
    a = oracle.splitmix64_bytes(n, seed)
    b = torch.empty(max(n, 16), dtype=torch.uint8, device="cuda:0")
    b[:n] = torch.from_numpy(a).to("cuda:0")
    return b, a


def _check(algo, out, first, arrays, sizes=SIZES):
    got = out.cpu().numpy().view(np.uint64)
    for i, a in enumerate(arrays):
        ref = oracle.cdc(algo, a, *sizes)
        seg = got[int(first[i]):int(first[i + 1])]
        assert seg.shape == ref.shape and (seg == ref).all(), f"{algo} stream {i} len={len(a)}"


@pytest.mark.parametrize("algo", ALGOS)
def test_walk_async_burst(algo):
    """Six back-to-back batches of varying shape (every context reused),
    results checked after one batch_sync."""
    import torch
    ch = make(algo)
    lens_all = [(12 << 20) + 5, 9 << 20, (5 << 20) + 999, 0, (10 << 20) + 64]
    data = [_dev(torch, n, 900 + i) for i, n in enumerate(lens_all)]
    shapes = [[0], [1, 2], [4, 3], [2, 0, 1], [1], [4, 2]]
    res = []
    for idx in shapes:
        lens = [lens_all[i] for i in idx]
        cap = ch.batch_max_chunks(lens)
        out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
        first = ch.chunk_batch_device_async([data[i][0].data_ptr() for i in idx], lens, out.data_ptr(), cap)
        res.append((idx, out, first))
    assert ch.batch_sync() == int(res[-1][2][-1])
    assert ch.batch_sync() == 0
    for idx, out, first in res:
        _check(algo, out, first, [data[i][1] for i in idx])
    ch.close()


@pytest.mark.parametrize("algo", ["rabin", "seq"])
def test_walk_async_implicit_drain(algo):
    """A synchronous call on the handle completes the async batches first;
    the next batch_sync returns what that drain collected."""
    import torch
    ch = make(algo)
    b, a = _dev(torch, 11 << 20, 31)
    cap = ch.batch_max_chunks([len(a)])
    outs = [torch.empty((cap, 2), dtype=torch.int64, device="cuda:0") for _ in range(3)]
    firsts = [ch.chunk_batch_device_async([b.data_ptr()], [len(a)], o.data_ptr(), cap) for o in outs]
    small = oracle.splitmix64_bytes(300_000, 5)
    got = ch.chunk_array(small)  # (drains the three batches first)
    ref_small = oracle.cdc(algo, small, *SIZES)
    assert got.shape == ref_small.shape and (got.view(np.uint64) == ref_small).all()
    ref = oracle.cdc(algo, a, *SIZES)
    assert ch.batch_sync() == len(ref)
    for o, f in zip(outs, firsts):
        _check(algo, o, f, [a])
    ch.close()


def test_walk_async_off_equals_on(monkeypatch):
    """CHUNKFS_AMD_WALK_ASYNC=0 (batches complete inside the call) gives the
    same chunks."""
    import torch
    b, a = _dev(torch, 13 << 20, 77)
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("CHUNKFS_AMD_WALK_ASYNC", mode)
        ch = make("ultra")
        cap = ch.batch_max_chunks([len(a)])
        o = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
        f = ch.chunk_batch_device_async([b.data_ptr()], [len(a)], o.data_ptr(), cap)
        got = ch.batch_sync()
        n = int(f[-1])
        assert got == (n if mode == "1" else 0)  # (off: the batch completed inside the call)
        outs[mode] = o[:n].cpu().numpy()
        ch.close()
    assert (outs["1"] == outs["0"]).all()


def test_walk_async_rabin_poly_applies():
    """A polynomial set on the handle reaches the async contexts."""
    import torch
    ch = make("rabin")
    poly = 0x3DA3358B4DC173
    ch.set_poly(poly)
    b, a = _dev(torch, 10 << 20, 12)
    cap = ch.batch_max_chunks([len(a)])
    o = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    ch.chunk_batch_device_async([b.data_ptr()], [len(a)], o.data_ptr(), cap)
    n = ch.batch_sync()
    sync = make("rabin")
    sync.set_poly(poly)
    ref = sync.chunk_array(a)
    assert n == len(ref) and (o[:n].cpu().numpy().view(np.uint64) == ref.view(np.uint64)).all()
    ch.close()
    sync.close()
