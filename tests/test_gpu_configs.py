"""BASELINE configs 3 and 5 as GPU parity tests (-m gpu), plus low-entropy
streams at scale for every segment-walk rule.

  config 3  RabinChunker 2/4/8 KiB over SURVEY.md §8d's offline substitute for
            the gcc tarball (256 MiB base + 15 seeded edited copies, ~4 GiB):
            chunks bit-exact vs the oracle on every version, and the GPU
            chunk -> SHA-256 -> dedup-index flow gives the same dedup ratio as
            the oracle's chunks + hashlib + a dict with first insert winning
            (reference storage.rs:193-205, database.rs:76).
  config 5  Ultra / Leap (+ Rabin, Seq) at the three size triples, min = avg/4,
            max = 8 avg, on a 256 MiB device-resident stream.
  low entropy  64 MiB constant, 61-byte-period and "random | long zero run at
            an odd offset | random" streams: chains that never merge inside
            the run (every chunk the same length) go through the fix-up rounds.

Parity is vs the oracle's restatements (cdc-chunkers 0.1.3 is absent offline:
parity vs the crate is unpinned; LeapCDC's eligibility function is a stand-in).
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _chunker(algo, sizes):
    import chunkfs_amd as c
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker,
           "fast": c.FastChunker}.get(algo)
    s = c.SizeParams(*sizes)
    return cls(s) if cls else c.SeqChunker(c.OperationMode.Increasing, s)


def _assert_same(gpu, ref, what):
    gpu = np.asarray(gpu, dtype=np.uint64).reshape(-1, 2)
    ref = np.asarray(ref, dtype=np.uint64).reshape(-1, 2)
    if gpu.shape != ref.shape or not (gpu == ref).all():
        n = min(len(gpu), len(ref))
        bad = np.nonzero((gpu[:n] != ref[:n]).any(axis=1))[0]
        i = int(bad[0]) if len(bad) else n
        pytest.fail(f"{what}: {len(gpu)} vs {len(ref)} chunks; first mismatch at #{i}")


def _device_chunks(ch, dev_bufs, lens):
    import torch
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=DEV)
    torch.cuda.synchronize()
    first = ch.chunk_batch_device([b.data_ptr() for b in dev_bufs], lens, out.data_ptr(), cap)
    return first, out


def test_config3_versioned_archive_dedup_ratio():
    import torch
    import chunkfs_amd as c
    from chunkfs_amd.synthetic import versioned_archive
    sizes = (2048, 4096, 8192)
    files = versioned_archive(256 << 20, 16)
    lens = [f.size for f in files]
    assert sum(lens) > (4 << 30) - (64 << 20)
    bufs = [torch.from_numpy(f).to(DEV) for f in files]
    ch = _chunker("rabin", sizes)
    first, out = _device_chunks(ch, bufs, lens)
    total = int(first[-1])
    dig = torch.empty((total, 32), dtype=torch.uint8, device=DEV)
    ix = c.DedupIndex(total + 64)
    for i, b in enumerate(bufs):  # one file write per version: a fresh StorageWriter (storage.rs:79)
        a, z = int(first[i]), int(first[i + 1])
        ch.sha256_chunks_device(b.data_ptr(), out[a:].data_ptr(), z - a, dig[a:].data_ptr())
        ix.insert_device(dig[a:].data_ptr(), out[a:].data_ptr(), z - a)
    torch.cuda.synchronize()
    st = ix.stats()
    got = out[:total].cpu().numpy().view(np.uint64)
    digs = dig.cpu().numpy()
    db, written, k = {}, 0, 0
    for i, f in enumerate(files):
        ref = oracle.cdc("rabin", f, *sizes)
        _assert_same(got[int(first[i]):int(first[i + 1])], ref, f"config 3 version {i}")
        mv = memoryview(f)
        for o, ln in ref:
            d = hashlib.sha256(mv[int(o):int(o) + int(ln)]).digest()
            if k % 97 == 0:  # spot-check the device digests themselves
                assert digs[k].tobytes() == d, f"SHA-256 of chunk {k}"
            db.setdefault(d, int(ln))
            written += int(ln)
            k += 1
    assert st["chunks_written"] == total and st["bytes_written"] == written == sum(lens)
    assert st["unique_chunks"] == len(db) and st["unique_bytes"] == sum(db.values())
    ratio = written / sum(db.values())
    assert st["cdc_dedup_ratio"] == ratio
    assert ratio > 3.0  # 16 versions with ~1 % edits each deduplicate heavily
    ch.close()


@pytest.mark.parametrize("algo", ["ultra", "leap", "rabin", "seq"])
@pytest.mark.parametrize("avg", [2048, 8192, 65536])
def test_config5_size_triples(algo, avg):
    import torch
    from chunkfs_amd import _lib
    sizes = (avg // 4, avg, avg * 8)
    n = (256 << 20) + 4099
    b = torch.empty(n, dtype=torch.uint8, device=DEV)
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 55 + avg, None))
    ch = _chunker(algo, sizes)
    first, out = _device_chunks(ch, [b], [n])
    _assert_same(out[:int(first[1])].cpu().numpy().view(np.uint64), oracle.cdc(algo, b.cpu().numpy(), *sizes),
                 f"config 5 {algo} {sizes}")
    ch.close()


def _low_entropy(kind, n):
    if kind == "zeros":
        return np.zeros(n, dtype=np.uint8)
    if kind == "periodic61":
        return np.resize(oracle.splitmix64_bytes(61, 7), n)
    # random | 48 MiB of zeros starting at an odd offset | random
    d = oracle.splitmix64_bytes(n, 71)
    d[(8 << 20) + 13:(56 << 20) + 13] = 0
    return d


@pytest.mark.parametrize("algo", ["rabin", "ultra", "leap", "seq", "fast"])
@pytest.mark.parametrize("kind", ["zeros", "periodic61", "zero_run"])
@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (2048, 8192, 65536)])
def test_low_entropy_64MiB(algo, kind, sizes):
    import torch
    data = _low_entropy(kind, 64 << 20)
    b = torch.from_numpy(data).to(DEV)
    ch = _chunker(algo, sizes)
    first, out = _device_chunks(ch, [b], [data.size])
    ref = oracle.fastcdc(data, *sizes) if algo == "fast" else oracle.cdc(algo, data, *sizes)
    _assert_same(out[:int(first[1])].cpu().numpy().view(np.uint64), ref, f"{algo} {kind} {sizes}")
    ch.close()


@pytest.mark.parametrize("algo", ["ultra", "leap", "rabin", "seq"])
def test_config5_full_gib_stream_avg64k(algo):
    """Config 5 at its full stream size: one whole 1 GiB splitmix64 stream per
    segment-walk rule at 16/64/512 KiB (min = avg/4, max = 8 avg).  The
    size-independent invariants (exact tiling from 0, min <= len <= max but
    the last chunk, the chunk count near n/avg) hold, and every chunk equals
    the oracle's."""
    import torch
    from chunkfs_amd import _lib
    avg = 65536
    sizes = (avg // 4, avg, avg * 8)
    n = 1 << 30
    b = torch.empty(n, dtype=torch.uint8, device=DEV)
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 5000, None))
    ch = _chunker(algo, sizes)
    first, out = _device_chunks(ch, [b], [n])
    assert int(first[0]) == 0
    got = out[:int(first[1])].cpu().numpy().view(np.uint64)
    off, ln = got[:, 0].astype(np.int64), got[:, 1].astype(np.int64)
    assert off[0] == 0 and (off[1:] == np.cumsum(ln)[:-1]).all() and int(ln.sum()) == n
    assert (ln[:-1] >= sizes[0]).all() and (ln <= sizes[2]).all()
    assert n // sizes[2] <= len(ln) <= n // sizes[0] + 1
    host = b.cpu().numpy()
    del b
    _assert_same(got, oracle.cdc(algo, host, *sizes), f"config 5 full {algo} {sizes}")
    ch.close()
