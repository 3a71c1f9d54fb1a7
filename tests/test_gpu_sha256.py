"""SHA-256 chunk fingerprints on the GPU.

Oracle: Python's hashlib (FIPS 180-4), the same function as the reference's
Sha256Hasher (src/hashers.rs:20-36, sha2 crate).  Chunks come from the GPU
chunker and are checked against the CPU oracle first, so a digest mismatch is
a hashing fault.
"""
import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _digests(data, chunks):
    b = bytes(np.asarray(data, dtype=np.uint8))
    return np.array([list(hashlib.sha256(b[int(o):int(o) + int(l)]).digest()) for o, l in chunks],
                    dtype=np.uint8).reshape(-1, 32)


@pytest.mark.parametrize("sizes,n,seed", [
    ((4096, 8192, 16384), 4 << 20, 1),
    ((64, 256, 1024), 300_001, 2),           # tiny chunks: many tail blocks, odd offsets
    ((1000, 3000, 9000), (1 << 20) + 3, 3),  # unaligned chunk starts everywhere
])
def test_chunk_and_hash_matches_hashlib(sizes, n, seed):
    import chunkfs_amd as c
    data = oracle.splitmix64_bytes(n, seed)
    ch = c.FastChunker(c.SizeParams(*sizes))
    chunks, dig = ch.chunk_and_hash(data)
    assert (chunks == oracle.fastcdc(data, *sizes)).all()
    assert (dig == _digests(data, chunks)).all()
    assert ch.last_timing()["hash_ms"] > 0


def test_sha256_padding_lengths():
    """Every length class of the padding: 0..130 bytes and around block multiples."""
    import torch
    import chunkfs_amd as c
    lens = list(range(0, 131)) + [183, 184, 191, 192, 247, 248, 255, 256, 4095, 4096, 4097, 16384]
    offs = np.cumsum([0] + lens[:-1]) + 3  # odd offsets: unaligned starts
    total = int(offs[-1] + lens[-1] + 16)
    data = oracle.splitmix64_bytes(total, 11)
    chunks = np.stack([offs, lens], axis=1).astype(np.uint64)
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    d = torch.from_numpy(data).cuda()
    dc = torch.from_numpy(chunks.view(np.int64)).cuda()
    out = torch.empty((len(lens), 32), dtype=torch.uint8, device="cuda")
    ch.sha256_chunks_device(d.data_ptr(), dc.data_ptr(), len(lens), out.data_ptr())
    assert (out.cpu().numpy() == _digests(data, chunks)).all()


def test_fixed_chunker_hash_dedup_known_answer():
    """Config 1 shape (FSChunker 8 KiB): identical chunks hash identically --
    a 64 MiB buffer of 16 repeated 4 MiB blocks has 512 unique digests."""
    import chunkfs_amd as c
    block = oracle.splitmix64_bytes(4 << 20, 5)
    data = np.tile(block, 16)
    ch = c.FSChunker(8192)
    chunks, dig = ch.chunk_and_hash(data)
    assert chunks.shape[0] == 8192
    uniq = {bytes(r) for r in dig}
    assert len(uniq) == 512
    assert bytes(dig[0]) == hashlib.sha256(bytes(block[:8192])).digest()


def test_config1_fixed_8k_64mib_sha256():
    """BASELINE config 1: FSChunker 8 KiB over a 64 MiB splitmix64(seed=0x0C0FFEE1)
    buffer, every chunk fingerprinted (StorageWriter's Sha256Hasher) and put in a
    HashMap-style unique set: 8192 chunks, average 8192 B, dedup ratio 1.0
    (SURVEY.md §8d).  All 8192 digests are checked against hashlib."""
    import chunkfs_amd as c
    n = 64 << 20
    data = oracle.splitmix64_bytes(n, 0x0C0FFEE1)
    ch = c.FSChunker(8192)
    chunks, dig = ch.chunk_and_hash(data)
    assert (chunks == oracle.fixed(n, 8192)).all()
    assert chunks.shape[0] == 8192
    assert (dig == _digests(data, chunks)).all()
    unique = {}
    for (o, ln), d in zip(chunks, dig):
        unique.setdefault(bytes(d), int(ln))  # database.rs:74-77: first insert wins
    assert n / sum(unique.values()) == 1.0
    assert sum(unique.values()) / len(unique) == 8192.0


def _batch_check(ch, bufs, lens, first, out, torch):
    n = int(first[-1])
    dig = torch.empty((max(n, 1), 32), dtype=torch.uint8, device="cuda")
    ch.sha256_batch_device([b.data_ptr() for b in bufs], first, out.data_ptr(), dig.data_ptr())
    got = dig[:n].cpu().numpy()
    allc = out[:n].cpu().numpy().view(np.uint64)
    for i, (b, ln) in enumerate(zip(bufs, lens)):
        a, z = int(first[i]), int(first[i + 1])
        assert (got[a:z] == _digests(b[:ln].cpu().numpy(), allc[a:z])).all(), f"stream {i}"


def test_sha256_batch_multi_stream_rabin():
    """cdc_sha256_batch_device over a multi-stream Rabin batch (config 3's
    shape): one launch, per-stream bases, empty and tiny streams included."""
    import torch
    import chunkfs_amd as c
    sizes = (2048, 4096, 8192)
    lens = [(6 << 20) + 5, 0, 1, 67, 4097, (3 << 20) + 1, 130]
    bufs = [torch.from_numpy(oracle.splitmix64_bytes(max(n, 1), 40 + i)).cuda() for i, n in enumerate(lens)]
    ch = c.RabinChunker(c.SizeParams(*sizes))
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    first = ch.chunk_batch_device([b.data_ptr() for b in bufs], lens, out.data_ptr(), cap)
    _batch_check(ch, bufs, lens, first, out, torch)
    assert ch.last_timing()["hash_ms"] > 0


def test_sha256_batch_contiguous_short_neighbours():
    """Contiguous chunks whose successors are shorter / longer than the
    68-byte over-read window, ending exactly at the end of the data, at odd
    offsets: every load-path choice of the kernel."""
    import torch
    import chunkfs_amd as c
    pat = [70, 67, 68, 69, 1, 0, 200, 3, 64, 55, 56, 119, 120, 4096, 66, 5000, 2, 1000]
    bufs, lens_b, chunk_lists = [], [], []
    for k, skew in enumerate((0, 1, 2, 3)):
        lens_c = pat[k:] + pat[:k]
        total = skew + sum(lens_c)
        bufs.append(torch.from_numpy(oracle.splitmix64_bytes(total, 90 + k)).cuda())
        lens_b.append(total)
        offs = np.cumsum([skew] + lens_c[:-1])
        chunk_lists.append(np.stack([offs, lens_c], axis=1).astype(np.uint64))
    first = np.cumsum([0] + [len(cl) for cl in chunk_lists]).astype(np.uint64)
    out = torch.from_numpy(np.concatenate(chunk_lists).view(np.int64)).cuda()
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    _batch_check(ch, bufs, lens_b, first, out, torch)


def test_sha256_batch_rejects_bad_tables():
    import torch
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    b = torch.zeros(64, dtype=torch.uint8, device="cuda")
    out = torch.zeros((2, 2), dtype=torch.int64, device="cuda")
    dig = torch.empty((2, 32), dtype=torch.uint8, device="cuda")
    with pytest.raises(c.CdcError):
        ch.sha256_batch_device([b.data_ptr()], [1, 2], out.data_ptr(), dig.data_ptr())  # first[0] != 0
    with pytest.raises(c.CdcError):
        ch.sha256_batch_device([b.data_ptr(), b.data_ptr()], [0, 2, 1], out.data_ptr(), dig.data_ptr())
