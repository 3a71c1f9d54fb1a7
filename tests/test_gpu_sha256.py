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
