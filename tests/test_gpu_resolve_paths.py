"""Resolve-kernel rare paths (-m gpu), forced with the CHUNKFS_AMD_DIAG test
hooks (read once at cdc_create; chunkfs_amd/csrc/fastcdc.hip):

  1 -- walks start at the span start instead of a warm-up point, so nearly
       every span entry is stale: the in-block settle and the look-back's
       stale-entry re-walk (and its wait on the predecessor's final exit) run
       at every block boundary;
  2 -- every wave takes the dense path (exact walks from the bytes and the
       global record lists) instead of the LDS window.

Results must stay bit-exact vs the oracle.
"""
import os

import numpy as np
import pytest

import oracle
from gen_golden import make_input

pytestmark = pytest.mark.gpu


def _chunker(sizes, diag):
    """(The one-launch small-stream kernel is off: these tests drive the
    two-kernel pipeline's resolve, whatever the stream size.)"""
    import chunkfs_amd as c
    old = os.environ.get("CHUNKFS_AMD_DIAG")
    old_small = os.environ.get("CHUNKFS_AMD_SMALL")
    os.environ["CHUNKFS_AMD_DIAG"] = str(diag)
    os.environ["CHUNKFS_AMD_SMALL"] = "0"
    try:
        return c.FastChunker(c.SizeParams(*sizes))
    finally:
        if old_small is None:
            os.environ.pop("CHUNKFS_AMD_SMALL", None)
        else:
            os.environ["CHUNKFS_AMD_SMALL"] = old_small
        if old is None:
            del os.environ["CHUNKFS_AMD_DIAG"]
        else:
            os.environ["CHUNKFS_AMD_DIAG"] = old


def _same(got, ref, what):
    got = np.asarray(got, dtype=np.uint64).reshape(-1, 2)
    ref = np.asarray(ref, dtype=np.uint64).reshape(-1, 2)
    assert got.shape == ref.shape and (got == ref).all(), what


@pytest.mark.parametrize("diag", [1, 2, 3])
@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (512, 2048, 16384), (8192, 16384, 65536)])
def test_forced_paths_single_stream(diag, sizes):
    ch = _chunker(sizes, diag)
    try:
        for n, seed in [(9 << 20, 5), (3 * 65536 + 77, 6), (65536 * 32 + 1, 7)]:
            data = oracle.splitmix64_bytes(n, seed)
            _same(ch.chunk_array(data), oracle.fastcdc(data, *sizes), f"diag={diag} {sizes} n={n}")
        if diag & 1:
            assert ch.last_timing()["fixup_iterations"] > 0  # the re-walk paths really ran
    finally:
        ch.close()


@pytest.mark.parametrize("diag", [1, 2])
def test_forced_paths_batch(diag):
    """Many ragged streams in one batch: stream starts inside blocks and waves,
    low-entropy streams among random ones."""
    import torch
    sizes = (4096, 8192, 16384)
    ch = _chunker(sizes, diag)
    try:
        rng = np.random.default_rng(123 + diag)
        lens = [int(x) for x in rng.integers(0, 1_500_000, size=40)]
        lens[5] = 32 * 65536          # exactly one resolve block
        lens[6] = 32 * 65536 + 1
        lens[7] = 0
        arrays = []
        for i, n in enumerate(lens):
            pat = "const" if i % 9 == 4 else "splitmix64"
            arrays.append(make_input(pat, n, 4000 + i))
        dev = torch.device("cuda", 0)
        bufs = [torch.from_numpy(a).to(dev) if len(a) else torch.empty(16, dtype=torch.uint8, device=dev)
                for a in arrays]
        cap = ch.batch_max_chunks(lens)
        out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=dev)
        first = ch.chunk_batch_device([b.data_ptr() for b in bufs], lens, out.data_ptr(), cap)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint64)
        for i, a in enumerate(arrays):
            _same(got[first[i]:first[i + 1]], oracle.fastcdc(a, *sizes), f"diag={diag} stream {i} len={len(a)}")
    finally:
        ch.close()


def test_non_merging_chains_cascade():
    """All-zero data at max = 20000: chunks are all max cuts from the stream
    start, so no speculative chain merges and every block waits for its
    predecessor's final exit (the look-back's worst case) -- still exact."""
    sizes = (4096, 8192, 20000)
    ch = _chunker(sizes, 0)
    try:
        data = np.zeros(24 << 20, dtype=np.uint8)
        _same(ch.chunk_array(data), oracle.fastcdc(data, *sizes), "zeros max=20000")
    finally:
        ch.close()
