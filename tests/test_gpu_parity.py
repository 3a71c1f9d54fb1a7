"""GPU parity suite (-m gpu): the HIP engine through the C ABI vs the CPU oracle.

Bit-exact (integer / index work): every (offset, length) must equal the
oracle's on the same bytes.  FastCDC parity is vs the oracle restatement
(parity vs the fastcdc 3.1.0 crate is unpinned: GEAR placeholder); FSChunker
and the write path are additionally pinned by the reference's known answers.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from gen_golden import make_input

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SIZES = [(4096, 8192, 16384), (8192, 16384, 65536), (2048, 8192, 65536), (512, 2048, 16384),
         (16384, 65536, 262144), (64, 256, 1024), (8192, 4096, 16384)]

_cache = {}


def chunker(sizes, path="small"):
    """path "small": single streams up to 4 MiB take the one-launch kernel
    (small.hip; the default); "pipeline": CHUNKFS_AMD_SMALL=0, every batch
    takes the scan + resolve pipeline (fastcdc.hip)."""
    import chunkfs_amd as c
    key = (sizes, path)
    if key not in _cache:
        old = os.environ.get("CHUNKFS_AMD_SMALL")
        if path == "pipeline":
            os.environ["CHUNKFS_AMD_SMALL"] = "0"
        try:
            _cache[key] = c.FastChunker(c.SizeParams(*sizes))
        finally:
            if old is None:
                os.environ.pop("CHUNKFS_AMD_SMALL", None)
            else:
                os.environ["CHUNKFS_AMD_SMALL"] = old
    return _cache[key]


PATHS = ["small", "pipeline"]


def assert_same(gpu, ref, what=""):
    gpu = np.asarray(gpu, dtype=np.uint64).reshape(-1, 2)
    ref = np.asarray(ref, dtype=np.uint64).reshape(-1, 2)
    if gpu.shape != ref.shape or not (gpu == ref).all():
        n = min(len(gpu), len(ref))
        bad = np.nonzero((gpu[:n] != ref[:n]).any(axis=1))[0]
        i = int(bad[0]) if len(bad) else n
        pytest.fail(f"{what}: {len(gpu)} vs {len(ref)} chunks; first mismatch at #{i}: "
                    f"gpu={gpu[i].tolist() if i < len(gpu) else None} ref={ref[i].tolist() if i < len(ref) else None}")


@pytest.mark.parametrize("path", PATHS)
def test_golden_vectors_on_gpu(path):
    with open(os.path.join(GOLDEN, "fastcdc_selfconsistent.json")) as f:
        vecs = json.load(f)["vectors"]
    for v in vecs:
        data = make_input(v["pattern"], v["len"], v["seed"])
        assert hashlib.sha256(data.tobytes()).hexdigest() == v["input_sha256"]
        got = chunker((v["min"], v["avg"], v["max"]), path).chunk_array(data)
        assert [int(x) for x in got[:, 1]] == v["lengths"], (v["pattern"], v["len"], v["min"])


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("sizes", SIZES)
@pytest.mark.parametrize("seed", [1, 2])
def test_random_streams_bit_exact(sizes, seed, path):
    for n in [3 * (1 << 20) + 17 * seed, (1 << 20)]:
        data = oracle.splitmix64_bytes(n, seed * 31 + n)
        assert_same(chunker(sizes, path).chunk_array(data), oracle.fastcdc(data, *sizes), f"{sizes} n={n} {path}")


@pytest.mark.parametrize("path", PATHS)
def test_tails_of_every_length(path):
    """Every length 0 .. 2*max+1 around the min/max thresholds (CS-3 edge cases)."""
    sizes = (4096, 8192, 16384)
    base = oracle.splitmix64_bytes(2 * 16384 + 64, 77)
    c = chunker(sizes, path)
    lens = list(range(0, 200)) + list(range(4000, 4200)) + list(range(8100, 8300)) + \
        list(range(16300, 16500)) + list(range(2 * 16384 - 100, 2 * 16384 + 2))
    for n in lens:
        assert_same(c.chunk_array(base[:n]), oracle.fastcdc(base[:n], *sizes), f"n={n}")


@pytest.mark.parametrize("pattern,n,seed", [
    ("const", 5 << 20, 0), ("const", 3 << 20, 0xFF), ("const", 3 << 20, 0x5A),
    ("periodic", 4 << 20, 61), ("periodic", 4 << 20, 4096), ("periodic", 4 << 20, 1),
    ("lowentropy", 4 << 20, 11), ("lowentropy", 4 << 20, 12)])
@pytest.mark.parametrize("path", PATHS)
def test_low_entropy_and_overflow_paths(pattern, n, seed, path):
    """Constant / periodic data: candidate lists are empty or overflow (slow exact path)."""
    data = make_input(pattern, n, seed)
    for sizes in [(4096, 8192, 16384), (512, 2048, 16384)]:
        assert_same(chunker(sizes, path).chunk_array(data), oracle.fastcdc(data, *sizes), f"{pattern} {sizes} {path}")


def test_unaligned_host_buffer():
    data = oracle.splitmix64_bytes((1 << 20) + 100, 5)
    for shift in [1, 3, 7, 13]:
        view = data[shift:]
        assert_same(chunker(SIZES[0]).chunk_array(view), oracle.fastcdc(view, *SIZES[0]), f"shift={shift}")


def test_chunk_data_mirror_and_estimate():
    import chunkfs_amd as c
    ch = chunker(SIZES[0])
    data = oracle.splitmix64_bytes(100_000, 3)
    got = ch.chunk_data(data.tobytes())
    ref = oracle.fastcdc(data, *SIZES[0])
    assert [(x.offset(), x.length()) for x in got] == [tuple(map(int, r)) for r in ref]
    assert ch.estimate_chunk_count(data) == 100_000 // 4096       # fast.rs:47-49
    assert ch.chunk_data(b"") == []
    assert "FastCDC (2020), sizes: SizeParams { min: 4096, avg: 8192, max: 16384 }" in repr(ch)
    fs = c.FSChunker(4096)
    assert fs.estimate_chunk_count(data) == 100_000 // 4096 + 1   # fixed_size.rs:45-47


@pytest.mark.parametrize("cs", [1, 7, 4096, 8192, 65536])
def test_fixed_size_chunker(cs):
    import chunkfs_amd as c
    fs = c.FSChunker(cs)
    for n in [0, 1, cs - 1 if cs > 1 else 2, cs, cs + 1, 3 * (1 << 20) + 50]:
        data = np.zeros(n, dtype=np.uint8)
        assert_same(fs.chunk_array(data), oracle.fixed(n, cs), f"cs={cs} n={n}")


def test_write_path_fixed_known_answers():
    """tests/filesystem.rs:135-166: FSChunker(4096) dedup ratios 256, 512, 384 through the GPU write path."""
    import chunkfs_amd as c
    fs = c.FSChunker(4096)
    db, written, ratios = {}, 0, []
    for val in [10, 10, 20]:
        data = np.full(1 << 20, val, dtype=np.uint8)
        spans, _ = c.write_spans(fs, data)
        off = 0
        for ln in spans:
            db.setdefault(hashlib.sha256(data[off:off + int(ln)].tobytes()).digest(), int(ln))
            off += int(ln)
        assert off == len(data)
        written += len(data)
        ratios.append(written / sum(db.values()))
    assert ratios == pytest.approx([256.0, 512.0, 384.0])


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (8192, 16384, 65536)])
def test_write_path_segmentation_invariance(sizes):
    """spans via the 1 MiB write path == one chunk_data over the whole write == oracle."""
    import chunkfs_amd as c
    data = oracle.splitmix64_bytes(5 * (1 << 20) + 4321, 9)
    spans, secs = c.write_spans(chunker(sizes), data)
    ref_spans, _ = oracle.fs_write("fast", data, *sizes)
    whole = oracle.fastcdc(data, *sizes)[:, 1]
    assert spans.tolist() == ref_spans.tolist() == whole.tolist()
    assert secs > 0


def _torch_batch(ch, arrays):
    import torch
    dev = torch.device("cuda", 0)
    bufs = [torch.from_numpy(a).to(dev) if len(a) else torch.empty(16, dtype=torch.uint8, device=dev)
            for a in arrays]
    lens = [len(a) for a in arrays]
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=dev)
    first = ch.chunk_batch_device([b.data_ptr() for b in bufs], lens, out.data_ptr(), cap)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint64), first


def test_ragged_batch_device():
    sizes = SIZES[0]
    ch = chunker(sizes)
    lens = [0, 1, 4096, 65536, 65537, 3 << 20, 100, 0, (1 << 20) + 12345, 16385, 2 * 65536]
    arrays = [oracle.splitmix64_bytes(n, 1000 + i) for i, n in enumerate(lens)]
    out, first = _torch_batch(ch, arrays)
    assert first[0] == 0
    for i, a in enumerate(arrays):
        assert_same(out[first[i]:first[i + 1]], oracle.fastcdc(a, *sizes), f"stream {i} len={len(a)}")


def test_many_streams_cross_wave_boundaries():
    """150 ragged streams: stream starts fall anywhere inside the walk's
    64-span waves, and the look-back crosses many stream boundaries."""
    sizes = SIZES[0]
    ch = chunker(sizes)
    rng = np.random.default_rng(77)
    lens = [int(x) for x in rng.integers(0, 700_000, size=150)]
    lens[3] = 64 * 65536  # exactly one wave of spans
    lens[4] = 64 * 65536 + 1
    arrays = [oracle.splitmix64_bytes(n, 2000 + i) for i, n in enumerate(lens)]
    out, first = _torch_batch(ch, arrays)
    for i, a in enumerate(arrays):
        assert_same(out[first[i]:first[i + 1]], oracle.fastcdc(a, *sizes), f"stream {i} len={len(a)}")


def test_mixed_entropy_batch():
    """Overflowed record lists (low-entropy streams) next to random ones in the
    same waves: the wave-cooperative fallback runs while other lanes walk."""
    sizes = SIZES[0]
    ch = chunker(sizes)
    arrays = []
    for i in range(12):
        pat = ["splitmix64", "const", "periodic", "lowentropy"][i % 4]
        arrays.append(make_input(pat, 300_000 + 7919 * i, 3000 + i))
    out, first = _torch_batch(ch, arrays)
    for i, a in enumerate(arrays):
        assert_same(out[first[i]:first[i + 1]], oracle.fastcdc(a, *sizes), f"stream {i}")


@pytest.mark.parametrize("lens", [[0, 100000], [0, 0, 3 * 65536 + 999], [0, 65536 + 1, 0, 200000]])
def test_empty_streams_next_to_multispan_low_entropy(lens):
    """Zero-length streams own no span, so they must not hide a multi-span
    stream from the cross-span join (a span count > stream count test would):
    all-zero data at (4096, 8192, 20000) makes every guessed chain wrong."""
    sizes = (4096, 8192, 20000)
    ch = chunker(sizes)
    arrays = [np.zeros(n, dtype=np.uint8) for n in lens]
    out, first = _torch_batch(ch, arrays)
    for i, a in enumerate(arrays):
        assert_same(out[first[i]:first[i + 1]], oracle.fastcdc(a, *sizes), f"stream {i} len={len(a)}")


def test_batch_composition_invariance():
    """Determinism: a stream's chunks do not depend on what else is in the batch."""
    sizes = SIZES[0]
    ch = chunker(sizes)
    a = oracle.splitmix64_bytes(2 << 20, 5)
    alone, f1 = _torch_batch(ch, [a])
    mixed, f2 = _torch_batch(ch, [oracle.splitmix64_bytes(777777, 6), a, oracle.splitmix64_bytes(12345, 7)])
    assert (alone[f1[0]:f1[1]] == mixed[f2[1]:f2[2]]).all()


def test_custom_gear_table():
    sizes = SIZES[0]
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(*sizes))
    gear = oracle.splitmix64_bytes(256 * 8, 12345).view(np.uint64).copy()
    ch.set_gear(gear)
    data = oracle.splitmix64_bytes(2 << 20, 8)
    assert_same(ch.chunk_array(data), oracle.fastcdc(data, *sizes, gear=gear), "custom gear")


def test_device_generator_matches_oracle():
    import ctypes
    import torch
    from chunkfs_amd import _lib
    n = (1 << 20) + 13
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(buf.data_ptr()), n, 1, None))
    assert (buf[:n].cpu().numpy() == oracle.splitmix64_bytes(n, 1)).all()


def test_one_gib_stream_and_timing():
    """Config 2 at full size: 1 GiB splitmix64(seed=1), FastCDC 4/8/16, bit-exact."""
    import ctypes
    import torch
    from chunkfs_amd import _lib
    sizes = SIZES[0]
    ch = chunker(sizes)
    n = 1 << 30
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(buf.data_ptr()), n, 1, None))
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    first = ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
    got = out[:int(first[1])].cpu().numpy().view(np.uint64)
    ref = oracle.fastcdc(buf.cpu().numpy(), *sizes)
    assert_same(got, ref, "1 GiB")
    t = ch.last_timing()
    assert t["bytes"] == n and t["scan_ms"] > 0 and t["overflow_spans"] == 0
    # size-independent properties
    assert int(got[:, 1].sum()) == n
    assert (got[:-1, 1] >= sizes[0]).all() and (got[:, 1] <= sizes[2]).all()
    # the event ring (cdc_debug_timing_back): back-to-back batches, read after
    for _ in range(3):
        ch.chunk_batch_device([buf.data_ptr()], [n], out.data_ptr(), cap)
    hist = [ch.timing_back(k) for k in range(4)]
    assert all(h["scan_ms"] > 0 and h["total_ms"] >= h["scan_ms"] for h in hist)
    assert hist[0]["scan_ms"] == ch.last_timing()["scan_ms"]
    from chunkfs_amd import CdcError
    with pytest.raises(CdcError):
        ch.timing_back(64)


def test_config4_batch_1024_streams_of_64mib():
    """BASELINE config 4 on one GPU: 1024 independent 64 MiB streams (64 GiB in
    HBM), stream i = splitmix64(seed=1000+i), FastCDC 4/8/16 KiB.  A seeded
    sample of 16 streams is compared bit-exact with the oracle; on all 1024 the
    size-independent invariants hold: exact tiling from 0, min <= len <= max
    except each stream's last chunk, first[] monotone with first[0] == 0."""
    import ctypes
    import torch
    from chunkfs_amd import _lib
    sizes = SIZES[0]
    ch = chunker(sizes)
    n_streams, slen = 1024, 64 << 20
    buf = torch.empty(n_streams * slen, dtype=torch.uint8, device="cuda")
    L = _lib.lib()
    for i in range(n_streams):
        _lib.check(L.cdc_fill_splitmix64_device(ctypes.c_void_p(buf.data_ptr() + i * slen), slen, 1000 + i, None))
    ptrs = [buf.data_ptr() + i * slen for i in range(n_streams)]
    lens = [slen] * n_streams
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda")
    first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
    torch.cuda.synchronize()
    first = np.asarray(first, dtype=np.int64)
    assert first[0] == 0 and (np.diff(first) > 0).all()
    got = out[:int(first[-1])].cpu().numpy().view(np.uint64)
    off, ln = got[:, 0].astype(np.int64), got[:, 1].astype(np.int64)
    for i in range(n_streams):
        o, l_ = off[first[i]:first[i + 1]], ln[first[i]:first[i + 1]]
        assert o[0] == 0 and (o[1:] == np.cumsum(l_)[:-1]).all() and int(l_.sum()) == slen, i
        assert (l_[:-1] >= sizes[0]).all() and (l_ <= sizes[2]).all(), i
    rng = np.random.default_rng(4)
    for i in sorted(rng.choice(n_streams, size=16, replace=False).tolist()):
        host = buf[i * slen:(i + 1) * slen].cpu().numpy()
        assert_same(got[first[i]:first[i + 1]], oracle.fastcdc(host, *sizes), f"config4 stream {i}")
    del buf, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (512, 2048, 16384), (16384, 65536, 262144)])
def test_dma_scan_variant_bit_exact(sizes, monkeypatch):
    """The LDS-DMA scan (A/B path, CHUNKFS_AMD_DIAG bit 10, read at cdc_create):
    ragged multi-stream batch incl. low-entropy data and a multi-span stream."""
    import chunkfs_amd as c
    monkeypatch.setenv("CHUNKFS_AMD_DIAG", "1024")
    monkeypatch.setenv("CHUNKFS_AMD_SMALL", "0")  # (single streams <= 4 MiB would take small.hip)
    ch = c.FastChunker(c.SizeParams(*sizes))
    streams = [oracle.splitmix64_bytes(n, 97 + n) for n in (5 * (1 << 20) + 3, 1 << 16, 777, 2 * (1 << 20))]
    streams.append(np.zeros(3 * (1 << 20) + 11, dtype=np.uint8))
    streams.append(np.tile(oracle.splitmix64_bytes(61, 5), 40000)[: 2 * (1 << 20) + 5])
    for data in streams:
        assert_same(ch.chunk_array(data), oracle.fastcdc(data, *sizes), f"dma {sizes} n={len(data)}")


@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (8192, 16384, 32768)])
def test_large_streams_max_cut_runs(sizes):
    """Streams past the 8 MiB small-batch line take the big-span pipeline
    (128 KiB spans at these sizes): zero runs of every length -- shorter than
    one max chunk, a few max chunks, longer than a span and than a walk
    window -- between random stretches, a constant run of another byte and a
    61-byte period.  The resolve's exact steps then run as wave-cooperative
    max-cut runs (walk_window, CDC_WALK_COOP) that must stop exactly where a
    record or a truncated-region hit takes over.  Synchronous and async."""
    import torch
    import chunkfs_amd as c
    rng = np.random.default_rng(4242)
    parts = []
    for k, run in enumerate([100, 5000, 16384, 40000, 131072, 300000, 1 << 20, 3 << 20, 7777, 262144 + 13]):
        parts.append(oracle.splitmix64_bytes(int(rng.integers(1000, 200000)), 500 + k))
        parts.append(np.zeros(run, dtype=np.uint8) if k % 3 else np.full(run, 0xA5, dtype=np.uint8))
    parts.append(np.tile(oracle.splitmix64_bytes(61, 7), 40000))
    parts.append(oracle.splitmix64_bytes(3 << 20, 77))
    data = np.concatenate(parts)
    assert len(data) > 8 << 20
    ch = c.FastChunker(c.SizeParams(*sizes))
    ref = oracle.fastcdc(data, *sizes)
    out, first = _torch_batch(ch, [data])
    assert_same(out[first[0]:first[1]], ref, f"sync {sizes}")
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(data).to(dev)
    cap = ch.batch_max_chunks([len(data)])
    outs = [torch.empty((cap, 2), dtype=torch.int64, device=dev) for _ in range(3)]
    firsts = [ch.chunk_batch_device_async([buf.data_ptr()], [len(data)], o.data_ptr(), cap) for o in outs]
    assert ch.batch_sync() == len(ref)
    torch.cuda.synchronize()
    for o, f in zip(outs, firsts):
        assert_same(o.cpu().numpy().view(np.uint64)[int(f[0]):int(f[1])], ref, f"async {sizes}")
