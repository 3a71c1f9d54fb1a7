"""The host-memory boundary on the GPU (-m gpu): cdc_chunk_data through the
pinned upload ring with the chunk list written into host-mapped memory, and the
streaming write path (cdc_write_begin / _segment / _finish) against the
reference's StorageWriter semantics (storage.rs:105-137, 302-383) restated by
the oracle: for every chunker here the spans of the per-segment loop equal
the chunks of the whole write, for any segment sizes."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
SIZES = {"fast": (4096, 8192, 16384), "rabin": (2048, 4096, 8192), "ultra": (4096, 8192, 16384),
         "leap": (4096, 8192, 16384), "seq": (4096, 8192, 16384), "fixed": (4096, 0, 0)}


def _chunker(algo):
    import chunkfs_amd as c
    s = SIZES[algo]
    if algo == "fixed":
        return c.FSChunker(s[0])
    if algo == "seq":
        return c.SeqChunker(c.OperationMode.Increasing, c.SizeParams(*s))
    cls = {"fast": c.FastChunker, "rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}[algo]
    return cls(c.SizeParams(*s))


def _whole(algo, data):
    s = SIZES[algo]
    if algo == "fast":
        return oracle.fastcdc(data, *s)[:, 1]
    if algo == "fixed":
        n, cs = data.size, s[0]
        return np.array([min(cs, n - o) for o in range(0, n, cs)], dtype=np.uint64)
    return oracle.cdc(algo, data, *s)[:, 1]


def _segments(n, rng):
    """Segment sizes of a write_from_stream: 1 MiB reads with short reads,
    empty reads and a few large ones."""
    out, left = [], n
    while left:
        r = rng.random()
        k = 1 << 20 if r < 0.6 else int(rng.integers(0, 5000)) if r < 0.8 else int(rng.integers(1, 9 << 20))
        k = min(k, left)
        out.append(k)
        left -= k
    return out


@pytest.mark.parametrize("algo", ["fast", "rabin", "ultra", "leap", "seq", "fixed"])
def test_stream_write_matches_storage_writer(algo):
    import chunkfs_amd as c
    rng = np.random.default_rng(hash(algo) & 0xFFFF)
    data = oracle.splitmix64_bytes((40 << 20) + 12345, 77)
    ch = _chunker(algo)
    w = c.StreamWriter(ch)
    off = 0
    for k in _segments(data.size, rng):
        w.write(data[off:off + k])
        off += k
    spans, secs = w.finish()
    assert secs > 0
    ref = _whole(algo, data)
    assert spans.shape == ref.shape and (spans == ref).all(), algo
    assert int(spans.sum()) == data.size
    if algo != "fixed":  # the oracle's own 1 MiB StorageWriter loop agrees too
        ref_fs, _ = oracle.fs_write(algo, data, *SIZES[algo])
        assert [int(x) for x in spans] == [int(x) for x in ref_fs]
    ch.close()


def test_stream_write_crosses_device_windows():
    """600 MiB in 1 MiB segments: the 256 MiB device windows and the carried
    chunk between them (the reference's `rest`, in HBM here).  Spans are
    drained as windows complete (cdc_write_drain): drains + finish == the
    whole write, and the first drain comes after the first window."""
    import chunkfs_amd as c
    data = oracle.splitmix64_bytes(600 << 20, 5)
    ch = _chunker("fast")
    w = c.StreamWriter(ch)
    drained, first_at, covered = [], None, 0
    for off in range(0, data.size, 1 << 20):
        w.write(data[off:off + (1 << 20)])
        d = w.drain()
        if d.size and first_at is None:
            first_at = off + (1 << 20)
        covered += int(d.sum())
        assert covered <= off + (1 << 20)  # a drained span lies in uploaded bytes
        drained.append(d)
    spans, _ = w.finish()
    spans = np.concatenate(drained + [spans])
    assert first_at is not None and first_at > (256 << 20)
    ref = _whole("fast", data)
    assert spans.shape == ref.shape and (spans == ref).all()
    st = c.host_stats(ch)
    assert st["write_segments"] == 600 and st["write_chunk_s"] > 0
    # the same handle serves a second write (fresh StorageWriter, storage.rs:79)
    spans2, _ = c.write_spans(ch, data[:3 << 20])
    ref2 = _whole("fast", data[:3 << 20])
    assert spans2.shape == ref2.shape and (spans2 == ref2).all()
    ch.close()


@pytest.mark.parametrize("algo", ["ultra", "seq"])
def test_stream_write_window_carry_walk_rules(algo):
    """The walk engine across the 256 MiB device windows (a lane-walk and a
    wave-walk rule): just over two windows of random bytes with a zero-filled
    region straddling the first window boundary, so a window starts inside a
    quiet run at a carried chunk."""
    import chunkfs_amd as c
    n = (512 << 20) + 77777
    data = oracle.splitmix64_bytes(n, 31)
    b = 256 << 20
    data[b - (3 << 20) + 11:b + (2 << 20) + 5] = 0
    ch = _chunker(algo)
    w = c.StreamWriter(ch)
    drained = []
    for off in range(0, n, 1 << 20):
        w.write(data[off:off + (1 << 20)])
        drained.append(w.drain())
    spans, _ = w.finish()
    spans = np.concatenate(drained + [spans])
    ref = _whole(algo, data)
    assert spans.shape == ref.shape and (spans == ref).all(), algo
    ch.close()


def test_stream_write_begin_twice_and_failure_rules():
    """cdc_write_begin on a write in progress is refused (the write in
    progress is kept); finish ends it; a drain without a write is refused."""
    import chunkfs_amd as c
    ch = _chunker("fast")
    data = oracle.splitmix64_bytes(3 << 20, 8)
    w = c.StreamWriter(ch)
    w.write(data[:1 << 20])
    with pytest.raises(c.CdcError):
        c.StreamWriter(ch)
    with pytest.raises(c.CdcError):
        c.write_spans(ch, data)  # cdc_fs_write also begins a write
    with pytest.raises(c.CdcError):
        ch.set_gear(np.arange(256, dtype=np.uint64))  # no table swap inside a write
    w.write(data[1 << 20:])
    spans, _ = w.finish()
    ref = _whole("fast", data)
    assert spans.shape == ref.shape and (spans == ref).all()
    with pytest.raises(c.CdcError):
        w.drain()
    spans2, _ = c.write_spans(ch, data)  # the handle is free again
    assert (spans2 == ref).all()
    ch.close()
    # a Rabin handle refuses a new polynomial while its write is open
    rb = _chunker("rabin")
    w = c.StreamWriter(rb)
    w.write(data[:1 << 20])
    with pytest.raises(c.CdcError):
        rb.set_poly(0x3DA3358B4DC173)
    w.write(data[1 << 20:])
    spans, _ = w.finish()
    ref = _whole("rabin", data)
    assert spans.shape == ref.shape and (spans == ref).all()
    rb.set_poly(0x3DA3358B4DC173)  # free again
    rb.close()


def test_stream_write_edge_cases():
    import chunkfs_amd as c
    ch = _chunker("fast")
    w = c.StreamWriter(ch)  # empty write: no span (storage.rs:318-320, 364-366)
    spans, _ = w.finish()
    assert spans.size == 0
    w = c.StreamWriter(ch)
    for part in (b"", b"abc", b"", b"defgh"):
        w.write(part)
    spans, _ = w.finish()
    assert [int(x) for x in spans] == [8]
    with pytest.raises(c.CdcError):
        w.finish()  # no write in progress
    ch.close()


@pytest.mark.parametrize("algo", ["fast", "rabin", "ultra", "leap", "seq", "fixed"])
def test_chunk_data_pinned_path(algo):
    """cdc_chunk_data over host buffers of every size class (pieces of the
    pinned ring, the host-mapped chunk list), unaligned views included."""
    ch = _chunker(algo)
    base = oracle.splitmix64_bytes((20 << 20) + 64, 11)
    for n, off in [(1, 0), (4097, 3), ((1 << 20) + 5, 1), ((8 << 20) + 1, 7), ((20 << 20) + 3, 13)]:
        data = base[off:off + n]
        got = ch.chunk_array(data)
        ref = _whole(algo, np.ascontiguousarray(data))
        assert got.shape[0] == ref.size and (got[:, 1] == ref).all(), (algo, n)
        assert int(got[0, 0]) == 0 and (got[1:, 0] == np.cumsum(got[:-1, 1])).all()
    ch.close()


def test_reference_1MiB_loop_through_chunk_data():
    """The Rust shim's loop (StorageWriter::write per 1 MiB: buffer = rest ++
    segment, chunk_data, rest = last chunk; flush) through cdc_chunk_data."""
    data = oracle.splitmix64_bytes((24 << 20) + 999, 123)
    ch = _chunker("fast")
    spans, rest = [], np.empty(0, dtype=np.uint8)
    for off in range(0, data.size, 1 << 20):
        buf = np.concatenate([rest, data[off:off + (1 << 20)]])
        chunks = ch.chunk_array(buf)
        spans += [int(x) for x in chunks[:-1, 1]]
        o, ln = (int(x) for x in chunks[-1])
        rest = buf[o:o + ln]
    spans.append(rest.size)
    ref, _ = oracle.fs_write("fast", data, *SIZES["fast"])
    assert spans == [int(x) for x in ref]
    ch.close()


def test_host_placement_reported_and_followed():
    """cdc_debug_host_placement: the device's PCI address, node and link; with
    NUMA placement on, the pinned ring and chunk list sit on the GPU's node."""
    import chunkfs_amd as c
    ch = _chunker("fast")
    p = c.host_placement(ch)
    assert p["pci"] and p["copy_threads"] >= 1 and p["allowed_cpus"] >= 1
    if p["numa_placement"]:
        assert p["gpu_node"] >= 0 and p["node_cpus_allowed"] >= 1
        assert p["ring_node"] in (p["gpu_node"], -1)  # (-1: the kernel would not say)
        assert p["helpers_pinned"] == p["copy_threads"] - 1 or p["helpers_pinned"] == 0  # (the node's pool may predate)
    data = oracle.splitmix64_bytes((1 << 20) + 77, 5)
    assert (ch.chunk_array(data)[:, 1] == _whole("fast", data)).all()
    ch.close()


def test_chunk_data_two_handles_two_threads():
    """Handles on one node share that node's copy pool, one job at a time:
    two threads calling chunk_data on two handles get bit-exact chunks; the
    small path handles the calls (a wait that outlasts the kernel's feed poll
    becomes a fallback to the regular pipeline, still exact: counted, not
    required to be 0)."""
    import threading
    import chunkfs_amd as c
    chs = [_chunker("fast"), _chunker("fast")]
    datas = [oracle.splitmix64_bytes((1 << 20) + 4099 * i, 40 + i) for i in range(8)]
    refs = [_whole("fast", d) for d in datas]
    errs = []
    before = [c.host_stats(h) for h in chs]

    def run(k):
        try:
            for rep in range(20):
                i = (rep * 2 + k) % len(datas)
                got = chs[k].chunk_array(datas[i])[:, 1]
                if not (got.shape == refs[i].shape and (got == refs[i]).all()):
                    errs.append((k, rep))
        except Exception as e:  # noqa: BLE001
            errs.append((k, repr(e)))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    after = [c.host_stats(h) for h in chs]
    small = sum(a["small_calls"] - b["small_calls"] for a, b in zip(after, before))
    fb = sum(a["small_fallbacks"] - b["small_fallbacks"] for a, b in zip(after, before))
    assert small == 40 and fb <= small
    for h in chs:
        h.close()


def test_host_placement_off_is_exact(monkeypatch):
    """CHUNKFS_AMD_COPY_NUMA=0 (the A/B path): no placement, unpinned helpers
    (their own pool), same chunks."""
    import chunkfs_amd as c
    monkeypatch.setenv("CHUNKFS_AMD_COPY_NUMA", "0")
    ch = _chunker("fast")
    p = c.host_placement(ch)
    assert p["numa_placement"] is False and p["helpers_pinned"] == 0
    for n in ((1 << 20) + 5, (6 << 20) + 77, 40 << 20):  # small kernel, ring upload, pageable copy
        data = oracle.splitmix64_bytes(n, 90 + n % 7)
        assert (ch.chunk_array(data)[:, 1] == _whole("fast", data)).all(), n
    ch.close()
