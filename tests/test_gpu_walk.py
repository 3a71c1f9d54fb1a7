"""GPU parity of the segment-walk engine (-m gpu): Rabin / UltraCDC / LeapCDC /
SeqCDC through the C ABI vs the CPU oracle, bit-exact.

Parity is vs the oracle's restatement of the published algorithms (the
reference's crate, cdc-chunkers 0.1.3, is absent offline: parity vs the crate
is UNPINNED, see oracle/cdc_oracle.c and DESIGN.md).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from gen_golden import make_input

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "cdc_walk_selfconsistent.json")
ALGOS = ["rabin", "ultra", "leap", "seq"]
SIZES = {
    "rabin": [(2048, 4096, 8192), (4096, 8192, 16384), (64, 256, 1024), (16384, 65536, 524288)],
    "ultra": [(4096, 8192, 16384), (1024, 2048, 8192), (8, 64, 256), (16384, 65536, 524288)],
    "leap": [(4096, 8192, 16384), (256, 1024, 4096), (32, 64, 128), (16384, 65536, 524288)],
    "seq": [(4096, 8192, 16384), (64, 256, 1024), (1, 2, 3), (16384, 65536, 524288)],
}
_cache = {}


def chunker(algo, sizes):
    import chunkfs_amd as c
    key = (algo, sizes)
    if key not in _cache:
        cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(algo)
        if cls is None:
            _cache[key] = c.SeqChunker(c.OperationMode.Increasing, c.SizeParams(*sizes))
        else:
            _cache[key] = cls(c.SizeParams(*sizes))
    return _cache[key]


def assert_same(gpu, ref, what=""):
    gpu = np.asarray(gpu, dtype=np.uint64).reshape(-1, 2)
    ref = np.asarray(ref, dtype=np.uint64).reshape(-1, 2)
    if gpu.shape != ref.shape or not (gpu == ref).all():
        n = min(len(gpu), len(ref))
        bad = np.nonzero((gpu[:n] != ref[:n]).any(axis=1))[0]
        i = int(bad[0]) if len(bad) else n
        pytest.fail(f"{what}: {len(gpu)} vs {len(ref)} chunks; first mismatch at #{i}: "
                    f"gpu={gpu[i].tolist() if i < len(gpu) else None} ref={ref[i].tolist() if i < len(ref) else None}")


def test_walk_golden_vectors_on_gpu():
    with open(GOLDEN) as f:
        vecs = json.load(f)["vectors"]
    for v in vecs:
        data = make_input(v["pattern"], v["len"], v["seed"])
        assert hashlib.sha256(data.tobytes()).hexdigest() == v["input_sha256"]
        got = chunker(v["algo"], (v["min"], v["avg"], v["max"])).chunk_array(data)
        assert [int(x) for x in got[:, 1]] == v["lengths"], (v["algo"], v["pattern"], v["len"])


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("si", range(4))
def test_random_streams_bit_exact(algo, si):
    sizes = SIZES[algo][si]
    for n in [(3 << 20) + 17 * si, 1 << 20, 100003]:
        data = oracle.splitmix64_bytes(n, n + 7 * si + 1)
        assert_same(chunker(algo, sizes).chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} {sizes} n={n}")


@pytest.mark.parametrize("algo", ALGOS)
def test_tail_lengths(algo):
    sizes = SIZES[algo][1]
    base = oracle.splitmix64_bytes(sizes[2] * 3 + 400, 99)
    for n in list(range(0, 70)) + list(range(sizes[0] - 3, sizes[0] + 3)) + [sizes[2] * 3 + k for k in range(0, 400, 37)]:
        data = base[:n]
        assert_same(chunker(algo, sizes).chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} n={n}")


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("pattern,seed", [("const", 0), ("const", 0xAA), ("periodic", 61), ("periodic", 4096),
                                          ("lowentropy", 3)])
def test_low_entropy_exact(algo, pattern, seed):
    """Chains that never merge (periodic cuts) go through the fix-up rounds and
    the serial pass; the result must still be exact."""
    sizes = SIZES[algo][1]
    data = make_input(pattern, 600000, seed)
    assert_same(chunker(algo, sizes).chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} {pattern}")


@pytest.mark.parametrize("algo", ALGOS)
def test_ragged_device_batch(algo):
    """cdc_chunk_batch_device over streams of mixed lengths (empty ones too)."""
    import torch
    sizes = SIZES[algo][0]
    lens = [0, 5, 1 << 20, 0, 12345, 3 * sizes[2] + 1, (2 << 20) + 77, 0, sizes[0], 700001]
    bufs, host = [], []
    for i, n in enumerate(lens):
        h = oracle.splitmix64_bytes(n, 500 + i)
        host.append(h)
        bufs.append(torch.from_numpy(h.copy()).to("cuda:0") if n else torch.empty(16, dtype=torch.uint8, device="cuda:0"))
    ch = chunker(algo, sizes)
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    first = ch.chunk_batch_device([b.data_ptr() for b in bufs], lens, out.data_ptr(), cap)
    got = out.cpu().numpy().astype(np.uint64)
    for i, h in enumerate(host):
        assert_same(got[first[i]:first[i + 1]], oracle.cdc(algo, h, *sizes), f"{algo} stream {i} (len {lens[i]})")


@pytest.mark.parametrize("algo", ALGOS)
def test_write_path_matches_oracle(algo):
    import chunkfs_amd as c
    sizes = SIZES[algo][0]
    data = oracle.splitmix64_bytes((3 << 20) + 999, 4242)
    spans, _ = c.write_spans(chunker(algo, sizes), data)
    ref, _ = oracle.fs_write(algo, data, *sizes)
    assert [int(x) for x in spans] == [int(x) for x in ref]


def test_seq_decreasing_and_custom_config():
    import chunkfs_amd as c
    data = oracle.splitmix64_bytes((1 << 20) + 3, 31337)
    for mode, cfg in [(c.OperationMode.Decreasing, c.SeqConfig()), (c.OperationMode.Increasing, c.SeqConfig(3, 10, 64)),
                      (c.OperationMode.Decreasing, c.SeqConfig(7, 200, 1000))]:
        ch = c.SeqChunker(mode, c.SizeParams(700, 1500, 6000), cfg)
        ref = oracle.cdc("seq", data, 700, 1500, 6000,
                         seqcfg=(mode, cfg.seq_length, cfg.jump_trigger, cfg.jump_size))
        assert_same(ch.chunk_array(data), ref, f"seq mode={mode} {cfg}")
        assert "mode: " + ("Decreasing" if mode else "Increasing") in repr(ch)


def test_estimates_and_debug_strings():
    import chunkfs_amd as c
    s = c.SizeParams(4096, 8192, 16384)
    n = 10 ** 7
    assert c.RabinChunker(s).estimate_chunk_count(n) == n // 4096   # rabin.rs:53-55
    assert c.UltraChunker(s).estimate_chunk_count(n) == n // 4096   # ultra.rs:41-43
    assert c.LeapChunker(s).estimate_chunk_count(n) == n // 4096    # leap.rs:41-43
    assert c.SeqChunker(0, s).estimate_chunk_count(n) == n // 8192  # seq.rs:52-54
    assert repr(c.RabinChunker(s)).startswith("RabinCDC, sizes: SizeParams { min: 4096, avg: 8192, max: 16384 }")
    assert repr(c.UltraChunker(s)).startswith("UltraCDC, sizes: ")
    assert repr(c.LeapChunker(s)).startswith("LeapCDC, sizes: ")


@pytest.mark.parametrize("algo", ALGOS)
def test_large_stream_device_resident(algo):
    """64 MiB device-resident stream (the config-5 shape at reduced size):
    bit-exact against the oracle, plus the timing fields."""
    import torch
    import chunkfs_amd as c
    from chunkfs_amd import _lib
    sizes = SIZES[algo][0]
    n = 64 << 20
    b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 5, None))
    ch = chunker(algo, sizes)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    first = ch.chunk_batch_device([b.data_ptr()], [n], out.data_ptr(), cap)
    got = out[:first[1]].cpu().numpy().astype(np.uint64)
    ref = oracle.cdc(algo, b.cpu().numpy(), *sizes)
    assert_same(got, ref, f"{algo} 64 MiB")
    t = ch.last_timing()
    assert t["bytes"] == n and t["total_ms"] > 0


@pytest.mark.parametrize("algo", ["rabin", "ultra", "leap", "seq"])
def test_byte_mode_equals_oracle(algo, monkeypatch):
    """The byte-serial walks (used for Rabin with min < 48, and forced here with
    CHUNKFS_AMD_WALK_BYTES=1, read at handle creation) stay exact: the bitmap
    mode is the default for these rules."""
    import chunkfs_amd as c
    monkeypatch.setenv("CHUNKFS_AMD_WALK_BYTES", "1")
    sizes = SIZES[algo][0]
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(algo)
    ch = cls(c.SizeParams(*sizes)) if cls else c.SeqChunker(0, c.SizeParams(*sizes))
    for n, seed in [((1 << 20) + 5, 8), (300001, 9)]:
        data = oracle.splitmix64_bytes(n, seed)
        assert_same(ch.chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} byte mode n={n}")
    data = make_input("lowentropy", 300000, 5)
    assert_same(ch.chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} byte mode low entropy")
    ch.close()


@pytest.mark.parametrize("sizes", [(16, 64, 256), (40, 100, 400), (47, 2048, 8192), (48, 2048, 8192)])
def test_rabin_small_min_byte_path(sizes):
    """Rabin with min < 48 (partial windows at the chunk start) takes the byte
    walks; min = 48 is the first bitmap-mode size."""
    data = oracle.splitmix64_bytes(400003, sizes[0])
    assert_same(chunker("rabin", sizes).chunk_array(data), oracle.cdc("rabin", data, *sizes), f"rabin {sizes}")


def test_seq_bitmap_long_runs_and_configs():
    """SeqCDC's word-at-a-time walk: runs and opposing counts carried across
    64-bit steps (ramps, short periods), long seq_length, jump_trigger 1."""
    import chunkfs_amd as c
    ramp = (np.arange(700000) % 256).astype(np.uint8)          # long increasing runs
    saw = (np.arange(700000) % 7).astype(np.uint8)            # runs of 6, then a drop
    rnd = oracle.splitmix64_bytes(700001, 77)
    for data in (ramp, saw, rnd):
        for mode, cfg in [(0, c.SeqConfig(5, 50, 256)), (1, c.SeqConfig(5, 50, 256)), (0, c.SeqConfig(63, 1, 3)),
                          (0, c.SeqConfig(6, 100, 1)), (1, c.SeqConfig(2, 64, 65)), (0, c.SeqConfig(64, 5, 10))]:
            ch = c.SeqChunker(mode, c.SizeParams(300, 1000, 5000), cfg)
            ref = oracle.cdc("seq", data, 300, 1000, 5000, seqcfg=(mode, cfg.seq_length, cfg.jump_trigger, cfg.jump_size))
            assert_same(ch.chunk_array(data), ref, f"seq mode={mode} {cfg}")
            ch.close()


@pytest.mark.parametrize("algo", ALGOS)
def test_many_small_streams_batch(algo):
    """2000 streams of 0..40000 bytes in one device batch: per-stream segment
    tables, bitmap offsets and stream-end handling in every kernel."""
    import torch
    sizes = SIZES[algo][1]
    rng = np.random.default_rng(11)
    lens = [int(x) for x in rng.integers(0, 40000, 2000)]
    lens[::97] = [0] * len(lens[::97])
    host = oracle.splitmix64_bytes(sum(lens) + 16, 2024)
    offs = np.concatenate([[0], np.cumsum(lens)])
    # one device buffer, each stream 16-byte aligned inside it
    starts, pos = [], 0
    for n in lens:
        starts.append(pos)
        pos += (n + 15) // 16 * 16 + 16
    dev = torch.zeros(pos + 16, dtype=torch.uint8, device="cuda:0")
    for i, n in enumerate(lens):
        if n:
            dev[starts[i]:starts[i] + n] = torch.from_numpy(host[offs[i]:offs[i] + n].copy()).to("cuda:0")
    ch = chunker(algo, sizes)
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    first = ch.chunk_batch_device([dev.data_ptr() + s for s in starts], lens, out.data_ptr(), cap)
    got = out.cpu().numpy().astype(np.uint64)
    for i, n in enumerate(lens):
        ref = oracle.cdc(algo, host[offs[i]:offs[i] + n], *sizes)
        assert_same(got[first[i]:first[i + 1]], ref, f"{algo} stream {i} len {n}")


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("walk,ahead", [("12,1", "0,64"), ("12,1", "2,3"), ("13,2", "16,1")])
def test_fixup_schedules_exact(algo, walk, ahead, monkeypatch):
    """Fix-up round schedules the defaults rarely reach: tiny segments with a
    1-avg warm-up make most entries wrong, then run-ahead from round 0
    (ahead 64), a short run-ahead limit (3 segments), and plain Jacobi that
    runs out of rounds into the serial pass.  Grouped rounds with device-side
    gating are in every case.  Env is read at handle creation."""
    import torch
    import chunkfs_amd as c
    from chunkfs_amd import _lib
    monkeypatch.setenv("CHUNKFS_AMD_WALK", walk)
    monkeypatch.setenv("CHUNKFS_AMD_AHEAD", ahead)
    sizes = SIZES[algo][0]
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(algo)
    ch = cls(c.SizeParams(*sizes)) if cls else c.SeqChunker(0, c.SizeParams(*sizes))
    n = (16 << 20) + 4321
    b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    _lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 17, None))
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    first = ch.chunk_batch_device([b.data_ptr()], [n], out.data_ptr(), cap)
    got = out[:first[1]].cpu().numpy().astype(np.uint64)
    assert_same(got, oracle.cdc(algo, b.cpu().numpy(), *sizes), f"{algo} walk={walk} ahead={ahead}")
    assert ch.last_timing()["fixup_iterations"] > 0  # the fix-up rounds did run
    data = make_input("periodic", 600000, 61)
    assert_same(ch.chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} periodic walk={walk} ahead={ahead}")
    ch.close()


def repeat_run_stream(n, seed):
    """Random bytes with long 8-byte-repeat regions at unaligned offsets: zero
    runs (one of them broken by single bytes), a constant byte, an 8-byte
    period -- where UltraCDC chains keep their phase (LEST chunks) and the
    walks take them many at a time (walk.hip ultra_run / serial_run)."""
    d = oracle.splitmix64_bytes(n, seed)
    rng = np.random.default_rng(seed)
    pos = 12345
    while pos < n - 64:
        ln = int(rng.integers(1, 6 << 20))
        kind = int(rng.integers(0, 4))
        e = min(n, pos + ln)
        if kind == 0:
            d[pos:e] = 0
        elif kind == 1:
            d[pos:e] = 0x41
        elif kind == 2:
            d[pos:e] = np.resize(np.arange(8, dtype=np.uint8) * 37 + 1, e - pos)
        else:
            d[pos:e] = 0
            d[pos:e:int(rng.integers(20000, 300000))] = 7
        pos = e + int(rng.integers(1000, 2 << 20))
    return d


QUIET_SIZES = [(4096, 8192, 16384), (512, 2048, 16384), (2048, 8192, 65536), (16384, 65536, 524288)]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("sizes", QUIET_SIZES)
def test_quiet_runs_exact(algo, sizes):
    """Every walk rule over long zero-filled / constant / 8-byte-periodic runs
    at unaligned offsets (quiet runs: walk.hip quiet_run) in a 3-stream device
    batch (40 MiB, 24 MiB of zeros, 7 MiB + 1): bit-exact vs the oracle."""
    import torch
    lens = [40 << 20, 24 << 20, (7 << 20) + 1]
    hosts = [repeat_run_stream(lens[0], 31), np.zeros(lens[1], dtype=np.uint8), repeat_run_stream(lens[2], 32)]
    devs = [torch.from_numpy(h).to("cuda:0") for h in hosts]
    ch = chunker(algo, sizes)
    cap = ch.batch_max_chunks(lens)
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    first = ch.chunk_batch_device([d.data_ptr() for d in devs], lens, out.data_ptr(), cap)
    got = out[:first[-1]].cpu().numpy().astype(np.uint64)
    for i, h in enumerate(hosts):
        assert_same(got[first[i]:first[i + 1]], oracle.cdc(algo, h, *sizes), f"{algo} {sizes} stream {i}")


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("walk,ahead", [("13,2", "16,1"), ("17,1", "0,64")])
def test_quiet_runs_serial_pass(algo, walk, ahead, monkeypatch):
    """The in-order pass over quiet runs (segment lists written per run,
    serial_run): schedules that leave most segments to it."""
    import chunkfs_amd as c
    monkeypatch.setenv("CHUNKFS_AMD_WALK", walk)
    monkeypatch.setenv("CHUNKFS_AMD_AHEAD", ahead)
    sizes = SIZES[algo][0]
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(algo)
    ch = cls(c.SizeParams(*sizes)) if cls else c.SeqChunker(0, c.SizeParams(*sizes))
    zr = oracle.splitmix64_bytes((16 << 20) + 77, 34)
    zr[123457:] = 0  # random, then zeros from an arbitrary phase
    for data in (zr, repeat_run_stream(24 << 20, 33)):
        assert_same(ch.chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} serial {walk} {ahead}")
    ch.close()


def test_quiet_summary_off_paths(monkeypatch):
    """Bitmap passes that write no quiet summary (CHUNKFS_AMD_BITS_FINE=0: the
    lane-per-range kernels) leave the quiet runs off: still exact."""
    import chunkfs_amd as c
    monkeypatch.setenv("CHUNKFS_AMD_BITS_FINE", "0")
    data = repeat_run_stream(12 << 20, 35)
    for algo in ("ultra", "leap", "seq"):
        sizes = SIZES[algo][0]
        cls = {"ultra": c.UltraChunker, "leap": c.LeapChunker}.get(algo)
        ch = cls(c.SizeParams(*sizes)) if cls else c.SeqChunker(0, c.SizeParams(*sizes))
        assert_same(ch.chunk_array(data), oracle.cdc(algo, data, *sizes), f"{algo} bits_fine=0")
        ch.close()
