"""CPU suite: the oracle itself, pinned where the reference allows.

* FastCDC: C oracle == independent pure-Python twin == committed fixtures
  (self-consistent; parity vs fastcdc 3.1.0 UNPINNED, see oracle/cdc_oracle.c).
* FSChunker + write-path segmentation: the reference's own known answers.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from gen_golden import make_input

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _vectors():
    with open(os.path.join(GOLDEN, "fastcdc_selfconsistent.json")) as f:
        return json.load(f)["vectors"]


@pytest.mark.parametrize("v", _vectors(), ids=lambda v: f"{v['pattern']}-{v['len']}-{v['min']}")
def test_oracle_matches_golden(v):
    data = make_input(v["pattern"], v["len"], v["seed"])
    assert hashlib.sha256(data.tobytes()).hexdigest() == v["input_sha256"]
    c = oracle.fastcdc(data, v["min"], v["avg"], v["max"])
    assert [int(x) for x in c[:, 1]] == v["lengths"]


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("sizes", [(4096, 8192, 16384), (8192, 16384, 65536), (256, 1024, 4096),
                                   (16384, 65536, 262144), (8192, 4096, 16384)])
def test_c_oracle_equals_python_twin(seed, sizes):
    n = 200_000 + seed * 777
    data = oracle.splitmix64_bytes(n, seed)
    a = oracle.fastcdc(data, *sizes)
    b = oracle.py_fastcdc(data, *sizes)
    assert a.shape == b.shape and (a == b).all()


def _check_tiling(c, n, mn, mx):
    if n == 0:
        assert len(c) == 0
        return
    assert c[0, 0] == 0
    assert (c[1:, 0] == c[:-1, 0] + c[:-1, 1]).all()
    assert int(c[-1, 0] + c[-1, 1]) == n
    assert (c[:, 1] > 0).all()
    assert (c[:, 1] <= mx).all()
    if len(c) > 1:
        assert (c[:-1, 1] >= mn).all()


@pytest.mark.parametrize("n", [0, 1, 63, 64, 4095, 4096, 4097, 8191, 8192, 16383, 16384, 16385, 32769, 100003])
def test_oracle_properties(n):
    data = oracle.splitmix64_bytes(n, 42)
    c = oracle.fastcdc(data, 4096, 8192, 16384)
    _check_tiling(c, n, 4096, 16384)


def test_oracle_rejects_bad_sizes():
    data = oracle.splitmix64_bytes(1000, 1)
    for sizes in [(32, 8192, 16384), (4096, 128, 16384), (4096, 8192, 512), (4096, 8192, 1 << 25)]:
        with pytest.raises(ValueError):
            oracle.fastcdc(data, *sizes)


@pytest.mark.parametrize("pattern,n,seed", [("splitmix64", 3 * (1 << 20) + 12345, 5),
                                            ("lowentropy", 2 * (1 << 20) + 7, 3),
                                            ("periodic", 2 * (1 << 20), 4096)])
def test_write_path_segmentation_invariance(pattern, n, seed):
    """FastCDC through the 1 MiB StorageWriter path == whole-stream chunking."""
    data = make_input(pattern, n, seed)
    whole = oracle.fastcdc(data, 4096, 8192, 16384)[:, 1]
    spans, _ = oracle.fs_write("fast", data, 4096, 8192, 16384)
    assert spans.tolist() == whole.tolist()


def _dedup_ratio(writes_spans):
    """ChunkStorage::cdc_dedup_ratio (storage.rs:203-205) with a HashMap keyed by content."""
    db = {}
    written = 0
    for data, spans in writes_spans:
        off = 0
        for ln in spans:
            chunk = data[off:off + int(ln)].tobytes()
            db.setdefault(hashlib.sha256(chunk).digest(), len(chunk))  # first insert wins (database.rs:76)
            off += int(ln)
        assert off == len(data)
        written += len(data)
    return written / sum(db.values()), sum(db.values())


def test_fixed_known_answers_from_reference():
    with open(os.path.join(GOLDEN, "reference_known_answers.json")) as f:
        cases = json.load(f)["cases"]
    for case in cases:
        cs = case["chunk_size"]
        hist = []
        ratios = []
        for pattern, n, seed in case["writes"]:
            data = make_input(pattern, n, seed)
            spans, _ = oracle.fs_write("fixed", data, cs)
            assert int(spans.sum()) == n
            hist.append((data, spans))
            ratios.append(_dedup_ratio(hist)[0])
        if "dedup_ratio_after_each" in case:
            assert ratios == pytest.approx(case["dedup_ratio_after_each"]), case["ref"]
        if "total_cdc_size" in case:
            assert _dedup_ratio(hist)[1] == case["total_cdc_size"], case["ref"]
        if "total_len" in case:
            assert sum(len(d) for d, _ in hist) == case["total_len"]


def test_fixed_oracle_matches_reference_loop():
    for n in [0, 1, 4095, 4096, 4097, 3 * (1 << 20) + 50]:
        c = oracle.fixed(n, 4096)
        exp = [(o, min(4096, n - o)) for o in range(0, n, 4096)]
        assert c.tolist() == [list(x) for x in exp]


def test_splitmix64_generator_definition():
    """word i = mix64(seed + (i+1)*golden), little-endian."""
    M = (1 << 64) - 1

    def mix(z):
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    seed = 1
    words = [mix((seed + (i + 1) * 0x9E3779B97F4A7C15) & M) for i in range(5)]
    exp = b"".join(w.to_bytes(8, "little") for w in words)[:37]
    assert oracle.splitmix64_bytes(37, seed).tobytes() == exp


def test_threaded_cpu_baseline_helper():
    """bench.py's multi-thread CPU baseline: workers chunk disjoint slices."""
    data = oracle.splitmix64_bytes(8 << 20, 3)
    nb, wall = oracle.time_fastcdc_threads(data, 4096, 8192, 16384, threads=4, seconds=0.2)
    assert nb >= data.size and nb % (data.size // 4) == 0 and wall > 0


def test_synthetic_generator_matches_oracle_and_device_fill_definition():
    """chunkfs_amd.synthetic (bench / config-3 data) = the oracle's splitmix64
    bytes = the definition of cdc_fill_splitmix64_device."""
    from chunkfs_amd import synthetic
    for n, seed in [(0, 1), (1, 1), (7, 3), (8, 3), (12345, 99), (1 << 16, 1000)]:
        assert np.array_equal(synthetic.splitmix64_bytes(n, seed), oracle.splitmix64_bytes(n, seed))
    vs = synthetic.versioned_archive(1 << 20, 3, seed=5)
    assert len(vs) == 3 and vs[0].size == 1 << 20
    assert all(abs(v.size - (1 << 20)) < (1 << 20) // 20 for v in vs)
    assert not np.array_equal(vs[1][:100000], vs[2][:100000]) or not np.array_equal(vs[0], vs[1])
