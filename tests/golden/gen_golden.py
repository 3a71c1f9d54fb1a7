#!/usr/bin/env python3
"""Generate tests/golden/*.json fixtures.

Two kinds of vectors live here:

* fastcdc_selfconsistent.json -- FastCDC v2020 cut lists over seeded inputs,
  produced by oracle/cdc_oracle.c AND the independent pure-Python twin
  (oracle/oracle.py:py_fastcdc); the script refuses to write unless both agree.
  LABEL: "self-consistent, unverified vs fastcdc 3.1.0" -- the reference ships
  no CDC golden vector and the crate (with its GEAR table) is absent offline
  (SURVEY.md §4, §8c).  Regenerate and diff once the crate's GEAR is installed.
* reference_known_answers.json -- the reference's OWN known answers for the
  fixed-size chunker and the write path, transcribed from its tests
  (tests/filesystem.rs:135-166, src/system/storage.rs:471-509,
  tests/filesystem.rs:32-94): these pin FSChunker + segmentation parity.

Inputs are regenerated from (pattern, seed, length); the sha256 of the input
bytes is stored so a generator change is caught.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402


def make_input(pattern, n, seed):
    if pattern == "splitmix64":
        return oracle.splitmix64_bytes(n, seed)
    if pattern == "const":
        return np.full(n, seed & 0xFF, dtype=np.uint8)
    if pattern == "periodic":  # period = seed bytes of splitmix64
        base = oracle.splitmix64_bytes(max(seed, 1), 7)
        return np.resize(base, n)
    if pattern == "lowentropy":  # 4 distinct byte values, runs of random length
        rnd = oracle.splitmix64_bytes(n, seed)
        vals = np.array([0, 1, 0x20, 0xFF], dtype=np.uint8)
        out = np.empty(n, dtype=np.uint8)
        i = 0
        r = 0
        while i < n:
            run = int(rnd[r % n]) + 1
            out[i:i + run] = vals[int(rnd[(r + 1) % n]) & 3]
            i += run
            r += 2
        return out
    raise ValueError(pattern)


CASES = [
    # (pattern, len, seed, min, avg, max)
    ("splitmix64", 0, 1, 4096, 8192, 16384),
    ("splitmix64", 1, 1, 4096, 8192, 16384),
    ("splitmix64", 4096, 1, 4096, 8192, 16384),
    ("splitmix64", 4097, 1, 4096, 8192, 16384),
    ("splitmix64", 16384, 2, 4096, 8192, 16384),
    ("splitmix64", 16385, 2, 4096, 8192, 16384),
    ("splitmix64", 65537, 3, 4096, 8192, 16384),
    ("splitmix64", 262144, 1, 4096, 8192, 16384),
    ("splitmix64", 1 << 20, 1, 4096, 8192, 16384),
    ("splitmix64", (1 << 20) + 333, 9, 8192, 16384, 65536),
    ("splitmix64", 1 << 20, 5, 2048, 8192, 65536),
    ("splitmix64", 1 << 20, 6, 512, 2048, 16384),
    ("splitmix64", 2 << 20, 7, 16384, 65536, 262144),
    ("splitmix64", 300001, 8, 64, 256, 1024),
    ("const", 200000, 0, 4096, 8192, 16384),
    ("const", 200000, 0xFF, 4096, 8192, 16384),
    ("periodic", 300000, 61, 4096, 8192, 16384),
    ("periodic", 300000, 4096, 4096, 8192, 16384),
    ("lowentropy", 400000, 11, 4096, 8192, 16384),
]


# Rabin / UltraCDC / LeapCDC / SeqCDC vectors (cdc_walk_selfconsistent.json):
# oracle/cdc_oracle.c cross-checked by oracle.py:py_cdc.  LABEL: "self-consistent,
# unverified vs cdc-chunkers 0.1.3" (the crate is absent offline).
WALK_CASES = [
    # (algo, pattern, len, seed, min, avg, max)
    ("rabin", "splitmix64", 0, 1, 2048, 4096, 8192),
    ("rabin", "splitmix64", 2047, 1, 2048, 4096, 8192),
    ("rabin", "splitmix64", 300001, 2, 2048, 4096, 8192),
    ("rabin", "splitmix64", 200000, 3, 64, 256, 1024),
    ("rabin", "const", 100000, 0, 512, 1024, 4096),
    ("rabin", "lowentropy", 200000, 4, 512, 2048, 8192),
    ("ultra", "splitmix64", 300000, 5, 4096, 8192, 16384),
    ("ultra", "splitmix64", 200003, 6, 1024, 2048, 8192),
    ("ultra", "const", 100000, 7, 1024, 2048, 8192),
    ("ultra", "periodic", 200000, 61, 2048, 4096, 16384),
    ("leap", "splitmix64", 300000, 8, 4096, 8192, 16384),
    ("leap", "splitmix64", 150001, 9, 256, 1024, 4096),
    ("leap", "lowentropy", 150000, 10, 512, 2048, 8192),
    ("seq", "splitmix64", 300000, 11, 4096, 8192, 16384),
    ("seq", "splitmix64", 100001, 12, 64, 256, 1024),
    ("seq", "const", 50000, 13, 1000, 2000, 5000),
    ("seq", "periodic", 200000, 4096, 2048, 4096, 16384),
]


def gen_walk():
    vecs = []
    for algo, pattern, n, seed, mn, avg, mx in WALK_CASES:
        data = make_input(pattern, n, seed)
        c = oracle.cdc(algo, data, mn, avg, mx)
        p = oracle.py_cdc(algo, data, mn, avg, mx)
        assert p.shape == c.shape and (p == c).all(), ("C and Python oracles disagree", algo, pattern, n)
        vecs.append({
            "algo": algo, "pattern": pattern, "len": n, "seed": seed, "min": mn, "avg": avg, "max": mx,
            "input_sha256": hashlib.sha256(data.tobytes()).hexdigest(),
            "lengths": [int(x) for x in c[:, 1]],
        })
    meta = {
        "label": "self-consistent, unverified vs cdc-chunkers 0.1.3 (crate absent offline)",
        "generator": "tests/golden/gen_golden.py via oracle/cdc_oracle.c, cross-checked by oracle.py:py_cdc",
        "vectors": vecs,
    }
    with open(os.path.join(HERE, "cdc_walk_selfconsistent.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"))
    return len(vecs)


def main():
    print("wrote", gen_walk(), "Rabin/Ultra/Leap/Seq vectors")
    vecs = []
    for pattern, n, seed, mn, avg, mx in CASES:
        data = make_input(pattern, n, seed)
        c = oracle.fastcdc(data, mn, avg, mx)
        if n <= (1 << 20) + 4096:
            p = oracle.py_fastcdc(data, mn, avg, mx)
            assert p.shape == c.shape and (p == c).all(), ("C and Python oracles disagree", pattern, n)
        vecs.append({
            "pattern": pattern, "len": n, "seed": seed, "min": mn, "avg": avg, "max": mx,
            "input_sha256": hashlib.sha256(data.tobytes()).hexdigest(),
            "lengths": [int(x) for x in c[:, 1]],
        })
    meta = {
        "label": "self-consistent, unverified vs fastcdc 3.1.0 (GEAR placeholder)",
        "generator": "tests/golden/gen_golden.py via oracle/cdc_oracle.c, cross-checked by oracle.py:py_fastcdc",
        "vectors": vecs,
    }
    with open(os.path.join(HERE, "fastcdc_selfconsistent.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"))

    known = {
        "label": "reference known answers (transcribed from the reference's own tests)",
        "cases": [
            {"ref": "tests/filesystem.rs:135-166 dedup_ratio_is_correct_for_fixed_size_chunker",
             "chunker": "fixed", "chunk_size": 4096,
             "writes": [["const", 1 << 20, 10], ["const", 1 << 20, 10], ["const", 1 << 20, 20]],
             "dedup_ratio_after_each": [256.0, 512.0, 384.0]},
            {"ref": "src/system/storage.rs:471-485 total_cdc_size_is_calculated_correctly_for_fixed_size_chunker_on_simple_data",
             "chunker": "fixed", "chunk_size": 4096,
             "writes": [["const", 1 << 20, 10]], "total_cdc_size": 4096},
            {"ref": "tests/filesystem.rs:32-65 write_read_blocks_test (sizes written)",
             "chunker": "fixed", "chunk_size": 4096,
             "writes": [["const", 1 << 20, 1], ["const", 1 << 20, 2], ["const", 1 << 20, 3], ["const", 50, 3]],
             "total_len": 3 * (1 << 20) + 50},
            {"ref": "tests/filesystem.rs:67-80 read_file_with_size_less_than_1mb",
             "chunker": "fixed", "chunk_size": 4096, "writes": [["const", 10, 1]], "total_len": 10},
            {"ref": "tests/filesystem.rs:82-94 write_read_big_file_at_once",
             "chunker": "fixed", "chunk_size": 4096, "writes": [["const", 3 * (1 << 20) + 50, 1]],
             "total_len": 3 * (1 << 20) + 50},
        ],
    }
    with open(os.path.join(HERE, "reference_known_answers.json"), "w") as f:
        json.dump(known, f, indent=1)
    print("wrote", len(vecs), "FastCDC vectors")


if __name__ == "__main__":
    main()
