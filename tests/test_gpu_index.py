"""Device dedup index against the reference semantics.

Reference: the chunk Database is a HashMap written with
`entry(key).or_insert(value)` (src/system/database.rs:74-77 -- the first
insert of a digest wins), and cdc_dedup_ratio = size_written / total_cdc_size
(src/system/storage.rs:193-205).  The oracle here is a Python dict fed in
chunk order with hashlib digests; the known answers are the reference's own
(tests/filesystem.rs:135-166, tests/golden/reference_known_answers.json).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _write(ch, ix, data):
    """One write: GPU chunks + SHA-256 + index insert; returns (chunks, new flags)."""
    import torch
    chunks, dig = ch.chunk_and_hash(data)
    dd = torch.from_numpy(np.ascontiguousarray(dig)).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(chunks).view(np.int64)).cuda()
    new = torch.empty(len(chunks), dtype=torch.uint8, device="cuda")
    n_new = ix.insert_device(dd.data_ptr(), dc.data_ptr(), len(chunks), new.data_ptr())
    new = new.cpu().numpy().astype(bool)
    assert n_new == int(new.sum())
    return chunks, dig, new


def test_reference_known_answer_dedup_ratios():
    """tests/filesystem.rs:135-166: FSChunker(4096), three 1 MiB constant writes -> 256, 512, 384."""
    import chunkfs_amd as c
    case = json.load(open(os.path.join(HERE, "golden", "reference_known_answers.json")))["cases"][0]
    fs = c.FSChunker(case["chunk_size"])
    ix = c.DedupIndex(4096)
    ratios = []
    for _, n, val in case["writes"]:
        _write(fs, ix, np.full(n, val, dtype=np.uint8))
        ratios.append(ix.stats()["cdc_dedup_ratio"])
    assert ratios == pytest.approx(case["dedup_ratio_after_each"])
    ix.clear()
    assert ix.stats()["bytes_written"] == 0 and ix.stats()["unique_chunks"] == 0


def test_first_insert_wins_across_and_within_batches():
    """Versioned data (a base blob plus mutated copies, SURVEY.md config 3's
    offline substitute in miniature): per-chunk `new` flags equal a dict fed in
    chunk order, across several writes."""
    import chunkfs_amd as c
    rng = np.random.default_rng(3)
    base = oracle.splitmix64_bytes(2 << 20, 7)
    versions = [base]
    for k in range(3):
        v = versions[-1].copy()
        for _ in range(20):  # overwrite / insert / delete small runs
            p = int(rng.integers(0, v.size - 5000))
            op = k % 3
            if op == 0:
                v[p:p + 100] = rng.integers(0, 256, 100, dtype=np.uint8)
            elif op == 1:
                v = np.concatenate([v[:p], rng.integers(0, 256, 333, dtype=np.uint8), v[p:]])
            else:
                v = np.concatenate([v[:p], v[p + 777:]])
        versions.append(v)
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    ix = c.DedupIndex(1 << 16)
    db, written = {}, 0
    for v in versions:
        chunks, dig, new = _write(ch, ix, v)
        want = []
        for (o, l), d in zip(chunks, dig):
            k = bytes(d)
            assert k == hashlib.sha256(v[int(o):int(o) + int(l)].tobytes()).digest()
            want.append(k not in db)
            db.setdefault(k, int(l))
        written += v.size
        assert (new == np.array(want)).all()
    st = ix.stats()
    assert st["unique_chunks"] == len(db) and st["unique_bytes"] == sum(db.values())
    assert st["bytes_written"] == written
    assert st["cdc_dedup_ratio"] == pytest.approx(written / sum(db.values()))
    assert st["cdc_dedup_ratio"] > 1.5  # the copies share most chunks


def test_capacity_is_enforced_loudly():
    import chunkfs_amd as c
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    ix = c.DedupIndex(10)
    with pytest.raises(c.CdcError):
        _write(ch, ix, oracle.splitmix64_bytes(1 << 20, 1))
