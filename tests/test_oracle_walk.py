"""CPU checks of the Rabin / UltraCDC / LeapCDC / SeqCDC oracle (no GPU).

The reference takes these algorithms from cdc-chunkers 0.1.3 (absent offline),
so their parity is UNPINNED: the oracle restates the published algorithms
(DESIGN.md), the C restatement is cross-checked by an independently written
Python twin, and the fixtures are labelled self-consistent.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from gen_golden import make_input

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "cdc_walk_selfconsistent.json")
ALGOS = ["rabin", "ultra", "leap", "seq"]


def _vectors():
    with open(GOLDEN) as f:
        return json.load(f)["vectors"]


@pytest.mark.parametrize("v", _vectors(), ids=lambda v: f"{v['algo']}-{v['pattern']}-{v['len']}")
def test_oracle_matches_walk_golden(v):
    data = make_input(v["pattern"], v["len"], v["seed"])
    assert hashlib.sha256(data.tobytes()).hexdigest() == v["input_sha256"]
    got = oracle.cdc(v["algo"], data, v["min"], v["avg"], v["max"])
    assert [int(x) for x in got[:, 1]] == v["lengths"]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("seed", [21, 22])
def test_c_oracle_equals_python_twin(algo, seed):
    sizes = {"rabin": (1024, 2048, 8192), "ultra": (1024, 4096, 8192),
             "leap": (512, 2048, 8192), "seq": (512, 1024, 4096)}[algo]
    data = oracle.splitmix64_bytes(120000 + seed, seed)
    a = oracle.cdc(algo, data, *sizes)
    b = oracle.py_cdc(algo, data, *sizes)
    assert a.shape == b.shape and (a == b).all()


def test_seq_modes_and_config_twin():
    data = oracle.splitmix64_bytes(90001, 5)
    for cfg in [(1, 5, 50, 256), (0, 3, 10, 64), (1, 7, 200, 1000)]:
        a = oracle.cdc("seq", data, 700, 1500, 6000, seqcfg=cfg)
        b = oracle.py_cdc("seq", data, 700, 1500, 6000, seqcfg=cfg)
        assert a.shape == b.shape and (a == b).all(), cfg


@pytest.mark.parametrize("algo", ALGOS)
def test_tiling_and_size_bounds(algo):
    mn, avg, mx = 2048, 4096, 16384
    for n in [0, 1, mn, mn + 1, 100003, 1 << 20]:
        data = oracle.splitmix64_bytes(n, n + 3)
        c = oracle.cdc(algo, data, mn, avg, mx)
        if n == 0:
            assert len(c) == 0
            continue
        assert c[0, 0] == 0 and int(c[:, 1].sum()) == n
        assert (c[1:, 0] == np.cumsum(c[:-1, 1])).all()
        assert (c[:, 1] <= mx).all() and (c[:-1, 1] >= mn).all()


@pytest.mark.parametrize("algo", ALGOS)
def test_write_path_segmentation_invariance(algo):
    """StorageWriter's 1 MiB carry-over loop (storage.rs:302-357) gives the
    whole-buffer chunks: every rule restarts at each boundary and looks only
    forward."""
    mn, avg, mx = 4096, 8192, 32768
    data = oracle.splitmix64_bytes((3 << 20) + 12345, 77)
    spans, _ = oracle.fs_write(algo, data, mn, avg, mx, seg_size=1 << 20)
    whole = oracle.cdc(algo, data, mn, avg, mx)
    assert [int(x) for x in spans] == [int(x) for x in whole[:, 1]]


def test_bad_sizes_rejected():
    L = oracle.lib()
    assert L.oracle_cdc_check(2, 0, 10, 20) != 0
    assert L.oracle_cdc_check(4, 4, 8, 16) != 0      # Ultra min >= 8
    assert L.oracle_cdc_check(5, 16, 64, 128) != 0   # Leap min >= 32
    assert L.oracle_cdc_check(6, 100, 50, 200) != 0  # min <= avg
    assert L.oracle_cdc_check(3, 100, 200, 400) != 0  # SuperCDC: not restated
    assert L.oracle_cdc_check(6, 1, 1, 1) == 0
