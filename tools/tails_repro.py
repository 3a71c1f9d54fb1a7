#!/usr/bin/env python3
"""Repeat the tail-length parity sweep of tests/test_gpu_parity.py
(test_tails_of_every_length, regular pipeline) R times in one process and
report every mismatch (diagnostics for a flaky result).  Usage:
tails_repro.py [R] [walk_coop_lib]"""
import os
import sys

os.environ["CHUNKFS_AMD_SMALL"] = "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import oracle  # noqa: E402
import chunkfs_amd as c  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sizes = (4096, 8192, 16384)
base = oracle.splitmix64_bytes(2 * 16384 + 64, 77)
lens = list(range(0, 200)) + list(range(4000, 4200)) + list(range(8100, 8300)) + \
    list(range(16300, 16500)) + list(range(2 * 16384 - 100, 2 * 16384 + 2))
refs = {n: oracle.fastcdc(base[:n], *sizes) for n in lens}
ch = c.FastChunker(c.SizeParams(*sizes))
bad = 0
for r in range(R):
    for n in lens:
        got = np.asarray(ch.chunk_array(base[:n]), dtype=np.uint64).reshape(-1, 2)
        ref = refs[n]
        if got.shape != ref.shape or not (got == ref).all():
            bad += 1
            if bad <= 10:
                print("rep", r, "n", n, "gpu", got.tolist()[-3:], "ref", ref.tolist()[-3:], flush=True)
    print("rep", r, "mismatches so far", bad, flush=True)
print("total calls", R * len(lens), "mismatches", bad)
