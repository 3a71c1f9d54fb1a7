#!/usr/bin/env python3
"""Repeat the golden-vector parity check of tests/test_gpu_parity.py
(test_golden_vectors_on_gpu, default = small path) R times in one process and
report every mismatch (diagnostics for a flaky result).  Usage:
golden_repro.py [R] [small|pipeline]"""
import hashlib
import json
import os
import sys

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20
if len(sys.argv) > 2 and sys.argv[2] == "pipeline":
    os.environ["CHUNKFS_AMD_SMALL"] = "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import chunkfs_amd as c  # noqa: E402
from gen_golden import make_input  # noqa: E402

vecs = json.load(open(os.path.join(ROOT, "tests", "golden", "fastcdc_selfconsistent.json")))["vectors"]
chs = {}
bad = total = 0
for r in range(R):
    for v in vecs:
        key = (v["min"], v["avg"], v["max"])
        if key not in chs:
            chs[key] = c.FastChunker(c.SizeParams(*key))
        data = make_input(v["pattern"], v["len"], v["seed"])
        got = [int(x) for x in chs[key].chunk_array(data)[:, 1]]
        total += 1
        if got != v["lengths"]:
            bad += 1
            if bad <= 8:
                i = next((k for k in range(min(len(got), len(v["lengths"]))) if got[k] != v["lengths"][k]), None)
                print("rep", r, v["pattern"], v["len"], key, "chunks", len(got), "vs", len(v["lengths"]), "first diff", i,
                      flush=True)
print("calls", total, "mismatches", bad)
