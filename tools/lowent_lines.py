#!/usr/bin/env python3
"""The bench's low-entropy walk lines alone (bench.lowentropy_walk_lines: zeros,
a 61-byte period, random bytes with 1-32 MiB zero regions, random bytes with
small zero islands; Rabin / Ultra / Leap / Seq at 4/8/16 KiB), one JSON object
per input with GiB/s, re-walks, in-order pass and parity.  Diagnostics only.
usage: tools/lowent_lines.py [--no-parity]"""
import json
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

args = SimpleNamespace(min=4096, avg=8192, max=16384, no_parity="--no-parity" in sys.argv)
res = bench.lowentropy_walk_lines(args, SimpleNamespace(dev="cuda:0", local=0))
for k, v in res["lines"].items():
    print(f"{k:22s} {json.dumps(v)}", flush=True)
