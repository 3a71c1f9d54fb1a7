#!/usr/bin/env python3
"""Phase stamps of the one-launch small-stream kernel (CHUNKFS_AMD_DIAG=4096):
a few cdc_chunk_data calls per size, each printing (stderr) the microseconds
from block 0's start to the last block's arrival, records, links, walk and
output.  Diagnostics only.  Usage: small_stamps.py [sizes...]"""
import os
import sys

os.environ["CHUNKFS_AMD_DIAG"] = "4096"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd.synthetic import splitmix64_bytes  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [1 << 20, (1 << 20) + 12000, 4 << 20]
ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
data = splitmix64_bytes(max(sizes), 9)
for n in sizes:
    for _ in range(4):
        ch.chunk_array(data[:n])
