#!/usr/bin/env python3
"""Timing experiment for the resolve kernel (CHUNKFS_AMD_DIAG bits; see fastcdc.hip).

Usage: python3 tools/diag_resolve.py [DIAG] [stream_bytes]
Runs a few batches of one splitmix64 stream and prints the timing dict.  With
DIAG & 128 the engine prints the per-wave phase times of the resolve kernel
to stderr.  Not a product path; diagnostics only.
"""
import ctypes
import os
import sys

os.environ["CHUNKFS_AMD_DIAG"] = sys.argv[1] if len(sys.argv) > 1 else "128"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import chunkfs_amd as cfa  # noqa: E402
from chunkfs_amd import _lib  # noqa: E402

ch = cfa.FastChunker(cfa.SizeParams(4096, 8192, 16384), device=0)
b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
_lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 1, None))
cap = ch.batch_max_chunks([n])
out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
torch.cuda.synchronize()
for it in range(5):
    first = ch.chunk_batch_device([b.data_ptr()], [n], out.data_ptr(), cap)
    torch.cuda.synchronize()
    t = ch.last_timing()
    print(it, int(first[1]), {k: (round(v, 4) if isinstance(v, float) else v) for k, v in t.items()}, flush=True)
