#!/usr/bin/env python3
"""Per-step cost of reading the kernel events inside the timed loop
(diagnostics only): config 2 (1 GiB, FastCDC 4/8/16 KiB), K steps with
last_timing() after every step vs none."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd import _lib  # noqa: E402

n = 1 << 30
b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
_lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 1, None))
ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
cap = ch.batch_max_chunks([n])
out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
ptrs, lens = [b.data_ptr()], [n]
for _ in range(5):
    ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
torch.cuda.synchronize()
K = 50
for rep in range(3):
    for read in (True, False):
        t0 = time.perf_counter()
        for _ in range(K):
            ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
            if read:
                ch.last_timing()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / K
        print(f"rep {rep} read_events={read}: {el * 1e3:.4f} ms/step  {n / el / 2**30:.1f} GiB/s", flush=True)
