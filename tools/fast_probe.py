#!/usr/bin/env python3
"""Config 2 (one 1 GiB splitmix64 stream, FastCDC 4/8/16 KiB) on the device:
ms per step, scan / resolve kernel times (HIP events), parity vs the oracle.
With CHUNKFS_AMD_DIAG=128 the resolve prints its per-wave phase times.
Diagnostics only.  Usage: fast_probe.py [steps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd import _lib  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << 30
b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
_lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 1, None))
ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
cap = ch.batch_max_chunks([n])
out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
ptrs, lens = [b.data_ptr()], [n]
for _ in range(3):
    first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    for _ in range(K):
        first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / K
    tims = [ch.timing_back(k) for k in range(min(K, 64))]
    sc = sum(t["scan_ms"] for t in tims) / len(tims)
    rs = sum(t["resolve_ms"] for t in tims) / len(tims)
    print(f"rep {rep}: {el * 1e3:.4f} ms/step {n / el / 2**30:.1f} GiB/s  scan {sc:.4f} ms  resolve {rs:.4f} ms  "
          f"rewalked {max(t['fixup_iterations'] for t in tims)}", flush=True)
if "--no-parity" not in sys.argv:
    import oracle
    got = out[:int(first[1])].cpu().numpy().view(np.uint64)
    ref = oracle.fastcdc(b.cpu().numpy(), 4096, 8192, 16384)
    print("parity", bool(got.shape == ref.shape and (got == ref).all()), got.shape[0], flush=True)
