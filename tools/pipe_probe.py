#!/usr/bin/env python3
"""Timing probe: back-to-back FastCDC batches of one 1 GiB stream, synchronous
(cdc_chunk_batch_device) vs pipelined (cdc_chunk_batch_device_async + one
cdc_batch_sync), ms per step, checked against the oracle once.  Diagnostics only.
Usage: python3 tools/pipe_probe.py [steps] [stream_bytes]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunkfs_amd as cfa  # noqa: E402
from chunkfs_amd import _lib  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
ch = cfa.FastChunker(cfa.SizeParams(4096, 8192, 16384), device=0)
b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
_lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 1, None))
cap = ch.batch_max_chunks([n])
out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
ptrs, lens = np.array([b.data_ptr()], np.uint64), np.array([n], np.uint64)
for _ in range(3):
    first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(steps):
        first = ch.chunk_batch_device(ptrs, lens, out.data_ptr(), cap)
    torch.cuda.synchronize()
    ts = (time.perf_counter() - t0) / steps
    t0 = time.perf_counter()
    for _ in range(steps):
        fa = ch.chunk_batch_device_async(ptrs, lens, out.data_ptr(), cap)
    ch.batch_sync()
    torch.cuda.synchronize()
    ta = (time.perf_counter() - t0) / steps
    tims = [t for t in (ch.timing_back(k) for k in range(min(steps, 60))) if t["timed"]]  # (async: one in four)
    sc = sum(t["scan_ms"] for t in tims) / max(1, len(tims))
    print(f"sync {ts * 1e3:.4f} ms/step ({n / ts / 2**30:.0f} GiB/s)   async {ta * 1e3:.4f} ms/step "
          f"({n / ta / 2**30:.0f} GiB/s)   fused scan launch {sc:.4f} ms   chunks {int(fa[-1])}", flush=True)
import oracle  # noqa: E402
got = out[:int(fa[-1])].cpu().numpy().view(np.uint64)
ref = oracle.fastcdc(b.cpu().numpy(), 4096, 8192, 16384)
print("parity", bool(got.shape == ref.shape and (got == ref).all()), "first equal", bool((fa == first).all()))
