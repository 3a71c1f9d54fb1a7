#!/usr/bin/env python3
"""Why the two-stream schedule's first steps are slow (diagnostics): 20 timed
async steps of the config-2 stream on a two-stream handle after (a) 5 warmup
steps, (b) 200 warmup steps of a ONE-stream handle + 5 of its own, (c) 200 of
its own.  Transfer from (b) means device state (clocks), not the handle's
streams / events.  Usage: pipe_warm.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402

n = 1 << 30
buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
c.check(c.lib().cdc_fill_splitmix64_device(c.ctypes.c_void_p(buf.data_ptr()), n, 1, None))
sizes = c.SizeParams(4096, 8192, 16384)


def handle(ovl):
    os.environ["CHUNKFS_AMD_OVERLAP"] = ovl
    try:
        return c.FastChunker(sizes)
    finally:
        del os.environ["CHUNKFS_AMD_OVERLAP"]


ptrs = np.array([buf.data_ptr()], dtype=np.uint64)
lens = np.array([n], dtype=np.uint64)


def steps(ch, k):
    cap = ch.batch_max_chunks([n])
    out = getattr(ch, "_o", None)
    if out is None:
        out = ch._o = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    ch.batch_sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        ch.chunk_batch_device_async(ptrs, lens, out.data_ptr(), cap)
    ch.batch_sync()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


for rep in range(2):
    if rep == 0 and os.environ.get("CHUNKFS_AMD_NO_PREWARM"):
        print("(no prewarm)")
    a = handle("2")
    steps(a, 5)
    print("rep", rep, "(a) 5 own warmup:      %.4f ms/step" % steps(a, 20), flush=True)
    one = handle("0")
    steps(one, 200)
    b = handle("2")
    steps(b, 5)
    print("rep", rep, "(b) 200 one-stream + 5: %.4f ms/step" % steps(b, 20), flush=True)
    cc = handle("2")
    steps(cc, 200)
    print("rep", rep, "(c) 200 own warmup:    %.4f ms/step" % steps(cc, 20), flush=True)
    print("rep", rep, "(c') same handle again: %.4f ms/step" % steps(cc, 20), flush=True)
    print("rep", rep, "(a') first handle again: %.4f ms/step" % steps(a, 20), flush=True)
    for h in (a, one, b, cc):
        h.close()
