#!/usr/bin/env python3
"""Per-step wall times of back-to-back async FastCDC batches (config-2 stream,
1 GiB): each call returns once batch k-3 is collected, so in steady state a
call's duration is the device's step period.  Prints the mean of every 10
calls for the two-stream default and for one stream (diagnostics).
Usage: pipe_steps.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402

n = 1 << 30
K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
c.check(c.lib().cdc_fill_splitmix64_device(c.ctypes.c_void_p(buf.data_ptr()), n, 1, None))
ptrs = np.array([buf.data_ptr()], dtype=np.uint64)
lens = np.array([n], dtype=np.uint64)
for ovl in ("2", "0", "2"):
    os.environ["CHUNKFS_AMD_OVERLAP"] = ovl
    ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    for _ in range(5):
        ch.chunk_batch_device_async(ptrs, lens, out.data_ptr(), cap)
    ch.batch_sync()
    torch.cuda.synchronize()
    ts = []
    t = time.perf_counter()
    for _ in range(K):
        ch.chunk_batch_device_async(ptrs, lens, out.data_ptr(), cap)
        t2 = time.perf_counter()
        ts.append(t2 - t)
        t = t2
    ch.batch_sync()
    ms = np.array(ts) * 1e3
    print("overlap", ovl, "per-10-call means (ms):", " ".join("%.3f" % ms[i:i + 10].mean() for i in range(0, K, 10)),
          flush=True)
    ch.close()
