#!/usr/bin/env python3
"""Would pipelined walk-engine batches overlap?  (diagnostics)  For each
segment-walk algorithm: K synchronous 1 GiB calls on one handle, then the same
K calls split over two handles driven from two host threads (ctypes releases
the GIL, each handle has its own stream), GiB/s both ways.
Usage: walk_concurrency.py [K]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = 1 << 30
buf = torch.empty(n, dtype=torch.uint8, device="cuda:0")
c.check(c.lib().cdc_fill_splitmix64_device(c.ctypes.c_void_p(buf.data_ptr()), n, 1, None))
sizes = c.SizeParams(4096, 8192, 16384)
mk = {"rabin": lambda: c.RabinChunker(sizes), "ultra": lambda: c.UltraChunker(sizes),
      "leap": lambda: c.LeapChunker(sizes), "seq": lambda: c.SeqChunker(c.OperationMode.Increasing, sizes)}
for name, f in mk.items():
    hs = [f(), f()]
    cap = hs[0].batch_max_chunks([n])
    outs = [torch.empty((cap, 2), dtype=torch.int64, device="cuda:0") for _ in hs]

    def run(i, k):
        for _ in range(k):
            hs[i].chunk_batch_device([buf.data_ptr()], [n], outs[i].data_ptr(), cap)

    for i in range(2):
        run(i, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(0, K)
    t1 = time.perf_counter() - t0
    ths = [threading.Thread(target=run, args=(i, K // 2)) for i in range(2)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    t2 = time.perf_counter() - t0
    print("%-6s one handle %.0f GiB/s (%.3f ms/call)   two handles, two threads %.0f GiB/s (%.3f ms/call)" %
          (name, K / t1, t1 / K * 1e3, K / t2, t2 / K * 1e3), flush=True)
    for h in hs:
        h.close()
