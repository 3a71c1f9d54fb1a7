#!/usr/bin/env python3
"""Timing of the segment-walk engine (Rabin / Ultra / Leap / Seq) on one
device-resident splitmix64 stream.  CHUNKFS_AMD_WALK="seg_log2,warm_over_max"
overrides the segment size and warm-up (experiments).  Diagnostics only.

Usage: python3 tools/walk_bench.py [stream_bytes] [min avg max]   (WB_ALGOS=leap,seq selects)
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
sz = c.SizeParams(*(int(x) for x in sys.argv[2:5])) if len(sys.argv) > 4 else c.SizeParams(4096, 8192, 16384)
b = torch.empty(n, dtype=torch.uint8, device="cuda:0")
_lib.check(_lib.lib().cdc_fill_splitmix64_device(ctypes.c_void_p(b.data_ptr()), n, 1, None))
print("walk", os.environ.get("CHUNKFS_AMD_WALK", "default"), "bytes", n, sz, flush=True)
for name in os.environ.get("WB_ALGOS", "rabin,ultra,leap,seq").split(","):
    cls = {"rabin": c.RabinChunker, "ultra": c.UltraChunker, "leap": c.LeapChunker}.get(name)
    ch = cls(sz) if cls else c.SeqChunker(0, sz)
    cap = ch.batch_max_chunks([n])
    out = torch.empty((cap, 2), dtype=torch.int64, device="cuda:0")
    first = ch.chunk_batch_device([b.data_ptr()], [n], out.data_ptr(), cap)
    torch.cuda.synchronize()
    ts = time.perf_counter()  # settle: ~80 ms of load first (the clocks ramp over ~20 ms)
    while time.perf_counter() - ts < 0.08:
        ch.chunk_batch_device([b.data_ptr()], [n], out.data_ptr(), cap)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        first = ch.chunk_batch_device([b.data_ptr()], [n], out.data_ptr(), cap)
    el = (time.perf_counter() - t0) / 3
    t = ch.last_timing()
    print(f"{name:6s} {n / el / 2**30:8.1f} GiB/s  walk {t['scan_ms']:.3f} ms  rest {t['resolve_ms']:.3f} ms  "
          f"rewalked {t['fixup_iterations']}  serial {t['overflow_spans']}  chunks {int(first[1])}", flush=True)
    ch.close()
