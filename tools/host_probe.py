#!/usr/bin/env python3
"""Latency of cdc_chunk_data on small host buffers (the reference's 1 MiB
StorageWriter segments): wall time per call, its upload part, and the device
phases of the last call.  Diagnostics only.  Usage: host_probe.py [sizes...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import chunkfs_amd as c  # noqa: E402
from chunkfs_amd.synthetic import splitmix64_bytes  # noqa: E402

gap_us = 0.0  # --gap-us N: busy work between calls (StorageWriter hashes and indexes between its calls)
argv = sys.argv[1:]
if "--gap-us" in argv:
    i = argv.index("--gap-us")
    gap_us = float(argv[i + 1])
    del argv[i:i + 2]
sizes = [int(x) for x in argv] or [1 << 20, (1 << 20) + 12000, 4 << 20, 16 << 20]


def gap():
    if gap_us > 0:
        t = time.perf_counter() + gap_us * 1e-6
        while time.perf_counter() < t:
            pass

ch = c.FastChunker(c.SizeParams(4096, 8192, 16384))
data = splitmix64_bytes(max(sizes), 9)
for n in sizes:
    buf = data[:n]
    for _ in range(5):
        ch.chunk_array(buf)
    st0 = c.host_stats(ch)
    t0 = time.perf_counter()
    reps = 50
    for _ in range(reps):
        gap()
        ch.chunk_array(buf)
    el = (time.perf_counter() - t0) / reps - gap_us * 1e-6
    st1 = c.host_stats(ch)
    t = ch.last_timing()
    print(f"n={n:9d}  {el * 1e6:8.1f} us/call  {n / el / 2**30:6.2f} GiB/s  small "
          f"{st1['small_calls'] - st0['small_calls']}/{reps} (fallback {st1['small_fallbacks'] - st0['small_fallbacks']})  upload "
          f"{(st1['upload_s'] - st0['upload_s']) / reps * 1e6:6.1f} us  in C {(st1['total_s'] - st0['total_s']) / reps * 1e6:6.1f} us  scan {t['scan_ms'] * 1e3:6.1f} us  "
          f"resolve {t['resolve_ms'] * 1e3:6.1f} us  device {t['total_ms'] * 1e3:6.1f} us", flush=True)
